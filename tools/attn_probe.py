"""GPU probe: the S2EFT attention core (vc_s2eft_attn_fwd / _bwd, config 5: B = 64, T = 146 tokens, 4 heads x
16) timed alone with HIP events (us per launch), and its outputs' checksum (to compare variants).
usage: [VITCNN_ATTN_BWD_WPB=w] python tools/attn_probe.py [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    B, T, H = 64, 146, 4
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * T, 3 * H * 16, device=dev, generator=g)
    dout = torch.randn(B * T, H * 16, device=dev, generator=g)
    out = torch.empty(B * T, H * 16, device=dev)
    lse = torch.empty(B * H * T, device=dev)
    dqkv = torch.zeros_like(qkv)
    L = lib()
    st = torch.cuda.current_stream().cuda_stream
    scale = 16 ** -0.5
    fwd = lambda: L.vc_s2eft_attn_fwd(B, T, H, qkv.data_ptr(), scale, out.data_ptr(), lse.data_ptr(), st)  # noqa: E731
    bwd = lambda: L.vc_s2eft_attn_bwd(B, T, H, qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),  # noqa: E731
                                      scale, dqkv.data_ptr(), st)
    for name, fn in (("attn_fwd", fwd), ("attn_bwd", bwd)):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / reps * 1e3:.2f} us", flush=True)
    print(f"checksum dqkv {float(dqkv.double().abs().sum()):.9e} {float(dqkv.double().sum()):.9e}")


if __name__ == "__main__":
    main()
