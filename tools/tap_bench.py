"""GPU tool: HIP-event timing of the tap-major conv kernels (conv_tap.hip) per mode on FusAtNet's B=64
shapes.  usage: python tools/tap_bench.py [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402

SHAPES = [  # B, H, C, O, pad, ldx
    (64, 11, 256, 256, 1, 256),
    (64, 11, 2193, 256, 1, 2196),
    (64, 11, 256, 1024, 1, 256),
    (64, 11, 144, 256, 1, 144),
    (64, 11, 1024, 256, 0, 1024),
    (64, 5, 256, 256, 0, 256),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    L = lib()
    dev = "cuda"
    s = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(1 << 26, device=dev)
    only = os.environ.get("TAP_SHAPE")   # e.g. "0": run SHAPES[0] only
    shapes = [SHAPES[int(i)] for i in only.split(",")] if only else SHAPES
    for B, H, C, O, pad, ldx in shapes:
        OH = H + 2 * pad - 2
        x = torch.randn(B * H * H, ldx, device=dev)
        wt = torch.randn(O * 9 * C, device=dev)
        bias = torch.randn(O, device=dev)
        y = torch.empty(B * OH * OH, O, device=dev)
        dy = torch.randn(B * OH * OH, O, device=dev)
        dwt = torch.empty(O * 9 * C, device=dev)
        dx = torch.zeros(B * H * H, ldx, device=dev)
        flops = 2.0 * B * OH * OH * O * 9 * C
        runs = {
            "fwd": lambda: L.vc_conv3x3_tap_fwd(B, H, H, C, O, pad, x.data_ptr(), ldx, wt.data_ptr(), bias.data_ptr(),
                                                y.data_ptr(), O, ws.data_ptr(), ws.numel(), s),
            "wgrad": lambda: L.vc_conv3x3_tap_wgrad(B, H, H, C, O, pad, x.data_ptr(), ldx, dy.data_ptr(), O,
                                                    dwt.data_ptr(), ws.data_ptr(), ws.numel(), s),
            "dgrad": lambda: L.vc_conv3x3_tap_dgrad(B, H, H, C, O, pad, dy.data_ptr(), O, wt.data_ptr(), 1.0,
                                                    dx.data_ptr(), ldx, ws.data_ptr(), ws.numel(), s),
        }
        out = []
        for name, fn in runs.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            out.append(f"{name} {us:7.1f} us {flops / us / 1e6:6.1f} TF/s")
        print(f"B{B} H{H} C{C} O{O} pad{pad}: " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
