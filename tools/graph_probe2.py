"""GPU probe: which multi-stream capture pattern breaks hipGraph capture end?"""
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
import faulthandler
import os
import sys

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402


def capture(name, fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print(name, "eager ok", flush=True)
    with torch.cuda.graph(g, capture_error_mode=os.environ.get("CAPTURE_MODE", "global")):
        fn()
    g.replay()
    torch.cuda.synchronize()
    print(name, "graph ok", flush=True)


def main():
    which = sys.argv[1]
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    ev1, ev2 = torch.cuda.Event(), torch.cuda.Event()
    a = torch.ones(1000, device=dev)
    b = torch.empty(1000, device=dev)
    if which == "torch":
        def fn():
            ev1.record()
            side.wait_event(ev1)
            with torch.cuda.stream(side):
                b.copy_(a * 2)
            ev2.record(side)
            torch.cuda.current_stream().wait_event(ev2)
            a.add_(b)
        capture("torch fork/join", fn)
    elif which == "lib":
        from vitcnn_amd._lib import lib
        L = lib()

        def fn():
            ev1.record()
            side.wait_event(ev1)
            L.vc_fill(1000, b.data_ptr(), 3.0, side.cuda_stream)
            ev2.record(side)
            torch.cuda.current_stream().wait_event(ev2)
            a.add_(b)
        capture("lib fork/join", fn)
    elif which in ("fwd", "fwdbwd"):
        from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba
        m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
        crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
        hsi = torch.rand(64, 144, 9, 9, device=dev)
        lidar = torch.rand(64, 1, 9, 9, device=dev)
        tgt = torch.randint(1, 16, (64,), device=dev)

        def fn():
            if which == "fwd":
                with torch.no_grad():
                    m(hsi, lidar)
            else:
                crit(m(hsi, lidar), tgt).backward()
        capture(which, fn)


if __name__ == "__main__":
    main()
