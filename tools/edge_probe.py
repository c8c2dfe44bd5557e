"""GPU probe: the cost of a cross-stream dependency inside a replayed hipGraph.

  serial : N dependent trivial kernels (vc_fill of 256 floats) on one stream
  pingpong: the same N kernels alternating between two streams, each waiting on the other's event
            (N - 1 cross-stream edges on the critical path)
  forks  : N kernels on stream 0; after each, stream 1 is forked off (waits on an event of stream 0)
           and runs one kernel; one join at the end (stream 0's chain carries no cross-stream wait)
  fork/k, forkjoin/k: a fork (and a join back into stream 0) after every k-th kernel
Prints us per kernel for each, captured once and replayed.  usage: python tools/edge_probe.py [N]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def replay_us(build, n, reps=50):
    s0 = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        build()   # eager once
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        build()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    L = lib()
    buf = torch.empty(4096, device="cuda")
    side = torch.cuda.Stream()
    evs = [torch.cuda.Event() for _ in range(2 * n + 4)]

    def serial():
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(n):
            L.vc_fill(256, buf.data_ptr(), 1.0, s)

    def pingpong():
        cur = torch.cuda.current_stream()
        streams = [cur, side]
        evs[0].record(cur)
        side.wait_event(evs[0])
        for i in range(n):
            st = streams[i & 1]
            if i > 0:
                st.wait_event(evs[i])
            L.vc_fill(256, buf.data_ptr() + 4 * 256 * (i & 1), 1.0, st.cuda_stream)
            evs[i + 1].record(st)
        cur.wait_event(evs[n])

    def forks():
        cur = torch.cuda.current_stream()
        for i in range(n):
            L.vc_fill(256, buf.data_ptr(), 1.0, cur.cuda_stream)
            evs[i].record(cur)
            side.wait_event(evs[i])
            L.vc_fill(256, buf.data_ptr() + 1024, 1.0, side.cuda_stream)
        evs[n].record(side)
        cur.wait_event(evs[n])

    def forks_every(k, join):
        def fn():
            cur = torch.cuda.current_stream()
            e = 0
            for i in range(n):
                L.vc_fill(256, buf.data_ptr(), 1.0, cur.cuda_stream)
                if i % k == k - 1:
                    evs[e].record(cur)
                    side.wait_event(evs[e])
                    e += 1
                    L.vc_fill(256, buf.data_ptr() + 1024, 1.0, side.cuda_stream)
                    if join:
                        evs[e].record(side)
                        cur.wait_event(evs[e])
                        e += 1
            evs[e].record(side)
            cur.wait_event(evs[e])
        return fn

    def long_branches(nm, ns):
        """main chain of nm kernels with two side chains of ns kernels forked at its start and joined
        at its end (the step's lane pattern)"""
        s2 = torch.cuda.Stream()

        def fn():
            cur = torch.cuda.current_stream()
            evs[0].record(cur)
            side.wait_event(evs[0])
            s2.wait_event(evs[0])
            for _ in range(ns):
                L.vc_fill(256, buf.data_ptr() + 1024, 1.0, side.cuda_stream)
                L.vc_fill(256, buf.data_ptr() + 2048, 1.0, s2.cuda_stream)
            for _ in range(nm):
                L.vc_fill(256, buf.data_ptr(), 1.0, cur.cuda_stream)
            evs[1].record(side)
            evs[2].record(s2)
            cur.wait_event(evs[1])
            cur.wait_event(evs[2])
        return fn

    def lane_graphs(nm, ns, reps=50):
        """the same DAG as long_branches, but each lane's chain is its own (linear) graph, launched on
        its own stream; the fork / join are events between the graph launches"""
        s0, s1, s2 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()

        def chain(off, k):
            def fn():
                st = torch.cuda.current_stream().cuda_stream
                for _ in range(k):
                    L.vc_fill(256, buf.data_ptr() + off, 1.0, st)
            return fn

        graphs = []
        for off, k, st in ((0, nm, s0), (1024, ns, s1), (2048, ns, s2)):
            g = torch.cuda.CUDAGraph()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                chain(off, k)()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                chain(off, k)()
            graphs.append(g)
        e_fork, e1, e2 = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()

        def step():
            e_fork.record(s0)
            s1.wait_event(e_fork)
            s2.wait_event(e_fork)
            with torch.cuda.stream(s1):
                graphs[1].replay()
            e1.record(s1)
            with torch.cuda.stream(s2):
                graphs[2].replay()
            e2.record(s2)
            with torch.cuda.stream(s0):
                graphs[0].replay()
            s0.wait_event(e1)
            s0.wait_event(e2)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e6

    print(f"lane graphs: main 40 + 2 side chains of 10 as three graphs on three streams: "
          f"{lane_graphs(40, 10):7.1f} us per step", flush=True)
    tot = replay_us(long_branches(40, 10), 40)
    print(f"branches: main chain of 40 with 2 open side chains of 10: {tot * 40:7.1f} us total "
          f"(serial 40: {40 * 1.61:.1f}, serial 60: {60 * 1.61:.1f})", flush=True)
    for name, fn in (("serial", serial), ("pingpong", pingpong), ("forks", forks),
                     ("fork/5", forks_every(5, False)), ("fork/25", forks_every(25, False)),
                     ("forkjoin/1", forks_every(1, True)), ("forkjoin/5", forks_every(5, True)),
                     ("forkjoin/25", forks_every(25, True))):
        print(f"{name:11s} {replay_us(fn, n):6.2f} us per kernel of the critical chain", flush=True)


if __name__ == "__main__":
    main()
