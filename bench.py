"""ViT-CNN training throughput on MI355X (BASELINE.json metric): patches/s, 9x9 HSI(144)+LiDAR, batch 64/GPU.

One step = forward + weighted CE + backward (+ RCCL gradient all-reduce when N > 1) + fused AdamW
over one resident synthetic batch (hsi U[0,1) [64,144,9,9], lidar U[0,1) [64,1,9,9], labels in
[1,15]; random-init weights of the reference architecture).  The whole step is ONE hipGraph at every
N: for N > 1 the gradient leaves the backward in three head-first buckets whose RCCL all-reduces run
on a side stream while the backward continues (parallel.GradExchange), and AdamW waits for the last.

  python bench.py [--gpus N --steps K --warmup W] [--precision fp32|bf16]   (torch.distributed.run for N > 1)

`--precision` picks the headline step's GEMM operand precision (fp32 = the parity mode, default;
bf16 = BASELINE config 2: bf16 operands, fp32 accumulation, fp32 master weights / scan state /
norm statistics).  At N = 1 the line also carries the other precision's step (`config2_bf16`), the
whole-image inference leg (`f1_test`), and the config-4/5 legs.

Prints ONE JSON line on rank 0 (contract in the task statement) with `roofline` for the dominant
kernel (HIP-event timed inside this process) and `cpu_baseline` (the CPU oracle, rank 0, N=1).
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "vit-cnn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GFLOP_PER_PATCH = 0.5235      # SURVEY.md section 8d (de-duplicated algebra, fwd+bwd)
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_*_f32 dense peak
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-s2eft", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU-baseline steps (median reported)")
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--force-exchange", action="store_true",
                    help="run the bucketed RCCL exchange even at N = 1 (world-1 process group)")
    ap.add_argument("--no-f1", action="store_true")
    ap.add_argument("--no-train-loop", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--roofline-only", action="store_true",
                    help="build the step, then only the roofline legs (for a rocprofv3 --stats run whose "
                         "per-kernel average is the roofline leg's launch alone)")
    return ap.parse_args()


def synthetic(batch, seed, device):
    g = torch.Generator().manual_seed(seed)
    hsi = torch.rand(batch, 144, 9, 9, generator=g)
    lidar = torch.rand(batch, 1, 9, 9, generator=g)
    target = torch.randint(1, 16, (batch,), generator=g)
    return hsi.to(device), lidar.to(device), target.to(device)


def time_kernel(fn, reps, stream):
    """Average device time of fn() (one kernel launch sequence) with HIP events on `stream`."""
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(reps):
        fn()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


PMC_PROFILES = ("r06_pmc.json", "r05_pmc.json", "r03_pmc.json", "r02_pmc_s4.json", "r02_pmc.json", "r01_pmc.json")   # newest first


def _pmc_from_profile(kernel_key):
    """Per-launch PMC record of `kernel_key` from the newest committed profile that has it
    (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ passes, separate runs: tools/pmc_step.sh ->
    tools/pmc_summary_json.py -> profiles/r05_pmc.json; tools/pmc_to_json.py before it), or None."""
    for name in PMC_PROFILES:
        path = os.path.join(REPO, "profiles", name)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            prof = json.load(f)
        kernels = prof.get("kernels", {})
        # "scan_bwd<9>" also names the instantiations with further template arguments ("scan_bwd<9, true>")
        hits = [v for n, v in kernels.items() if n == kernel_key or n.startswith(kernel_key[:-1] + ",")]
        if hits:
            return dict(hits[0], profile="profiles/" + name)
    return None


def _traffic_from_profile(kernel_key):
    """HBM bytes per launch of `kernel_key` (2 x FETCH_SIZE + WRITE_SIZE, the round-1 correction) from
    the committed PMC profile, or None when no profile of this kernel is committed."""
    k = _pmc_from_profile(kernel_key)
    return None if k is None else k.get("hbm_bytes_per_launch")


_SCENE = {}


def synthetic_scene(seed, labelled_frac=1.0):
    """A Houston2013-size synthetic scene (349 x 1905 pixels, 144 HSI + 1 LiDAR bands, U[0,1) like the
    reference's per-band min-max normalisation, datasets.py:125-133) and a ground-truth map with
    classes 1..15 on `labelled_frac` of the pixels (0 = unlabelled elsewhere); generated once per seed."""
    key = (seed, labelled_frac)
    if key not in _SCENE:
        rng = np.random.default_rng(seed)
        W, H = 349, 1905
        img1 = rng.random((W, H, 144), dtype=np.float32)
        img2 = rng.random((W, H, 1), dtype=np.float32)
        gt = rng.integers(1, 16, size=(W, H))
        if labelled_frac < 1.0:
            gt[rng.random((W, H)) >= labelled_frac] = 0
        _SCENE[key] = (img1, img2, gt)
    return _SCENE[key]


def batch_assembly_ms(step, hsi, lidar, target, dev, steps, seed):
    """ms per training step when every batch is assembled on the device (vitcnn_amd.window.PatchBatcher:
    vc_patch_gather of B windows + flip / rot90 codes, datasets.py:511-593) from a synthetic
    HBM-resident 349 x 1905 cube with a uniform ground-truth map, then copied into the captured
    step's input buffers."""
    from vitcnn_amd.window import PatchBatcher
    img1, img2, gt = synthetic_scene(seed)
    batcher = PatchBatcher(img1, img2, gt, hsi.shape[-1], ignored_labels=(0,), batch_size=hsi.shape[0],
                           flip_augmentation=True, device=dev, seed=seed)
    it = iter(batcher)

    def asm_step():
        x1, x2, y = next(it)
        hsi.copy_(x1)
        lidar.copy_(x2)
        target.copy_(y)
        step()

    for _ in range(3):
        asm_step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        asm_step()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def train_loop_leg(dev, epochs, seed, headline_ms):
    """the rate the reference's main.py sees through the plugin surface --
    `vitcnn_amd.model_utils.train` (model_utils.py:854-1045) with the model, AdamW, weighted CE and
    StepLR of `get_model("Multimodality_Mamba")`, over a `PatchBatcher` loader (MultiModalX batches of
    64 gathered on the device from the HBM-resident synthetic scene, 2 % of its pixels labelled:
    ~13.3k patches = 208 batches per epoch, the last one short), `epochs` epochs, display every 100
    iterations, best / final checkpoints written (into a temporary directory).  Reported: the whole
    call (first batch of each shape eager, graph captures, checkpoints) and the steady state (epochs
    after the first), against the headline step."""
    import shutil
    import tempfile
    from vitcnn_amd import model_utils as mu
    from vitcnn_amd.window import PatchBatcher
    img1, img2, gt = synthetic_scene(seed, labelled_frac=0.02)
    torch.manual_seed(0)
    net, opt, crit, kw = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                      dataset="synthetic", device=dev)
    loader = PatchBatcher(img1, img2, gt, 9, ignored_labels=(0,), batch_size=kw["batch_size"],
                          flip_augmentation=kw["flip_augmentation"], device=dev, seed=seed)
    cwd = os.getcwd()
    tmp = tempfile.mkdtemp(prefix="vitcnn_train_leg_")
    try:
        os.chdir(tmp)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        mu.train("bench", 0, None, net, opt, crit, loader, epochs, scheduler=kw["scheduler"], display_iter=100,
                 device=dev)
        torch.cuda.synchronize(dev)
        total = time.perf_counter() - t0
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp, ignore_errors=True)
    st = mu.train.last_stats
    ep = st["epochs"]
    patches = sum(e["patches"] for e in ep)
    steady = ep[1:] if len(ep) > 1 else ep
    sp, ss = sum(e["patches"] for e in steady), sum(e["seconds"] for e in steady)
    steady_v = sp / ss
    ms_step = ss / sum(e["batches"] for e in steady) * 1e3
    return {"workload": "model_utils.train(): get_model('Multimodality_Mamba') defaults (AdamW 8e-4, weighted CE, "
                        "StepLR), PatchBatcher loader over the synthetic 349x1905 scene (2 % labelled), B=64, "
                        f"{epochs} epochs, display every 100 iterations, checkpoints written",
            "launch": st["launch"], "value": round(steady_v, 1), "unit": "patches/s",
            "ms_per_batch_steady": round(ms_step, 4), "steady_epochs": len(steady),
            "value_whole_call": round(patches / total, 1), "seconds_whole_call": round(total, 3),
            "batches_per_epoch": ep[0]["batches"], "patches_per_epoch": ep[0]["patches"],
            "vs_headline_step": round(headline_ms / ms_step, 4),
            "final_loss": round(float(st["losses"][-1]), 6)}


def dominant_kernel_roofline(model, batch, reps):
    """Re-launch the step's dominant kernel on its live workspace buffers and time it with HIP events
    on the stream it is launched on.

    Dominant kernel (profiles/r03_*): the hsiMamba selective-scan backward of block hsi1 with its fused
    tail (`scan_bwd<9, true, true>`, vc_mamba_scan_bwd_fused: grid 640 sequences x 5 channel chunks), the
    longest single launch of the step.  A sequential recurrence over 81 tokens, then the sequence's
    dt_proj / x_proj data gradients (MFMA) and conv1d + SiLU backward; its roofline is HBM.  Algorithmic
    bytes per launch = compulsory reads of u, x_proj rows, yp (each [10*B*L, *]), d(yp) [B*L, D], the x
    half of xz [B*L, D] (gathered, counted once) and the forward's 4-token state checkpoints
    [10*B][ceil(L/4)][16][D] + writes of d(dt_lin), the full dxdbl rows, dpre and the per-sequence
    parameter partials (A_log / D / gate, conv1d).  The parameter-gradient outputs
    are passed as NULL, so the timed launch is the kernel alone (the same kernel rocprofv3 reports in
    profiles/)."""
    from vitcnn_amd._lib import lib
    from vitcnn_amd.model import NDIR, _Program
    dev = model.flat_params.device
    prog = _Program(model, dev, batch, True, "grad")
    L = lib()
    blk, pfx, H = model.hsi1, "hsi1", model.patch
    E = blk.embed
    D, R, Lt = E // 2, -(-E // 16), H * H
    XW = R + 32
    rows, nr, nseq = batch * Lt, NDIR * batch * Lt, NDIR * batch
    f = prog.ws.f
    mx, gv = pfx + ".global_view.layers.0", pfx + ".global_view"
    P = prog.P
    order = prog.tab[("order", H)].data_ptr()
    ckpt = L.vc_mamba_scan_ckpt_floats(batch, Lt, D, NDIR)
    stream = torch.cuda.current_stream(dev)

    def fn():
        L.vc_mamba_scan_bwd_fused(batch, Lt, D, R, NDIR, f(pfx + ".U", nr * D), f(pfx + ".XD", nr * XW), order,
                                  f(pfx + ".XZ", rows * 2 * D), P[mx + ".conv1d.weight"], P[mx + ".conv1d.bias"],
                                  P[mx + ".x_proj.weight"], P[mx + ".dt_proj.weight"], P[mx + ".dt_proj.bias"],
                                  P[mx + ".A_log"], P[mx + ".D"], P[gv + ".weights"], f(pfx + ".Y", nr * D),
                                  f(pfx + ".dYP", rows * D), f(pfx + ".CKP", ckpt), f(pfx + ".dU", nr * D),
                                  f(pfx + ".dDTL", nr * D), f(pfx + ".dXD", nr * XW),
                                  f(pfx + ".convpart", nseq * 5 * D), None, None, None, prog.scr_p, prog.scr_n,
                                  stream.cuda_stream)

    t = time_kernel(fn, reps, stream)
    reads = nr * D + nr * XW + nr * D + rows * D + rows * D + ckpt
    writes = nr * D + nr * XW + nr * D + nseq * 5 * D + nseq * (D * 16 + D + 1)
    algo = 4.0 * (reads + writes)
    achieved = algo / t / 1e9
    key = "scan_bwd<9, true, true>"
    traffic = _traffic_from_profile(key)
    # the same launch against its two other bounds: compulsory HBM bytes only (the 4-token state
    # checkpoints the forward writes for it excluded), and VALU issue (the committed PMC profile's
    # SQ_INSTS_VALU per launch x 4 cycles / 1024 SIMDs at 2.4 GHz = the time the instructions need
    # with every SIMD issuing every cycle)
    compulsory = algo - 4.0 * ckpt
    pmc = _pmc_from_profile(key) or {}
    valu_us = pmc.get("valu_issue_bound_us")
    return {"kernel": key + " (hsi1 selective-scan backward + fused dt_proj / x_proj / conv1d data-gradient tail, "
                            "640 seq x 81 tokens x 72 ch x 16 states)",
            "bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic, "avg_launch_us": round(t * 1e6, 2),
            "algorithmic_bytes_per_launch": algo,
            "compulsory": {"bytes_per_launch": compulsory, "achieved": round(compulsory / t / 1e9, 2),
                           "frac": round(compulsory / t / 1e9 / PEAK_HBM_GBS, 5)},
            "valu_issue": None if valu_us is None else {
                "insts_per_launch": pmc.get("SQ_INSTS_VALU"), "bound_us": round(valu_us, 2),
                "frac": round(valu_us / (t * 1e6), 4), "profile": pmc.get("profile")}}


def gemm_roofline(model, batch, reps):
    """The largest GEMM of the step (hsi1.local_feature im2col'ed 3x3 conv, M = B*49, N = 256,
    K = 9*144; the automatic choice, round 4: the LDS-DMA pipelined kernel) timed the same way;
    MFMA-bound (fp32 peak).  Reported beside the dominant kernel."""
    from vitcnn_amd._lib import lib
    from vitcnn_amd.model import _Program
    dev = model.flat_params.device
    prog = _Program(model, dev, batch, True, "grad")
    L = lib()
    M, N, K = batch * 49, 256, 9 * 144
    col = prog.ws.f("hsi1.local_feature.col", M * K)
    out = prog.ws.f("hsi1.local_feature.out", M * N)
    W, b = prog.P["hsi1.local_feature.conv.weight"], prog.P["hsi1.local_feature.conv.bias"]
    stream = torch.cuda.current_stream(dev)

    def fn():
        L.vc_gemm(0, 1, M, N, K, 1.0, col, K, 0, W, K, 0, 0.0, out, N, 0, 1, b, None, 0, 0, 1, None, prog.scr_p,
                  prog.scr_n, stream.cuda_stream)

    t = time_kernel(fn, reps, stream)
    flops = 2.0 * M * N * K
    achieved = flops / t / 1e12
    return {"kernel": "gp::gemm_pipe<64,64> fp32, LDS-DMA pipelined (hsi1.local_feature conv3x3, M=%d N=%d K=%d)"
            % (M, N, K),
            "bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4), "avg_launch_us": round(t * 1e6, 2),
            "flop_per_launch": flops}


def log(msg):
    """progress on stderr (the one JSON line goes to stdout)"""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _cgroup_cpus():
    """the CPU quota of this process's cgroup (cgroup v2 cpu.max), or None when unlimited / absent"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, int(q) // int(per))
    except (OSError, ValueError):
        return None


def host_info():
    """The GPU box's host CPU as the SURVEY.md section 8(d) protocol asks: nproc, the cores this
    process may run on (affinity mask and cgroup quota: the box's CPU share), and the lscpu model name."""
    import subprocess
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    if model is None and os.path.exists("/proc/cpuinfo"):
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpus": _cgroup_cpus(), "model": model}


def cpu_threads():
    """torch CPU threads for the baselines: every core this process may use -- os.cpu_count() on an
    unrestricted host; on the GPU box the affinity mask / cgroup quota is the box's CPU share, and
    threads beyond it would only time-slice."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    q = _cgroup_cpus()
    return min(n, q) if q else n


def timed_median(fn, warmup, steps):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def cpu_baseline(warmup, steps):
    """The CPU oracle (reference op order, naive sequential scan; oracle/vitcnn_oracle.py) timed on
    this host by the SURVEY.md section 8(d) protocol: all available cores, `warmup` untimed then the
    median of `steps` timed B=64 training steps (forward, CE, backward, AdamW, loss.item())."""
    from oracle import vitcnn_oracle as O
    from vitcnn_amd import Multimodality_Mamba
    threads = cpu_threads()
    torch.set_num_threads(threads)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    state = O.make_state(m.state_dict())
    opt = O.make_adamw(state)
    hsi, lidar, target = synthetic(64, 1234, "cpu")
    w = O.ce_class_weights(16)
    med, ts = timed_median(lambda: O.train_step(state, hsi, lidar, target, w, opt), warmup, steps)
    return {"value": round(64 / med, 3), "unit": "patches/s", "cores": threads, "kind": "port",
            "host": host_info(),
            "sample": f"median of {steps} timed B=64 training steps after {warmup} warm-up steps of "
                      f"oracle/vitcnn_oracle.py (fp32, torch CPU, {threads} threads); s/step: "
                      + ", ".join(f"{t:.2f}" for t in ts)}


S2EFT_GFLOP_PER_STEP = 13.6  # S2EFT fwd + bwd GEMM work per B = 64 step


def s2eft_leg(dev, steps, cpu_steps):
    """Config 5: S2EFT train step (forward, weighted CE, backward, Adam)
    at B = 64 on [64, 145, 147] synthetic tokens, eager launches; plus the CPU oracle on the same
    shape (oracle/s2eft_oracle.py, autograd, torch CPU threads) as its baseline."""
    from vitcnn_amd import CrossEntropyLoss
    from vitcnn_amd.optim import AdamW
    from vitcnn_amd.s2eft import ViT
    torch.manual_seed(0)
    kw = dict(image_size=7, near_band=3, num_patches=144, num_classes=16, dim=64, depth=5, heads=4, mlp_dim=8,
              dropout=0.0, emb_dropout=0.0, mode="CAF")
    m = ViT(**kw).to(dev).train()
    opt = AdamW(m.parameters(), lr=5e-4, weight_decay=0.0)
    w = torch.ones(16)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w.to(dev))
    g = torch.Generator().manual_seed(7)
    x = torch.rand(64, 145, 147, generator=g)
    t = torch.randint(1, 16, (64,), generator=g)
    xd, td = x.to(dev), t.to(dev)

    def eager_step():
        opt.zero_grad(set_to_none=True)
        crit(m(xd), td).backward()
        opt.step()

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(5):
            eager_step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    # the whole step (forward, CE, hand-written backward, fused Adam) as one hipGraph
    launch = "hipGraph"
    try:
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(graph):
            crit(m(xd), td).backward()
            opt.step()
        step = graph.replay
    except RuntimeError as e:  # reported in the line, never silent
        launch = f"eager (graph capture failed: {str(e)[:80]})"
        step = eager_step
    warm(step, dev, WARM_S)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    tf = S2EFT_GFLOP_PER_STEP / ms   # GF / ms = TF/s
    out = {"workload": "S2EFT (CAF, depth 5, 4 heads x 16, dim 64) train step, x [64,145,147], 16 classes",
           "value": round(64 / ms * 1e3, 1), "unit": "patches/s", "ms_per_step": round(ms, 4), "dtype": "fp32",
           "launch": launch,
           # the step's algorithmic work (13.6 GF fwd + bwd per B = 64 step, FlopCounter)
           # against the dense fp32 MFMA peak; the whole step's time, so launch gaps and the non-GEMM kernels count
           "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / PEAK_FP32_MFMA_TFLOPS, 4), "traffic": None,
                        "work": f"{S2EFT_GFLOP_PER_STEP} GFLOP per B=64 step / the step time"}}
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}

    def cpu_leg():   # run after every GPU leg
        from oracle import s2eft_oracle as O
        threads = cpu_threads()
        torch.set_num_threads(threads)
        O.train_step(sd, x, t, w)
        t0 = time.perf_counter()
        for _ in range(cpu_steps):
            O.train_step(sd, x, t, w)
        dt = (time.perf_counter() - t0) / cpu_steps
        out["cpu_baseline"] = {"value": round(64 / dt, 2), "unit": "patches/s", "cores": threads, "kind": "port",
                               "sample": f"{cpu_steps} B=64 fwd+bwd steps of oracle/s2eft_oracle.py"}
    return out, (cpu_leg if cpu_steps > 0 else None)


def muufl_leg(dev, steps):
    """Config 4 (SURVEY.md section 8 row A-MUUFL): the ViT-CNN train step on the MUUFL shape
    (64 + 2 bands, 11x11 patches, 12 classes) at B = 64 per GPU, whole step as one hipGraph."""
    from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step
    torch.manual_seed(0)
    m = Multimodality_Mamba(11, 1, 1, 64, 2, 32, 12, "multi_clock_gate").to(dev).train()
    opt = AdamW(m.parameters(), lr=8e-4)
    w = torch.ones(12)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w.to(dev))
    g = torch.Generator().manual_seed(4)
    hsi = torch.rand(64, 64, 11, 11, generator=g).to(dev)
    lidar = torch.rand(64, 2, 11, 11, generator=g).to(dev)
    tgt = torch.randint(1, 12, (64,), generator=g).to(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            fused_train_step(m, crit, hsi, lidar, tgt)
            opt.step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    opt.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fused_train_step(m, crit, hsi, lidar, tgt)
        opt.step()
    warm(graph.replay, dev, WARM_S)
    t0 = time.perf_counter()
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"workload": "ViT-CNN train step, MUUFL shape 64+2 bands, 11x11, 12 classes", "value": round(64 / ms * 1e3, 1),
            "unit": "patches/s", "ms_per_step": round(ms, 4), "dtype": "fp32", "launch": "hipGraph"}


FUSAT_GFLOP_PER_PATCH = 6.92  # SURVEY.md section 8(d), FusAtNet forward


def fusat_leg(dev, steps, cpu):
    """Config 5: the FusAtNet TRAINING step at B = 64 on [64,144,11,11] +
    [64,1,11,11] (train-mode forward with batch-statistics BN and running-stat updates, weighted CE,
    hand-written backward with out-of-place residual semantics -- the reference's own backward raises --,
    and the reference's Adam(lr 1e-3, model_utils.py:109-118) as the fused kernel over the flat parameter
    buffer), captured as one hipGraph when the capture succeeds; the train-mode forward alone beside it.
    CPU baseline: the oracle's B = 4 training step (forward + autograd backward, oracle/fusat_oracle.py)."""
    from vitcnn_amd import CrossEntropyLoss
    from vitcnn_amd.fusatnet import FusAtNet
    from vitcnn_amd.optim import AdamW
    torch.manual_seed(0)
    m = FusAtNet(144, 1, 16).to(dev).train()
    g = torch.Generator().manual_seed(3)
    x1, x2 = torch.rand(64, 144, 11, 11, generator=g), torch.rand(64, 1, 11, 11, generator=g)
    a, b = x1.to(dev), x2.to(dev)
    tgt = torch.randint(1, 16, (64,), generator=g).to(dev)
    with torch.no_grad():
        for _ in range(2):
            m(a, b)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            m(a, b)
        torch.cuda.synchronize(dev)
        ms_fwd = (time.perf_counter() - t0) / steps * 1e3
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=0.0)
    w = torch.ones(16, device=dev)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w)

    def eager_step():
        opt.zero_grad(set_to_none=True)
        crit(m(a, b), tgt).backward()
        opt.step()

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            eager_step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    launch = "hipGraph"
    try:
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(graph):
            crit(m(a, b), tgt).backward()
            opt.step()
        step = graph.replay
    except RuntimeError as e:  # reported in the line, never silent
        launch = f"eager (graph capture failed: {str(e)[:80]})"
        torch.cuda.synchronize(dev)
        step = eager_step
    warm(step, dev, WARM_S)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    tf = 64 / ms * 1e3 * 3 * FUSAT_GFLOP_PER_PATCH * 1e-3
    tf_fwd = 64 / ms_fwd * 1e3 * FUSAT_GFLOP_PER_PATCH * 1e-3
    out = {"workload": "FusAtNet train step (fwd + CE + bwd + fused Adam), [64,144,11,11] + [64,1,11,11], 16 classes",
           "value": round(64 / ms * 1e3, 1), "unit": "patches/s", "ms_per_step": round(ms, 3), "dtype": "fp32",
           "launch": launch, "achieved_tflops": round(tf, 2), "mfma_frac": round(tf / PEAK_FP32_MFMA_TFLOPS, 4),
           "forward": {"value": round(64 / ms_fwd * 1e3, 1), "unit": "patches/s (train-mode forward)",
                       "ms_per_batch": round(ms_fwd, 3), "achieved_tflops": round(tf_fwd, 2),
                       "mfma_frac": round(tf_fwd / PEAK_FP32_MFMA_TFLOPS, 4)}}
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    tc, wc = tgt[:4].cpu(), w.cpu()

    def cpu_leg():   # run after every GPU leg
        from oracle import fusat_oracle as O
        threads = cpu_threads()
        torch.set_num_threads(threads)
        params = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}

        def cpu_step():
            for v in params.values():
                v.grad = None
            torch.nn.functional.cross_entropy(O.forward(params, x1[:4], x2[:4], train=True), tc, weight=wc).backward()

        med, _ = timed_median(cpu_step, 1, 3)
        out["cpu_baseline"] = {"value": round(4 / med, 2), "unit": "patches/s", "cores": threads, "kind": "port",
                               "sample": "median of 3 B=4 training steps (forward + autograd backward) of "
                                         "oracle/fusat_oracle.py after 1 warm-up"}
    return out, (cpu_leg if cpu else None)


PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (not the 2:1-sparsity figure)


def build_step(dev, precision, world, rank, batch, exchange, warmup, use_graph):
    """The benchmarked training step.  Returns (step, model, inputs, holder, launch).

    exchange: False (no collective) or True: a parallel.GradExchange, with which the backward hands its three
    head-first gradient buckets to RCCL on a side stream as it completes them, and AdamW is ordered
    after the last one (fused_train_step(exchange=...)).  The whole step — forward, CE, backward, the
    bucket all-reduces, AdamW — is captured as ONE hipGraph; if the capture fails the step runs eagerly
    and the line says so (`launch`)."""
    from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step, parallel
    torch.manual_seed(0)
    model = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, "multi_clock_gate", precision=precision).to(dev).train()
    exchange = parallel.GradExchange(model, force=True) if exchange else None
    if world > 1:
        dist.broadcast(model.flat_params.data, 0)
    opt = AdamW(model.parameters(), lr=8e-4)
    opt.grad_scale = 1.0 / world
    w = torch.ones(16)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w.to(dev))
    hsi, lidar, target = synthetic(batch, 1000 + rank, dev)
    holder = {}

    def body():
        holder["loss"] = fused_train_step(model, crit, hsi, lidar, target, optimizer=opt, exchange=exchange)

    def eager_step():
        opt.zero_grad(set_to_none=True)
        body()

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(max(3, warmup)):
            eager_step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    launch = "eager"
    step = eager_step
    if use_graph:
        try:
            opt.zero_grad(set_to_none=True)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                body()
            step = graph.replay
            launch = "hipGraph (whole step" + (", bucketed RCCL all-reduce inside)" if exchange is not None else ")")
            holder["graph"] = graph
        except RuntimeError as e:  # reported in the line, never silent
            launch = f"eager (graph capture failed: {str(e)[:100]})"
            torch.cuda.synchronize(dev)
    return step, model, (hsi, lidar, target), holder, launch


WARM_S = 0.4   # untimed replays before every timed leg


def warm(step, dev, seconds, world=1):
    """Untimed replays for at least `seconds`, so no timed leg starts cold (GPU clocks, caches, the
    allocator) whatever ran before it.  The count is fixed from a 5-step probe and agreed over the
    ranks (max), since the replayed step may hold collectives every rank must issue equally often."""
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(5):
        step()
    torch.cuda.synchronize(dev)
    per = max((time.perf_counter() - t0) / 5, 1e-5)
    n = torch.tensor([int(seconds / per) + 1], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
    for _ in range(int(n.item())):
        step()
    torch.cuda.synchronize(dev)
    return 5 + int(n.item())


def time_steps(step, dev, steps, world, warm_s=WARM_S):
    """K steps bracketed by barrier + synchronize on both sides; max over ranks.  Preceded by
    `warm_s` seconds of untimed replays."""
    warm(step, dev, warm_s, world)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bf16_gemm_roofline(model, batch, reps):
    """The largest contraction of the step in bf16-operand mode (hsi1.local_feature 3x3 conv, M = B*49,
    N = 256, K = 1296: the pipelined kernel's v_mfma_f32_16x16x32_bf16 over fp32 LDS stages, fp32
    accumulation) against the dense bf16 peak."""
    from vitcnn_amd._lib import lib
    from vitcnn_amd.model import _Program
    dev = model.flat_params.device
    prog = _Program(model, dev, batch, True, "grad")
    L = lib()
    M, N, K = batch * 49, 256, 9 * 144
    col = prog.ws.f("hsi1.local_feature.col", M * K)
    out = prog.ws.f("hsi1.local_feature.out", M * N)
    W, b = prog.P["hsi1.local_feature.conv.weight"], prog.P["hsi1.local_feature.conv.bias"]
    stream = torch.cuda.current_stream(dev)

    def fn():
        L.vc_gemm(0, 1, M, N, K, 1.0, col, K, 0, W, K, 0, 0.0, out, N, 0, 1, b, None, 0, 0, 1 | 2, None, prog.scr_p,
                  prog.scr_n, stream.cuda_stream)

    t = time_kernel(fn, reps, stream)
    flops = 2.0 * M * N * K
    achieved = flops / t / 1e12
    return {"kernel": "gp::gemm_pipe<64,64> bf16 MFMA over fp32 stages (hsi1.local_feature conv3x3, M=%d N=%d K=%d)"
            % (M, N, K),
            "bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_BF16_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_MFMA_TFLOPS, 5), "avg_launch_us": round(t * 1e6, 2),
            "flop_per_launch": flops}


def mfu(value_per_gpu, peak):
    tf = value_per_gpu * GFLOP_PER_PATCH * 1e-3
    return {"gflop_per_patch": GFLOP_PER_PATCH, "achieved_tflops": round(tf, 3), "peak_tflops": peak,
            "frac": round(tf / peak, 5)}


def precision_leg(dev, precision, steps, warmup, reps):
    """The same N = 1 training step in the other GEMM-operand precision (config 2 = bf16)."""
    step, model, _, holder, launch = build_step(dev, precision, 1, 0, 64, False, warmup, True)
    el = time_steps(step, dev, steps, 1)
    v = 64 * steps / el
    out = {"workload": "ViT-CNN train step, Houston2013 shape, B=64, GEMM operands " + precision,
           "value": round(v, 1), "unit": "patches/s", "ms_per_step": round(el / steps * 1e3, 4), "dtype": precision,
           "launch": launch, "final_loss": round(float(holder["loss"].item()), 6)}
    if precision == "bf16":
        out["model_flops_util"] = mfu(v, PEAK_BF16_MFMA_TFLOPS)
        out["roofline_gemm"] = bf16_gemm_roofline(model, 64, reps)
    else:
        out["model_flops_util"] = mfu(v, PEAK_FP32_MFMA_TFLOPS)
    return out


def f1_leg(dev, seed, cpu):
    """Row F1: whole-image inference, model_utils.test (model_utils.py:1067-1132)
    over a Houston2013-size synthetic scene (349 x 1905, 144 + 1 bands, 9x9 windows, stride 1:
    646,877 windows), eval-mode BatchNorm (running statistics), device-side window gather and fp64
    centre-pixel accumulation (vitcnn_amd.window.SlidingWindowInference).  CPU baseline: the oracle's
    eval-mode forward (the reference per-window path's arithmetic) on B=64 windows."""
    from vitcnn_amd import Multimodality_Mamba
    from vitcnn_amd.window import SlidingWindowInference
    torch.manual_seed(0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev)
    img1, img2, _ = synthetic_scene(seed)
    # warm-up on a small crop builds the eval workspaces of the batch sizes the full run uses
    for _ in range(3):
        SlidingWindowInference(m, img1[:80, :80], img2[:80, :80], 9, 1, 16, dev).run(batch_size=64)
    runner = SlidingWindowInference(m, img1, img2, 9, 1, 16, dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    probs = runner.run(batch_size=64)
    el = time.perf_counter() - t0
    out = {"workload": "test(): 349x1905 scene, 144+1 bands, 9x9 windows, stride 1, eval mode, 4096 windows per "
                       "forward, fp64 centre accumulation (incl. the probability map's copy to the host)",
           "windows": runner.n, "value": round(runner.n / el, 1), "unit": "windows/s", "seconds": round(el, 3),
           "dtype": "fp32", "probs_finite": bool(np.isfinite(probs).all())}
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}

    def cpu_leg():   # run after every GPU leg
        from oracle import vitcnn_oracle as O
        threads = cpu_threads()
        torch.set_num_threads(threads)
        st = O.make_state(sd, requires_grad=False)
        x1, x2, _ = synthetic(64, 77, "cpu")
        P = O.Params(st, training=False)
        with torch.no_grad():
            med, _ = timed_median(lambda: O.forward(P, x1, x2), 2, 3)
        out["cpu_baseline"] = {"value": round(64 / med, 2), "unit": "windows/s", "cores": threads, "kind": "port",
                               "sample": "median of 3 eval-mode B=64 forwards of oracle/vitcnn_oracle.py after 2 warm-up"}
    return out, (cpu_leg if cpu else None)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif args.force_exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    exchange = world > 1 or args.force_exchange
    log(f"rank {rank}/{world}: building the {args.precision} step")
    step, model, (hsi, lidar, target), holder, launch = build_step(
        dev, args.precision, world, rank, args.batch, exchange, args.warmup, not args.no_graph)
    if args.roofline_only:
        out = {"roofline": dominant_kernel_roofline(model, args.batch, args.kernel_reps),
               "roofline_gemm": gemm_roofline(model, args.batch, args.kernel_reps)}
        print(json.dumps(out), flush=True)
        return
    log(f"timing {args.steps} steps ({launch})")
    elapsed = time_steps(step, dev, args.steps, world)
    loss_val = float(holder["loss"].item())

    # reference-loop variant: loss.item() host sync every step (model_utils.py:936)
    warm(step, dev, WARM_S / 2, world)
    t1 = time.perf_counter()
    nsync = min(args.steps, 50)
    for _ in range(nsync):
        step()
        holder["loss"].item()
    torch.cuda.synchronize(dev)
    ms_sync = (time.perf_counter() - t1) / nsync * 1e3

    # second number: the same step fed by on-device batch assembly (row F2):
    # MultiModalX patches with flip / rot90 augmentation gathered from an HBM-resident
    # Houston2013-size cube (349 x 1905, 144 + 1 bands) into the step's input buffers
    ms_asm = batch_assembly_ms(step, hsi, lidar, target, dev, min(args.steps, 50), 1000 + rank)

    roof = dominant_kernel_roofline(model, args.batch, args.kernel_reps)
    roof_gemm = (gemm_roofline if args.precision == "fp32" else bf16_gemm_roofline)(model, args.batch,
                                                                                     args.kernel_reps)
    patches = world * args.batch * args.steps
    value = patches / elapsed
    peak = PEAK_FP32_MFMA_TFLOPS if args.precision == "fp32" else PEAK_BF16_MFMA_TFLOPS
    out = {
        "metric": "training patches/sec, 9×9 HSI(144)+LiDAR patch, batch 64, 1/2/4/8 GPU",
        "value": round(value, 1), "unit": "patches/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (U[0,1) HSI/LiDAR patches, random-init weights, resident in HBM)",
        "config": {"workload": "ViT-CNN (Multimodality_Mamba) train step, Houston2013 shape 144+1 bands, 9x9, "
                               "16 classes", "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                   "parallelism": f"dp{world}", "launch": launch,
                   "gradient_exchange": (None if not exchange else
                                         "RCCL all-reduce of 3 head-first buckets on a side stream, overlapped "
                                         "with the backward; 1/world folded into AdamW")},
        "ms_per_step_with_loss_item": round(ms_sync, 4),
        "value_with_loss_item": round(world * args.batch / ms_sync * 1e3, 1),
        "ms_per_step_with_batch_assembly": round(ms_asm, 4),
        "value_with_batch_assembly": round(world * args.batch / ms_asm * 1e3, 1),
        "final_loss": round(loss_val, 6),
        "model_flops_util": mfu(value / world, peak),
        "roofline": roof,
        "roofline_gemm": roof_gemm,
    }
    cpu_legs = []
    if world == 1 and not args.no_s2eft:
        other = "bf16" if args.precision == "fp32" else "fp32"
        log(f"{other} leg")
        out["config2_bf16" if other == "bf16" else "parity_fp32"] = precision_leg(
            dev, other, min(args.steps, 50), args.warmup, args.kernel_reps)
        log("config 5: S2EFT leg")
        out["config5_s2eft"], c = s2eft_leg(dev, min(args.steps, 50), 0 if args.no_cpu_baseline else 5)
        cpu_legs.append(c)
        log("config 5: FusAtNet leg")
        out["config5_fusatnet"], c = fusat_leg(dev, 5, not args.no_cpu_baseline)
        cpu_legs.append(c)
        log("config 4: MUUFL leg")
        out["config4_muufl"] = muufl_leg(dev, min(args.steps, 50))
    if world == 1 and not args.no_f1:
        log("F1: whole-image test()")
        out["f1_test"], c = f1_leg(dev, 1000 + rank, not args.no_cpu_baseline)
        cpu_legs.append(c)
    if world == 1 and not args.no_train_loop:
        log("train(): the plugin-surface loop over a PatchBatcher loader")
        # train() prints the reference's progress lines; stdout carries only the one JSON line
        with contextlib.redirect_stdout(sys.stderr):
            out["value_via_train_loop"] = train_loop_leg(dev, 3, 1000 + rank, elapsed / args.steps * 1e3)
    # the CPU baselines last: minutes of all-core CPU work that must not precede a timed GPU leg
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log(f"CPU baseline: {args.cpu_warmup} + {args.cpu_steps} oracle steps on {cpu_threads()} threads")
        out["cpu_baseline"] = cpu_baseline(args.cpu_warmup, args.cpu_steps)
        for c in cpu_legs:
            if c is not None:
                c()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
