"""Device-side patch windows: whole-image inference (test()) and training-batch assembly.

* `SlidingWindowInference` — model_utils.test (model_utils.py:1067-1132) over
  utils.sliding_window / count_sliding_window / grouper (utils.py:357-415, :567-582), centre-pixel
  mode.  The two image cubes are uploaded once in their source layout img[x][y][c]; each batch of
  windows is gathered on the device (vc_patch_gather) and its logits are added into an fp64
  probability map on the device (vc_center_accumulate).  Window order, clamping and the float64
  accumulation are the reference's; eval-mode BatchNorm uses running statistics, so the batch
  size only changes throughput, not results.
* `PatchBatcher` — MultiModalX (datasets.py:461-593): labelled centre pixels inside the border,
  shuffled once, batches gathered on the device with the reference's flip / rot90 augmentation
  decisions drawn on the host (datasets.py:511-526) and applied inside the gather.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import lib


def window_count(W: int, H: int, P: int, step: int) -> int:
    out = ctypes.c_long(0)
    lib().vc_window_count(W, H, P, step, ctypes.addressof(out))
    return int(out.value)


def _cube(img, device) -> torch.Tensor:
    t = torch.as_tensor(np.ascontiguousarray(img, dtype=np.float32))
    if t.dim() == 2:
        t = t.unsqueeze(-1)
    return t.to(device).contiguous()


class SlidingWindowInference:
    def __init__(self, net, img1, img2, patch_size: int, step: int = 1, n_classes: int = 16, device="cuda"):
        self.net = net
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("whole-image inference runs on a ROCm device; there is no CPU path")
        self.c1 = _cube(img1, self.device)
        self.c2 = _cube(img2, self.device)
        self.W, self.H = int(self.c1.shape[0]), int(self.c1.shape[1])
        if tuple(self.c2.shape[:2]) != (self.W, self.H):
            raise RuntimeError("the two modalities must cover the same image grid")
        self.P, self.step, self.ncls = int(patch_size), int(step), int(n_classes)
        self.n = window_count(self.W, self.H, self.P, self.step)

    @torch.no_grad()
    def run(self, batch_size: int = 64, max_batch: int = 4096) -> np.ndarray:
        """probs [W, H, n_classes] float64.  Windows go through the model `max(batch_size, ...)`
        at a time (eval-mode results do not depend on the grouping)."""
        L = lib()
        self.net.eval()
        bs = max(int(batch_size), min(int(max_batch), self.n))
        probs = torch.zeros(self.W, self.H, self.ncls, dtype=torch.float64, device=self.device)
        C1, C2, P = int(self.c1.shape[2]), int(self.c2.shape[2]), self.P
        buf1 = torch.empty(bs, C1, P, P, device=self.device)
        buf2 = torch.empty(bs, C2, P, P, device=self.device)
        s = torch.cuda.current_stream(self.device).cuda_stream
        for k0 in range(0, self.n, bs):
            n = min(bs, self.n - k0)
            x1, x2 = buf1[:n], buf2[:n]
            L.vc_patch_gather(self.W, self.H, C1, P, self.c1.data_ptr(), None, k0, self.step, n, None,
                              x1.data_ptr(), s)
            L.vc_patch_gather(self.W, self.H, C2, P, self.c2.data_ptr(), None, k0, self.step, n, None,
                              x2.data_ptr(), s)
            out = self.net(x1, x2)
            if isinstance(out, tuple):
                out = out[0]
            out = out.detach().to(torch.float32).contiguous()
            L.vc_center_accumulate(self.W, self.H, P, self.ncls, None, k0, self.step, n, out.data_ptr(),
                                   probs.data_ptr(), s)
        return probs.cpu().numpy()


class PatchBatcher:
    """Training batches of MultiModalX patches assembled on the device.

    Iterating yields (hsi [B,C1,P,P], lidar [B,C2,P,P], target [B] int64) on `device`, in the
    order of the shuffled `indices` (DataLoader(shuffle=False) over the dataset; the reference's train
    loader reshuffles every epoch, main.py:434-440, this one keeps its construction-time order).
    `rank`/`world` select a disjoint shard for data parallelism: every rank builds the batcher with the
    same `seed` and takes every world-th centre of the padded shuffled list (equal batch counts on every
    rank; `parallel.is_sharded` sees the attributes, so train() does not shard it again).

    Augmentations of MultiModalX.__getitem__ (datasets.py:559-568), per sample in the reference's
    order and with its probabilities, the decisions drawn from one host RandomState in the reference's
    call order: flip / rot90 (flip_augmentation, :511-526) folded into the gather; radiation noise
    (p 0.1: alpha ~ U(0.9, 1.1), x = alpha x + N/25, :529-532) and mixture noise (p 0.2: a1, a2 ~
    U(0.01, 1), x = (a1 x + a2 d2) / (a1 + a2) + N/25 with d2 the spectra of random same-class training
    pixels, :534-545) on the HSI patch by `vc_patch_noise`.  The per-element normal fields and the
    per-pixel same-class choices (the reference's np.random.normal(size=patch) / np.random.choice) are
    drawn on the device from a counter-based hash, so the host stream differs from the reference's
    after the first noisy sample (same distributions).

    Mixture noise is a deliberate divergence whose parity is UNPINNED: in the reference,
    datasets.py:540 evaluates `np.nonzero(self.labels == value)` with `self.labels` a Python list, so
    the comparison is a scalar False, np.random.choice receives an empty array and raises -- the
    reference's --mixture_augmentation never completes.  This path implements the evident intent,
    pairing the UNshuffled label list with the shuffled index list as the surrounding code does
    (:505-506, :540-543: for class v the candidates are indices[j] over the positions j with
    labels[j] == v), and is checked only against its own CPU restatement
    (oracle/patch_noise_oracle.py)."""

    def __init__(self, img1, img2, gt, patch_size: int, ignored_labels=(0,), batch_size: int = 64,
                 flip_augmentation: bool = False, device="cuda", seed: int = 0, rank: int = 0, world: int = 1,
                 name: str = "synthetic", radiation_augmentation: bool = False, mixture_augmentation: bool = False):
        self.device = torch.device(device)
        self.c1, self.c2 = _cube(img1, self.device), _cube(img2, self.device)
        self.P, self.bs, self.flip = int(patch_size), int(batch_size), bool(flip_augmentation)
        self.radiation, self.mixture = bool(radiation_augmentation), bool(mixture_augmentation)
        self.ignored_labels = set(ignored_labels)
        self.name = name
        self.seed = int(seed) & ((1 << 63) - 1)
        gt = np.asarray(gt)
        mask = np.ones_like(gt)
        for lab in self.ignored_labels:
            mask[gt == lab] = 0
        xs, ys = np.nonzero(mask)
        p = self.P // 2
        keep = (xs > p) & (xs < gt.shape[0] - p) & (ys > p) & (ys < gt.shape[1] - p)
        idx = np.stack([xs[keep], ys[keep]], axis=1)
        labels_unshuffled = gt[idx[:, 0], idx[:, 1]].astype(np.int64)
        self.rng = np.random.RandomState(seed)
        self.rng.shuffle(idx)
        self.W, self.H = int(self.c1.shape[0]), int(self.c1.shape[1])
        if self.mixture:
            self._mixture_tables(gt, idx, labels_unshuffled)
        self.rank, self.world = int(rank), int(world)
        if self.world > 1:
            # data-parallel shard: the shuffled list padded by wrapping to ceil(N / world) * world, then every
            # world-th centre from `rank` -- disjoint shards of equal length (equal batch counts: train()
            # exchanges one gradient per batch on every rank); parallel.check_loader_shard verifies that
            # every rank built its batcher from the same seed, i.e. cut its shard from the same permutation
            per = -(-len(idx) // self.world)
            idx = np.resize(idx, (per * self.world, 2))[self.rank::self.world] if len(idx) else idx
            if self.rank > 0:
                # augmentation draws of their own on every rank (rank 0 keeps the single-process stream)
                self.rng = np.random.RandomState((int(seed) + 7919 * self.rank) % (1 << 32))
        self.noise_seed = (self.seed ^ (0x9E3779B97F4A7C15 * self.rank)) & ((1 << 63) - 1)
        self.centers = idx
        self.labels = torch.as_tensor(gt[idx[:, 0], idx[:, 1]].astype(np.int64)).to(self.device)
        corners = (idx - p).astype(np.int32)
        self.corners = torch.as_tensor(np.ascontiguousarray(corners)).to(self.device)
        self.gid = 0     # samples drawn so far (the noise hash's counter)

    def _mixture_tables(self, gt, idx_shuffled, labels_unshuffled):
        """class v -> candidate source pixels idx_shuffled[j] for j with labels_unshuffled[j] == v, as
        CSR (off [nlab + 1], pix = x * H + y); ignored classes get none (d2 stays 0, :539); the label
        map as a float cube for the label-window gather"""
        nlab = int(max(int(gt.max()), int(labels_unshuffled.max()) if len(labels_unshuffled) else 0)) + 1
        order = np.argsort(labels_unshuffled, kind="stable")
        counts = np.bincount(labels_unshuffled, minlength=nlab)
        for lab in self.ignored_labels:
            if 0 <= lab < nlab:
                counts[lab] = 0
        keep = np.isin(labels_unshuffled[order], list(self.ignored_labels), invert=True)
        src = idx_shuffled[order[keep]]
        off = np.zeros(nlab + 1, dtype=np.int32)
        off[1:] = np.cumsum(counts)
        self.nlab = nlab
        self.mix_off = torch.as_tensor(off).to(self.device)
        self.mix_pix = torch.as_tensor((src[:, 0] * self.H + src[:, 1]).astype(np.int32)).to(self.device)
        self.gt_cube = torch.as_tensor(np.ascontiguousarray(gt, dtype=np.float32)[:, :, None]).to(self.device)

    def __len__(self):
        return -(-len(self.centers) // self.bs)

    @property
    def dataset(self):
        """DataLoader-style access (train() reads data_loader.dataset.name / .ignored_labels)"""
        return self

    def xform_codes(self, n: int) -> np.ndarray:
        """MultiModalX flip/rotate decisions (datasets.py:511-526, :559-564) as gather codes."""
        return self.decisions(n)[0]

    def decisions(self, n: int):
        """(xform codes [n] u8, radiation alpha [n] f32 (0: none), mixture (a1, a2) [n, 2] f32 (0: none)):
        per sample, in __getitem__'s order (datasets.py:559-568), from the batcher's RandomState"""
        codes = np.zeros(n, dtype=np.uint8)
        rad = np.zeros(n, dtype=np.float32)
        mix = np.zeros((n, 2), dtype=np.float32)
        r = self.rng
        flip = self.flip and self.P > 1
        if not (flip or self.radiation or self.mixture):
            return codes, rad, mix
        for i in range(n):
            if flip:
                if r.random_sample() > 0.5:
                    h = r.random_sample() > 0.5
                    v = r.random_sample() > 0.5
                    codes[i] = (1 if h else 0) | (2 if v else 0)
                elif r.random_sample() > 0.5:
                    codes[i] = int(r.choice([1, 2, 3])) << 2
            if self.radiation and r.random_sample() < 0.1:
                rad[i] = r.uniform(0.9, 1.1)
            if self.mixture and r.random_sample() < 0.2:
                mix[i] = r.uniform(0.01, 1.0, size=2)
        return codes, rad, mix

    def __iter__(self):
        L = lib()
        s = torch.cuda.current_stream(self.device).cuda_stream
        C1, C2, P = int(self.c1.shape[2]), int(self.c2.shape[2]), self.P
        for b0 in range(0, len(self.centers), self.bs):
            n = min(self.bs, len(self.centers) - b0)
            x1 = torch.empty(n, C1, P, P, device=self.device)
            x2 = torch.empty(n, C2, P, P, device=self.device)
            cor = self.corners[b0:b0 + n]
            codes, rad, mix = self.decisions(n)
            xf = torch.as_tensor(codes).to(self.device) if self.flip else None
            xfp = xf.data_ptr() if xf is not None else None
            L.vc_patch_gather(self.W, self.H, C1, P, self.c1.data_ptr(), cor.data_ptr(), 0, 0, n, xfp,
                              x1.data_ptr(), s)
            L.vc_patch_gather(self.W, self.H, C2, P, self.c2.data_ptr(), cor.data_ptr(), 0, 0, n, xfp,
                              x2.data_ptr(), s)
            if rad.any() or mix.any():
                self.apply_noise(x1, cor, xfp, rad, mix, s)
            self.gid += n
            yield x1, x2, self.labels[b0:b0 + n]

    def apply_noise(self, x1, cor, xfp, rad, mix, stream):
        L = lib()
        n, C1, P = x1.shape[0], x1.shape[1], self.P
        rad_d = torch.as_tensor(rad).to(self.device)
        mix_d = torch.as_tensor(np.ascontiguousarray(mix)).to(self.device)
        lab = off = pix = None
        nlab = 0
        if self.mixture:
            lab = torch.empty(n, 1, P, P, device=self.device)
            L.vc_patch_gather(self.W, self.H, 1, P, self.gt_cube.data_ptr(), cor.data_ptr(), 0, 0, n, xfp,
                              lab.data_ptr(), stream)
            off, pix, nlab = self.mix_off.data_ptr(), self.mix_pix.data_ptr(), self.nlab
        L.vc_patch_noise(n, C1, P, self.H, x1.data_ptr(), lab.data_ptr() if lab is not None else None,
                         rad_d.data_ptr(), mix_d.data_ptr(), off, pix, nlab, self.c1.data_ptr(), self.noise_seed, self.gid,
                         stream)
        self._last_noise = (rad_d, mix_d, lab)   # keep the uploads alive until the kernel has run
