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
    order of the shuffled `indices` (DataLoader(shuffle=False) over the dataset, as main.py builds
    it).  `rank`/`world` select a disjoint shard for data parallelism."""

    def __init__(self, img1, img2, gt, patch_size: int, ignored_labels=(0,), batch_size: int = 64,
                 flip_augmentation: bool = False, device="cuda", seed: int = 0, rank: int = 0, world: int = 1,
                 name: str = "synthetic"):
        self.device = torch.device(device)
        self.c1, self.c2 = _cube(img1, self.device), _cube(img2, self.device)
        self.P, self.bs, self.flip = int(patch_size), int(batch_size), bool(flip_augmentation)
        self.ignored_labels = set(ignored_labels)
        self.name = name
        gt = np.asarray(gt)
        mask = np.ones_like(gt)
        for lab in self.ignored_labels:
            mask[gt == lab] = 0
        xs, ys = np.nonzero(mask)
        p = self.P // 2
        keep = (xs > p) & (xs < gt.shape[0] - p) & (ys > p) & (ys < gt.shape[1] - p)
        idx = np.stack([xs[keep], ys[keep]], axis=1)
        self.rng = np.random.RandomState(seed)
        self.rng.shuffle(idx)
        idx = idx[rank::world] if world > 1 else idx
        self.centers = idx
        self.labels = torch.as_tensor(gt[idx[:, 0], idx[:, 1]].astype(np.int64)).to(self.device)
        corners = (idx - p).astype(np.int32)
        self.corners = torch.as_tensor(np.ascontiguousarray(corners)).to(self.device)
        self.W, self.H = int(self.c1.shape[0]), int(self.c1.shape[1])

    def __len__(self):
        return -(-len(self.centers) // self.bs)

    def xform_codes(self, n: int) -> np.ndarray:
        """MultiModalX flip/rotate decisions (datasets.py:511-526, :559-564) as gather codes."""
        codes = np.zeros(n, dtype=np.uint8)
        if not self.flip or self.P <= 1:
            return codes
        r = self.rng
        for i in range(n):
            if r.random_sample() > 0.5:
                h = r.random_sample() > 0.5
                v = r.random_sample() > 0.5
                codes[i] = (1 if h else 0) | (2 if v else 0)
            elif r.random_sample() > 0.5:
                codes[i] = int(r.choice([1, 2, 3])) << 2
        return codes

    def __iter__(self):
        L = lib()
        s = torch.cuda.current_stream(self.device).cuda_stream
        C1, C2, P = int(self.c1.shape[2]), int(self.c2.shape[2]), self.P
        for b0 in range(0, len(self.centers), self.bs):
            n = min(self.bs, len(self.centers) - b0)
            x1 = torch.empty(n, C1, P, P, device=self.device)
            x2 = torch.empty(n, C2, P, P, device=self.device)
            cor = self.corners[b0:b0 + n]
            xf = None
            if self.flip:
                xf = torch.as_tensor(self.xform_codes(n)).to(self.device)
            L.vc_patch_gather(self.W, self.H, C1, P, self.c1.data_ptr(), cor.data_ptr(), 0, 0, n,
                              xf.data_ptr() if xf is not None else None, x1.data_ptr(), s)
            L.vc_patch_gather(self.W, self.H, C2, P, self.c2.data_ptr(), cor.data_ptr(), 0, 0, n,
                              xf.data_ptr() if xf is not None else None, x2.data_ptr(), s)
            yield x1, x2, self.labels[b0:b0 + n]
