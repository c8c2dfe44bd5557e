"""Plugin surface of the reference (`model_utils.py`) for the ViT-CNN path, over the MI355X model.

Same names, arguments, defaults and error behaviour as the reference functions this file
replaces, so `main.py`-style drivers switch by changing one import:

* `get_model(name, **kwargs) -> (model, optimizer, criterion, kwargs)`  — model_utils.py:47-511,
  ViT-CNN branch :297-313, defaults :493-510, unknown name -> KeyError (:488-489).
* `train(savename, run, bands, net, optimizer, criterion, data_loader, epoch, ...)` — :854-1045.
* `save_model(savename, model, model_name, dataset_name, train_state, type, **kwargs)` — :1047-1064.
* `test(run, net, img1, img2, hyperparams) -> probs[W, H, n_classes]` — :1067-1132.
* `val(net, data_loader, device, supervision) -> accuracy` — :1135-1158.

Registered: "Multimodality_Mamba" (the README's "ViT-CNN (ours)"), "S2EFT" (config 5, :400-423) and
"FusAtNet" (config 5, :109-118).
The reference's other branches import modules absent from the reference tree (SURVEY.md section 2a
row 22) and are out of scope for this path.

Data parallelism: when a torch.distributed process group with more than
one rank is initialised, `train` starts every replica from rank 0's parameters, all-reduces the
gradient after every backward (RCCL) and folds the 1/world average into the fused AdamW update;
each rank iterates its own shard of the batches (a loader that is not already sharded is wrapped in
`parallel.ShardedLoader`, which shards a torch DataLoader at its sampler).

Precision (BASELINE.json config 2): `get_model(..., precision="bf16")` builds ViT-CNN with bf16
GEMM operands and fp32 accumulation (`Multimodality_Mamba.set_precision`); the default "fp32" is
the parity mode.
"""
from __future__ import annotations

import copy
import datetime
import os
import re

import numpy as np
import torch

from . import parallel
from .losses import CrossEntropyLoss
from .model import Multimodality_Mamba
from .optim import AdamW
from .window import SlidingWindowInference

REGISTERED = ("Multimodality_Mamba", "S2EFT", "FusAtNet")


def camel_to_snake(name: str) -> str:
    """utils.py camel_to_snake: 'Multimodality_Mamba' -> 'multimodality__mamba'."""
    s = re.sub("(.)([A-Z][a-z]+)", r"\1_\2", name)
    return re.sub("([a-z0-9])([A-Z])", r"\1_\2", s).lower()


def get_model(name, **kwargs):
    """Instantiate the model, optimizer and criterion with the reference's defaults.

    Required kwargs (as in the reference): n_classes, n_bands=(hsi_bands, lidar_bands),
    ignored_labels, dataset.  `device` defaults to the first ROCm device (the MI355X path has no
    CPU execution; the reference defaults to CPU).
    """
    if name not in REGISTERED:
        raise KeyError("{} model is unknown.".format(name))
    device = kwargs.setdefault("device", torch.device("cuda" if torch.cuda.is_available() else "cpu"))
    n_classes = kwargs["n_classes"]
    (n_bands, n_bands2) = kwargs["n_bands"]
    weights = torch.ones(n_classes)
    weights[torch.LongTensor(list(kwargs["ignored_labels"]))] = 0.0
    weights = weights.to(device)
    weights = kwargs.setdefault("weights", weights)
    if name == "S2EFT":
        return _get_s2eft(n_bands, n_classes, device, kwargs)
    if name == "FusAtNet":
        return _get_fusatnet(n_bands, n_bands2, n_classes, device, kwargs)
    kwargs.setdefault("patch_size", 9)
    patch_size = kwargs["patch_size"]
    center_pixel = True
    embed_dim = 64 // 2
    kwargs.setdefault("applyPCA", False)
    if kwargs["applyPCA"]:
        n_bands = 30
    path_type = "multi_clock_gate"
    precision = kwargs.setdefault("precision", "fp32")
    model = Multimodality_Mamba(img_size=patch_size, patch_size=1, stride=1, in_channels1=n_bands,
                                in_channels2=n_bands2, dim_embedding=embed_dim, num_class=n_classes,
                                path_type=path_type, precision=precision)
    lr = kwargs.setdefault("lr", 8e-4)
    model = model.to(device)
    optimizer = AdamW(model.parameters(), lr=lr)
    criterion = CrossEntropyLoss(weight=kwargs["weights"])
    kwargs.setdefault("epoch", 200)
    kwargs.setdefault("batch_size", 64)
    kwargs.setdefault("scheduler", torch.optim.lr_scheduler.StepLR(optimizer, step_size=30, gamma=0.9))
    kwargs.setdefault("supervision", "full")
    kwargs.setdefault("flip_augmentation", False)
    kwargs.setdefault("radiation_augmentation", False)
    kwargs.setdefault("mixture_augmentation", False)
    kwargs["center_pixel"] = center_pixel
    return model, optimizer, criterion, kwargs


def _get_s2eft(n_bands, n_classes, device, kwargs):
    """S2EFT branch of model_utils.py:400-423 (config 5): ViT(image_size=patch_size, near_band 3,
    num_patches=n_bands, dim 64, depth 5, heads 4, mlp_dim 8, dropout 0.1, mode 'CAF'), Adam(lr 5e-4),
    weighted CE, epoch 600, batch 64.  Adam = the fused AdamW kernel with weight_decay 0.  The model
    takes x [B, n_bands + 1, patch_size**2 * 3]."""
    from .s2eft import ViT
    kwargs.setdefault("patch_size", 7)
    kwargs.setdefault("applyPCA", False)
    if kwargs["applyPCA"]:
        n_bands = 30
    model = ViT(image_size=kwargs["patch_size"], near_band=3, num_patches=n_bands, num_classes=n_classes, dim=64,
                depth=5, heads=4, mlp_dim=8, dropout=0.1, emb_dropout=0.1, mode="CAF").to(device)
    lr = kwargs.setdefault("lr", 0.0005)
    optimizer = AdamW(model.parameters(), lr=lr, weight_decay=0.0)
    criterion = CrossEntropyLoss(weight=kwargs["weights"])
    kwargs.setdefault("epoch", 600)
    kwargs.setdefault("batch_size", 64)
    kwargs.setdefault("supervision", "full")
    kwargs["center_pixel"] = True
    return model, optimizer, criterion, kwargs


def _get_fusatnet(n_bands, n_bands2, n_classes, device, kwargs):
    """FusAtNet branch of model_utils.py:109-118: FusAtNet(n_bands, n_bands2, n_classes), patch 11,
    Adam(lr 1e-3) as in the reference -- the fused AdamW kernel with weight_decay 0 over the model's flat
    parameter buffer (torch.optim.Adam's update exactly) --, weighted CE, epoch 150, batch 64, applyPCA False.
    The reference's backward raises (in-place residual add); this path trains with
    out-of-place residual semantics (vitcnn_amd/fusatnet.py)."""
    from .fusatnet import FusAtNet
    kwargs.setdefault("patch_size", 11)
    model = FusAtNet(n_bands, n_bands2, n_classes).to(device)
    lr = kwargs.setdefault("lr", 0.001)
    optimizer = AdamW(model.parameters(), lr=lr, weight_decay=0.0)
    criterion = CrossEntropyLoss(weight=kwargs["weights"])
    kwargs.setdefault("epoch", 150)
    kwargs.setdefault("batch_size", 64)
    kwargs.setdefault("applyPCA", False)
    kwargs.setdefault("supervision", "full")
    kwargs["center_pixel"] = True
    return model, optimizer, criterion, kwargs


def save_model(savename, model, model_name, dataset_name, train_state, type, **kwargs):
    """Checkpoint scheme of model_utils.py:1047-1064: a plain state_dict (the reference's 1704 keys)
    at ./checkpoints/<model>/<dataset>/<train_state>/<type>/<time><savename>_run{run}_epoch{epoch}_{metric:.2f}.pth.
    Only rank 0 writes under data parallelism."""
    if parallel.rank() != 0:
        return None
    model_dir = "./checkpoints/" + model_name + "/" + dataset_name + "/" + train_state + "/" + type + "/"
    time_str = datetime.datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
    os.makedirs(model_dir, exist_ok=True)
    if not isinstance(model, torch.nn.Module):
        raise TypeError("save_model: only torch modules are checkpointed on this path")
    filename = time_str + savename + "_run{run}_epoch{epoch}_{metric:.2f}".format(**kwargs)
    path = model_dir + filename + ".pth"
    if hasattr(model, "snapshot_state_dict"):
        # the flat buffers in one device-to-host copy each (not 1704 per-tensor transfers)
        sd = model.snapshot_state_dict(device="cpu")
    else:
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save(sd, path)
    return path


def _stepper(net, optimizer, criterion):
    """the model's TrainStepper for this optimizer / criterion (kept across train() calls, so the
    captured per-shape graphs are reused)"""
    from .step import TrainStepper
    st = getattr(net, "_vc_stepper", None)
    if st is None or st.opt is not optimizer or st.crit is not criterion or \
            (st.exchange is None) == parallel.is_distributed():
        st = TrainStepper(net, optimizer, criterion)
        object.__setattr__(net, "_vc_stepper", st)
    return st


def train(savename, run, bands, net, optimizer, criterion, data_loader, epoch, scheduler=None, display_iter=100,
          device=torch.device("cpu"), display=None, val_loader=None, supervision="full"):
    """Training loop of model_utils.py:854-1045: per batch one optimizer step (zero_grad, forward,
    criterion, backward, step: :916-934), the loss recorded per iteration (:936-938) and its running
    mean printed every `display_iter` iterations (:940-962), the scheduler stepped per epoch
    (:997-1000), best-state tracking with best / final checkpoints (:1015-1043).  `display` (visdom)
    is optional here.

    The step is `vitcnn_amd.step.TrainStepper.step`: for ViT-CNN with the fused AdamW one hipGraph
    replay per batch (captured per batch shape; data parallel: bucketed RCCL all-reduce inside it).
    The per-iteration losses stay on the device and are read in one transfer at each display point
    and at the epoch end (the reference's `loss.item()` host sync per iteration would stall the queue
    every step); the recorded values are the same.

    Data parallel (a process group with more than one rank): replicas start from rank 0's parameters,
    a loader that is not already sharded is wrapped in `parallel.ShardedLoader` (every rank the same
    number of batches: one gradient exchange per batch on every rank; a torch DataLoader is sharded at
    its sampler, so each rank assembles only its own batches), a loader that shards itself
    (PatchBatcher(rank=, world=)) is checked against the group, and the per-epoch metric that
    decides the best-state branch -- whose buffer broadcast is a collective -- is the mean over the
    ranks (validation: accuracy over the union of the ranks' validation batches), so every rank takes
    the same branch.  `train.last_stats` holds per-epoch wall times and batch counts."""
    import time
    if criterion is None:
        raise Exception("Missing criterion. You must specify a loss function.")
    if supervision != "full":
        raise ValueError('supervision mode "{}" is unknown.'.format(supervision))
    net.to(device)
    distributed = parallel.is_distributed()
    if distributed:
        parallel.broadcast_parameters(net)       # replicas start identical (rank 0's values)
        parallel.check_loader_shard(data_loader)  # a self-sharding loader (PatchBatcher) agrees with the group
        if not parallel.is_sharded(data_loader):
            data_loader = parallel.ShardedLoader(data_loader, parallel.rank(), parallel.world())
    stepper = _stepper(net, optimizer, criterion)
    save_epoch = 16 if epoch == 128 else (epoch // 20 if epoch > 20 else 1)
    best_val_acc = 0.0
    best_model_wts = None
    losses = []
    iter_ = 1
    val_accuracies = []
    stats = {"epochs": [], "launch": None}
    train.last_stats = stats
    for e in range(1, epoch + 1):
        t_epoch = time.perf_counter()
        net.train()
        pending = []          # device losses not yet read back
        nb = npatch = 0
        avg_loss = 0.0
        n_batches = len(data_loader)
        for batch_idx, (data, data2, target) in enumerate(data_loader):
            loss = stepper.step(data, data2, target)
            if stepper.fused:
                loss = loss.clone()   # a replayed graph's loss buffer is overwritten by the next replay
            pending.append(loss.detach())
            nb += 1
            npatch += int(target.shape[0])
            if display_iter and iter_ % display_iter == 0:
                vals = torch.stack(pending).tolist() if pending else []
                pending = []
                losses.extend(vals)
                if parallel.rank() == 0:
                    mean_loss = float(np.mean(losses[max(0, len(losses) - 101):]))
                    print("Train (epoch {}/{}) [{}/{} ({:.0f}%)]\tLoss: {:.6f}".format(
                        e, epoch, batch_idx * len(data), len(data) * n_batches,
                        100.0 * batch_idx / max(n_batches, 1), mean_loss), flush=True)
                    if display is not None and hasattr(display, "line"):
                        display.line(X=np.arange(len(losses)), Y=np.asarray(losses), win="loss")
            iter_ += 1
        if pending:
            losses.extend(torch.stack(pending).tolist())
        avg_loss = float(np.sum(losses[len(losses) - nb:])) / max(nb, 1) if nb else 0.0
        if val_loader is not None:
            correct, total = _val_counts(net, val_loader, device)
            if distributed:
                correct, total = parallel.sum_over_ranks([correct, total])
            val_acc = correct / total
            val_accuracies.append(val_acc)
            metric = -val_acc
        else:
            metric = parallel.mean_over_ranks(avg_loss) if distributed else avg_loss
        if isinstance(scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
            scheduler.step(metric)
        elif scheduler is not None:
            scheduler.step()
        if abs(metric) >= best_val_acc:
            best_val_acc = abs(metric)
            parallel.broadcast_buffers(net)
            best_model_wts = (net.snapshot_state_dict() if hasattr(net, "snapshot_state_dict")
                              else copy.deepcopy(net.state_dict()))
            if e % save_epoch == 0:
                save_model(savename, net, camel_to_snake(str(net.__class__.__name__)), data_loader.dataset.name,
                           train_state="train", type="best_epoch", run=run, epoch=e, metric=abs(metric))
        if e == epoch:
            parallel.broadcast_buffers(net)
            save_model(savename, net, camel_to_snake(str(net.__class__.__name__)), data_loader.dataset.name,
                       train_state="train", type="final_epoch", run=run, epoch=e, metric=abs(metric))
        stats["epochs"].append({"seconds": time.perf_counter() - t_epoch, "batches": nb, "patches": npatch})
        stats["launch"] = stepper.launch
    stats["losses"] = losses
    return best_model_wts


def val(net, data_loader, device="cpu", supervision="full"):
    """model_utils.py:1135-1158: argmax accuracy over samples whose PREDICTION is not an ignored
    label.  Like the reference, the network is not switched to eval mode (it runs in whatever
    mode it is in — train mode when called from `train`).  The per-sample `.item()` loop becomes
    an on-device comparison with one host sync per batch."""
    correct, total = _val_counts(net, data_loader, device)
    return correct / total


def _val_counts(net, data_loader, device):
    """(correct, counted) of val(): the host counts, summed over ranks by train() under DP"""
    ignored = sorted(set(getattr(data_loader.dataset, "ignored_labels", [])))
    correct, total = 0, 0
    for data, data2, target in data_loader:
        with torch.no_grad():
            data, data2, target = data.to(device), data2.to(device), target.to(device)
            output = net(data, data2)
            if isinstance(output, tuple):
                output = output[0]
            pred = output.argmax(dim=1).view(-1)
            keep = torch.ones_like(pred, dtype=torch.bool)
            for lab in ignored:
                keep &= pred != lab
            correct += int(((pred == target.view(-1)) & keep).sum())
            total += int(keep.sum())
    return correct, total


def test(run, net, img1, img2, hyperparams):
    """Whole-image inference of model_utils.py:1067-1132 (center-pixel mode): eval-mode forward over
    every sliding window, probabilities accumulated at the window centres.  The image is uploaded
    once; windows are gathered on the device (vc_window_gather) and the logits scattered into an
    fp64 probability map on the device (vc_center_accumulate), so the Python generator + np.copy
    per window of the reference disappears.  Returns a float64 numpy array [W, H, n_classes] like
    the reference's `probs`."""
    net.eval()
    if hyperparams.get("applyPCA", False):
        img1 = apply_pca(img1, 3)   # model_utils.py:1076-1077 (3 components, as the reference)
    runner = SlidingWindowInference(net, img1, img2, patch_size=hyperparams["patch_size"],
                                    step=hyperparams.get("test_stride", 1), n_classes=hyperparams["n_classes"],
                                    device=hyperparams["device"])
    return runner.run(batch_size=hyperparams["batch_size"])


def apply_pca(X, num_components):
    """utils.py:85-93 applyPCA: whitened PCA of the [W, H, C] cube's pixel spectra (host-side data
    preparation, as in the reference; sklearn's PCA)."""
    from sklearn.decomposition import PCA
    X = np.asarray(X)
    flat = np.reshape(X, (-1, X.shape[2]))
    flat = PCA(n_components=num_components, whiten=True).fit_transform(flat)
    return np.reshape(flat, (X.shape[0], X.shape[1], num_components))
