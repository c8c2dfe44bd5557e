"""`model_utils.train` on the MI355X: the plugin-surface loop the reference's
main.py drives runs one hipGraph replay per batch (captured per batch shape; the first batch of a
shape runs eagerly, the short last batch is its own shape), and its result is bit-identical to the
reference-style eager loop (zero_grad, forward, criterion, backward, step per batch) over the same
batches, StepLR included (the lr reaches the replayed AdamW through its device hyper tensor).
"""
import pytest
import torch

from helpers import golden_batch, hash_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class _Loader(list):
    class _DS:
        name = "synthetic"
        ignored_labels = [0]

    dataset = _DS()


def _setup():
    from vitcnn_amd import model_utils as mu
    sd = hash_state_dict()
    m, opt, crit, kw = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                    dataset="synthetic", device=torch.device(DEV))
    m.load_state_dict(sd)
    sch = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    return mu, m, opt, crit, sch


def _batches():
    hsi, lidar, target = golden_batch("golden.train", 72)
    out = _Loader()
    for b0, n in ((0, 16), (16, 16), (32, 16), (48, 16), (64, 8)):   # 4 full batches + a short last one
        out.append((hsi[b0:b0 + n].to(DEV), lidar[b0:b0 + n].to(DEV), target[b0:b0 + n].to(DEV)))
    return out


def test_train_graph_replay_equals_eager_reference_loop(tmp_path, monkeypatch):
    _need_gpu()
    monkeypatch.chdir(tmp_path)
    epochs = 3
    mu, m, opt, crit, sch = _setup()
    batches = _batches()
    mu.train("t", 0, None, m, opt, crit, batches, epochs, scheduler=sch, display_iter=2,
             device=torch.device(DEV))
    st = mu.train.last_stats
    assert st["launch"] == "hipGraph", st["launch"]
    stepper = m._vc_stepper
    assert len(stepper.graphs) == 2           # B = 16 and the short last batch B = 8
    # the reference loop, eagerly through autograd, same batches and scheduler
    _, r, ropt, rcrit, rsch = _setup()
    ref_losses = []
    for _ in range(epochs):
        r.train()
        for data, data2, target in batches:
            ropt.zero_grad()
            loss = rcrit(r(data, data2), target)
            loss.backward()
            ropt.step()
            ref_losses.append(loss.item())
        rsch.step()
    torch.cuda.synchronize()
    assert opt.param_groups[0]["lr"] == ropt.param_groups[0]["lr"] == 8e-4 * 0.5 ** epochs
    assert st["losses"] == ref_losses
    assert torch.equal(m.flat_params.detach(), r.flat_params.detach())
    for a, b in zip(m.flat_buffers(), r.flat_buffers()):
        assert torch.equal(a, b)
    ck = list((tmp_path / "checkpoints").rglob("*.pth"))
    assert any("final_epoch" in str(p) for p in ck)


def test_train_second_call_reuses_graphs_and_invalidates_on_rebind(tmp_path, monkeypatch):
    """a second train() call replays the graphs captured by the first; load_state_dict(assign=True)
    re-flattens the parameters, and the stepper drops the graphs bound to the old buffers"""
    _need_gpu()
    monkeypatch.chdir(tmp_path)
    mu, m, opt, crit, sch = _setup()
    batches = _Loader(_batches()[:3])
    mu.train("t", 0, None, m, opt, crit, batches, 1, device=torch.device(DEV), display_iter=0)
    g0 = dict(m._vc_stepper.graphs)
    assert len(g0) == 1
    mu.train("t", 0, None, m, opt, crit, batches, 1, device=torch.device(DEV), display_iter=0)
    assert m._vc_stepper.graphs.keys() == g0.keys() and all(m._vc_stepper.graphs[k] is g0[k] for k in g0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m.load_state_dict(sd, assign=True)
    mu.train("t", 0, None, m, opt, crit, batches, 1, device=torch.device(DEV), display_iter=0)
    assert all(m._vc_stepper.graphs.get(k) is not g0[k] for k in g0)
    assert torch.isfinite(m.flat_params.detach()).all()
