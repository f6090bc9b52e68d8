"""Overlapped gradient reduction on a real PriGumbel step (single GPU: no collective is launched,
but GradReducer records the ranges it would all-reduce): every used parameter's gradient range is
covered exactly once, BERT layers are issued one block at a time during the backward (layer 11
first), and the step's gradients equal those of a step with the reducer's hooks disabled."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from eegfusion.modules import PriGumbelModel
    torch.manual_seed(3)
    return PriGumbelModel(1.0, contract="W", dropout=0.0).cuda()


def _batch(B=4):
    g = torch.Generator(device="cuda").manual_seed(11)
    eeg = torch.randn(B, 64, 256, generator=g, device="cuda")
    act = torch.randn(B, 32, generator=g, device="cuda") * 0.5
    labels = (torch.rand(B, generator=g, device="cuda") < 0.66).long()
    return {"eeg": eeg, "act": act}, labels


def test_reducer_covers_used_params_once():
    from eegfusion.modules import _LAYER_MATRICES
    from eegfusion.trainer import GradReducer, PriGumbelTrainer
    m = _model()
    r = GradReducer()
    tr = PriGumbelTrainer(m.engine, reducer=r)
    batch, labels = _batch()
    tr.step(batch, labels)
    torch.cuda.synchronize()
    a = m.arena
    log = sorted(r.log)
    assert all(log[i][1] <= log[i + 1][0] for i in range(len(log) - 1)), "overlapping ranges"
    for n in tr.model_params:
        off, s = a.offsets[n]
        end = off + a._numel(s)
        assert sum(max(0, min(hi, end) - max(lo, off)) for lo, hi in log) == end - off, n
    # issue order: decoder/head matrices, then layer 11 .. 0 blocks, then the deferred vectors
    blocks = [GradReducer.ranges(a, [f"bert.encoder.layer.{i}.{k}" for k in _LAYER_MATRICES])[0]
              for i in range(12)]
    pos = [r.log.index(b) for b in blocks]
    assert pos == sorted(pos, reverse=True)
    assert pos[11] >= 1 and pos[0] < len(r.log) - 1


def test_reducer_hooks_do_not_change_the_step():
    from eegfusion.trainer import GradReducer, PriGumbelTrainer

    class NoHooks(GradReducer):
        def ready(self, names):
            pass

    out = []
    for red in (GradReducer(), NoHooks()):
        m = _model()
        tr = PriGumbelTrainer(m.engine, lr=1e-3, reducer=red, consume_grads=False)
        batch, labels = _batch()
        tr.step(batch, labels)
        torch.cuda.synchronize()
        out.append(m.arena.grad.clone())
    torch.testing.assert_close(out[0], out[1], rtol=1e-5, atol=1e-7)
