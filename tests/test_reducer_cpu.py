"""GradReducer range bookkeeping on the real contract-W arena (CPU, no GPU calls): each BERT layer's
six weight matrices are one contiguous gradient range, and the coalesced ranges of the used
parameters leave out the unused template decoder layer and the word embeddings."""
import pytest
import torch


@pytest.fixture(scope="module")
def model():
    from eegfusion.modules import PriGumbelModel
    torch.manual_seed(0)
    return PriGumbelModel(1.0, contract="W", dropout=0.0)


def test_layer_matrices_one_range(model):
    from eegfusion.modules import _LAYER_MATRICES
    from eegfusion.trainer import GradReducer
    a = model.arena
    for i in range(12):
        names = [f"bert.encoder.layer.{i}.{k}" for k in _LAYER_MATRICES]
        rg = GradReducer.ranges(a, names)
        assert len(rg) == 1
        assert rg[0][1] - rg[0][0] == 4 * 768 * 768 + 2 * 768 * 3072


def test_used_ranges_exclude_unused(model):
    from eegfusion.trainer import GradReducer
    a = model.arena
    used = model.engine.graph_params() - {"DP"}
    rg = GradReducer.ranges(a, used)
    covered = sum(hi - lo for lo, hi in rg)
    total = sum(a._numel(s) for n, (_, s) in a.offsets.items() if n in used)
    assert total <= covered < total + 64 * len(used)
    for n in ("bert.embeddings.word_embeddings.weight", "multi_head_decoderlayer.linear1.weight"):
        off, s = a.offsets[n]
        assert all(hi <= off or lo >= off + a._numel(s) for lo, hi in rg), n
    assert covered < 0.8 * (a.model_range[1] - a.model_range[0])
