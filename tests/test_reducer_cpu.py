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


def test_consecutive_layer_blocks_adjacent(model):
    """layer i's six-matrix block ends where layer i + 1's begins, so a reducer bucket of k layers is one
    contiguous range (GradReducer merge_elems)"""
    from eegfusion.modules import _LAYER_MATRICES
    from eegfusion.trainer import GradReducer
    a = model.arena
    blocks = [GradReducer.ranges(a, [f"bert.encoder.layer.{i}.{k}" for k in _LAYER_MATRICES])[0] for i in range(12)]
    assert all(blocks[i][1] == blocks[i + 1][0] for i in range(11))
    # the fused Q|K|V bias is still one contiguous [2304] span
    qb = GradReducer.ranges(a, [f"bert.encoder.layer.3.attention.self.{k}.bias" for k in ("query", "key", "value")])
    assert len(qb) == 1 and qb[0][1] - qb[0][0] == 2304


def test_merge_plan(model):
    """merge_elems: ready() groups are held until they reach the threshold, then issued as one merged
    collective; finish() issues what is held"""
    from eegfusion.modules import _LAYER_MATRICES
    from eegfusion.trainer import GradReducer
    a = model.arena
    names = lambda i: [f"bert.encoder.layer.{i}.{k}" for k in _LAYER_MATRICES]
    blk = 4 * 768 * 768 + 2 * 768 * 3072
    r = GradReducer(bucket_elems=64 << 20, merge_elems=3 * blk)
    r.begin(a, [n for i in range(12) for n in names(i)])
    for i in (11, 10):
        r.ready(names(i))
    assert r.log == []
    r.ready(names(9))
    b9 = GradReducer.ranges(a, names(9))[0]
    b11 = GradReducer.ranges(a, names(11))[0]
    assert r.log == [(b9[0], b11[1])]
    r.ready(names(8))
    assert len(r.log) == 1                                   # held: below the threshold
    lo, hi = a.model_range
    r.finish(lo, hi)
    assert r.log[1] == GradReducer.ranges(a, names(8))[0]    # flushed first, then the never-ready rest


def test_plan_coalesces_small_ranges():
    """small ranges are gathered into bucket-sized groups; one that would sit alone is reduced by itself
    (the coalescing keeps going after it instead of giving up on the rest)"""
    from eegfusion.trainer import GradReducer
    r = GradReducer(bucket_elems=100, coalesce_elems=40)
    plan = r.plan([(0, 30), (64, 94), (128, 158), (192, 500), (512, 530)])
    groups = [g for g in plan if len(g) > 1]
    assert groups == [[(0, 30), (64, 94), (128, 158)]]     # 90 <= 100; (512, 530) would start a new group alone
    singles = [g[0] for g in plan if len(g) == 1]
    assert (512, 530) in singles
    assert [(i, j) for i, j in singles if i >= 192 and j <= 500] == [(192, 292), (292, 392), (392, 492), (492, 500)]
    assert GradReducer(bucket_elems=100).coalesce == 50      # clamped to half a bucket
