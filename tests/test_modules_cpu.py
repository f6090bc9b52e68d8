"""Host-side structure of the drop-in modules (no GPU compute)."""
import pytest
import torch

from oracle import fusion_oracle as O


def test_state_dict_names_match_reference_W():
    from eegfusion.modules import PriGumbelModel
    m = PriGumbelModel(1.0, contract="W")
    sd = m.state_dict()
    ref = O.param_shapes("W", "prigumbel")
    assert set(sd) == set(ref), set(sd) ^ set(ref)
    for k, s in ref.items():
        assert tuple(sd[k].shape) == tuple(s), k


def test_state_dict_names_match_reference_T_concat():
    from model import ConcatModel
    m = ConcatModel()
    ref = O.param_shapes("T", "concat")
    assert set(m.state_dict()) == set(ref)
    # attributes callers use (train.py:139, main_0430.py:144-151)
    assert m.DP.shape == (1, 2304)
    assert isinstance(m.bert.encoder.layer[-1], torch.nn.Module)
    assert isinstance(m.fc_layers, torch.nn.Sequential) and len(m.fc_layers) == 4
    assert m.classifier.weight.shape == (2, 768)


def test_priconcat_has_no_dp_and_keeps_epsilon():
    import types
    from main_0430 import ConcatModel
    m = ConcatModel(types.SimpleNamespace(EPSILON=0.5), dp_mode="feature_all_lap")
    assert "DP" not in m.state_dict()
    assert m.EPSILON == 0.5 and m.dp_mode == "feature_all_lap"


def test_optimizer_split_by_DP_substring():
    """past_acc.py:155-156 / train.py:71-72: the 'DP' substring split finds exactly one parameter."""
    from past_acc import ConcatModel
    m = ConcatModel(1.0)
    dp = [n for n, _ in m.named_parameters() if "DP" in n]
    assert dp == ["DP"]


def test_arena_views_and_qkv_adjacency():
    from eegfusion.modules import PriGumbelModel
    m = PriGumbelModel(1.0, contract="W")
    a = m.arena
    for n, p in m.named_parameters():
        assert p.data_ptr() == a.view(n).data_ptr(), n
    pre = "bert.encoder.layer.3.attention.self."
    q, k, v = (a.offset(pre + x + ".weight") for x in ("query", "key", "value"))
    assert k - q == 768 * 768 and v - k == 768 * 768
    qb, kb, vb = (a.offset(pre + x + ".bias") for x in ("query", "key", "value"))
    assert kb - qb == 768 and vb - kb == 768
    assert a.offset("DP") >= a.model_range[1]          # DP group after the model group
    assert all(a.offset(n) % 64 == 0 for n in a.offsets)


def test_load_state_dict_keeps_arena_binding():
    from eegfusion.modules import PriGumbelModel
    m = PriGumbelModel(1.0, contract="W")
    sd = {k: torch.full_like(v, 0.25) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert float(m.arena.master[m.arena.offset("classifier.weight")]) == 0.25
    assert m.classifier.weight.data_ptr() == m.arena.view("classifier.weight").data_ptr()


def test_host_path_scope():
    """the host path (configs[0] plumbing) covers the "ti" models only; the other pairings and DP-SGD
    say they need the GPU instead of computing something else"""
    from eegfusion.modules import TTCA_LapDropout
    m = TTCA_LapDropout("bert-base-uncased")
    ids = torch.ones(1, 8, dtype=torch.long)
    with pytest.raises(NotImplementedError, match="GPU"):
        m(ids, ids, ids, ids, 1.0, True)


def test_half_conversion_refused():
    from eegfusion.modules import PriGumbelModel
    m = PriGumbelModel(1.0, contract="W")
    with pytest.raises(RuntimeError):
        m.half()


@pytest.mark.parametrize("modal,cls", [("ti", "TICA_LapDropout"), ("it", "ITCA_LapDropout"), ("ii", "IICA_LapDropout"),
                                       ("tt", "TTCA_LapDropout"), ("tisc", "TISC_LapDropout")])
def test_modal_variant_state_dict_keys(modal, cls):
    """custom_models/models.py variants: the parameter names / shapes are the reference modules' (read
    from the reference-generated fixture's gradient records, tests/golden/modal_variants.npz)."""
    import custom_models.models as M
    from goldens import load, modal_case
    _, fx = load("modal_variants")
    ref = {k.split(":", 1)[1] for k in modal_case(fx, modal) if k.startswith(("gsum:", "gnone:"))}
    m = getattr(M, cls)() if modal == "ii" else getattr(M, cls)("no-such-dir")
    assert set(m.state_dict()) == ref, set(m.state_dict()) ^ ref
    from oracle import fusion_oracle as O
    shapes = O.param_shapes("T", "prigumbel", modal=modal)
    assert {k: tuple(v.shape) for k, v in m.state_dict().items()} == shapes
