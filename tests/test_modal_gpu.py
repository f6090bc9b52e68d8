"""The custom_models/models.py modality variants on the HIP engine against the golden
vectors the reference itself produced (tests/golden/modal_variants.npz: TICA / ITCA / IICA / TTCA /
TISC_LapDropout, token ids [2, 128] with real lengths, CLIP-like vectors, injected Laplace / Gumbel
draws, dropout 0, CE mean).

Tolerances: fp32 logits and every recorded gradient within 1e-4 relative (north_star's fp32 bar);
bf16: finite logits and gradients, logits within 5e-2 of the fp32 engine.
"""
import pytest
import torch

from goldens import check_grads, det_params, load, modal_case, rel_err

pytestmark = pytest.mark.gpu

CLASSES = {"ti": "TICA_LapDropout", "it": "ITCA_LapDropout", "ii": "IICA_LapDropout", "tt": "TTCA_LapDropout",
           "tisc": "TISC_LapDropout"}


def _args(modal, fx, dev):
    g = lambda k: torch.from_numpy(fx[k]).to(dev)          # noqa: E731
    one = torch.ones(fx["labels"].shape[0], 1, dtype=torch.long, device=dev)
    if modal == "ti" or modal == "tisc":
        return (g("title_input"), g("text_mask"), g("frame_input"), one)
    if modal == "it":
        return (g("frame_input"), one, g("title_input"), g("text_mask"))
    if modal == "ii":
        return (g("frame_input"), one, g("frame_input2"), one)
    return (g("title_input"), g("text_mask"), g("title_input2"), g("text_mask2"))


def _run(modal, dtype=torch.float32):
    import custom_models.models as M
    cfg, fx_all = load("modal_variants")
    fx = modal_case(fx_all, modal)
    torch.manual_seed(0)
    cls = getattr(M, CLASSES[modal])
    m = cls(dropout=0.0) if modal == "ii" else cls("no-such-dir", dropout=0.0)
    m.load_state_dict(det_params("T", "prigumbel", requires_grad=False, modal=modal), strict=False)
    m = m.cuda().train()
    if dtype != torch.float32:
        m.set_compute_dtype(dtype)
    dev = "cuda"
    m.engine.injected = dict(noise=torch.from_numpy(fx["noise"]).to(dev),
                             gumbels=torch.from_numpy(fx["gumbels"]).to(dev).contiguous())
    logits = m(*_args(modal, fx, dev), cfg["eps"], cfg["hard"][modal])
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"]).to(dev))
    loss.backward()
    torch.cuda.synchronize()
    return m, logits.detach().cpu(), fx


@pytest.mark.parametrize("modal", list(CLASSES))
def test_modal_variant_golden_fp32(modal):
    m, logits, fx = _run(modal)
    assert rel_err(logits, fx["logits"]) < 1e-4, rel_err(logits, fx["logits"])
    check_grads({n: p.grad for n, p in m.named_parameters()}, fx, 1e-4)


@pytest.mark.parametrize("modal", ["it", "ii", "tt", "tisc"])
def test_modal_variant_bf16(modal):
    m, logits, fx = _run(modal, torch.bfloat16)
    assert torch.isfinite(logits).all()
    assert rel_err(logits, fx["logits"]) < 5e-2, rel_err(logits, fx["logits"])
    for n, p in m.named_parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all(), n
