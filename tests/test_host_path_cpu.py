"""The host path (eegfusion/cpu_path.py: a model kept in host memory, configs[0]'s "CPU PyTorch via
train.py (plumbing, no GPU)") against the golden vectors the reference produced: logits within 1e-5
relative and every recorded gradient within 1e-4 (fp32 CPU vs fp32 CPU: summation order, SDPA vs the
reference's attention), and train.py -bs 32 end to end on the CPU with its first step checked
against the c1_batch32 fixture.  Also: the host path never serves device operands."""
import numpy as np
import pytest
import torch

from c1_split import write_c1_split
from goldens import check_grads, det_params, load, rel_err, w_values_dp


def _nodrop(m):
    c = m.engine.cfg
    c.hidden_dropout = c.attn_dropout = c.dec_dropout = 0.0
    return m


def test_concat_tokens_host():
    import model as drop_in
    _, fx = load("full_concat_tokens")
    m = _nodrop(drop_in.ConcatModel())
    m.load_state_dict(det_params("T", "concat", requires_grad=False), strict=False)
    m.train()
    x = tuple(torch.from_numpy(fx[k]) for k in ("frame_input", "vedio_mask", "title_input", "text_mask"))
    logits = m(x, hard=True)
    torch.nn.CrossEntropyLoss(reduction="none")(logits, torch.from_numpy(fx["labels"])).sum().backward()
    assert rel_err(logits.detach(), fx["logits"]) < 1e-5
    check_grads({n: q.grad for n, q in m.named_parameters()}, fx, 1e-4)
    assert m.arena.device.type == "cpu"


@pytest.mark.parametrize("name", ["full_prigumbel_soft", "full_prigumbel_hard_wvalues"])
def test_prigumbel_window_host(name):
    from eegfusion.modules import PriGumbelModel
    cfg, fx = load(name)
    dp = w_values_dp() if cfg["dp"] == "w_values" else None
    m = PriGumbelModel(cfg["eps"], contract="W", dropout=0.0)
    m.load_state_dict(det_params("W", "prigumbel", dp, requires_grad=False), strict=False)
    m.train()
    m.engine.injected = dict(noise=torch.from_numpy(fx["noise"]), gumbels=torch.from_numpy(fx["gumbels"]))
    logits = m.forward_window(torch.from_numpy(fx["eeg"]), torch.from_numpy(fx["act"]), cfg["hard"])
    torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"])).backward()
    assert rel_err(logits.detach(), fx["logits"]) < 1e-5
    check_grads({n: q.grad for n, q in m.named_parameters()}, fx, 1e-4)


def test_priconcat_lap_host():
    import types
    from eegfusion.modules import PriConcatModel
    cfg, fx = load("full_priconcat_lap")
    m = PriConcatModel(types.SimpleNamespace(EPSILON=1.0), dp_mode="feature_all_lap", honor_dp_mode=True,
                       contract="W", dropout=0.0)
    m.load_state_dict(det_params("W", "priconcat", requires_grad=False), strict=False)
    m.train()
    m.engine.injected = dict(row_noise=torch.from_numpy(fx["row_noise"]))
    logits = m.forward_window(torch.from_numpy(fx["eeg"]), torch.from_numpy(fx["act"]), True)
    torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"])).backward()
    assert rel_err(logits.detach(), fx["logits"]) < 1e-5
    check_grads({n: q.grad for n, q in m.named_parameters()}, fx, 1e-4)


def test_train_py_bs32_on_cpu(tmp_path, monkeypatch):
    """configs[0]: train.py -bs 32 over a 64-sample split in the reference's formats, on the CPU, one
    epoch; the first training step's logits / CE sum equal the reference's for the samples it drew."""
    import train
    feat = tmp_path / "feature"
    fx = write_c1_split(feat, "train")
    write_c1_split(feat, "test")
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(train, "DEVICE", torch.device("cpu"))
    seen = []

    def get_model(cfg):
        import model as drop_in
        m = _nodrop(drop_in.ConcatModel())
        m.load_state_dict(det_params("T", "concat", requires_grad=False), strict=False)
        m.eps = torch.tensor(cfg.eps)
        fwd = m.forward

        def capture(x, hard=True):
            out = fwd(x, hard)
            if m.training and not seen:
                seen.append((x[0].detach().clone(), out.detach().clone()))
            return out
        m.forward = capture
        return m

    monkeypatch.setattr(train, "get_model", get_model)
    train.set_seed(980616)
    res = train.main(train.parse_args(["-bs", "32", "-n", "1", "-ne", "1", "--exp", "c1cpu"]))
    frames, logits = seen[0]
    ref_frames = torch.from_numpy(fx["frame_input"])
    idx = [int(torch.nonzero((ref_frames == f).all(-1).all(-1)).view(-1)[0]) for f in frames]
    assert len(set(idx)) == 32
    assert rel_err(logits, fx["logits_all"][idx]) < 1e-5
    ref = float(fx["ce_all"][idx].astype(np.float64).sum())
    assert abs(float(res["train_loss"][0].sum()) - ref) < 1e-5 * abs(ref)
    assert len(res["train_loss"]) == 2 and not res["labels"].is_cuda
    assert (tmp_path / "experiment" / "c1cpu" / "test" / "results.pth").exists()


def test_host_model_refuses_device_inputs():
    from eegfusion.modules import ConcatModel
    m = ConcatModel(contract="W", dropout=0.0)
    fake = torch.empty(0)
    with pytest.raises(RuntimeError):
        m._host(type("T", (), {"is_cuda": True})(), fake)


def test_host_model_refused_when_a_gpu_is_present(monkeypatch):
    """A model left in host memory on a GPU machine is a forgotten .cuda(): refused with a pointer to it,
    unless the model asks for the host path explicitly (host_path=True, or EEGF_HOST_PATH=1)."""
    from eegfusion.modules import ConcatModel
    m = ConcatModel(contract="W", dropout=0.0)
    x = torch.empty(0)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.delenv("EEGF_HOST_PATH", raising=False)
    with pytest.raises(RuntimeError, match="model.cuda"):
        m._host(x)
    monkeypatch.setenv("EEGF_HOST_PATH", "1")
    assert m._host(x)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    monkeypatch.delenv("EEGF_HOST_PATH")
    assert m._host(x)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    assert ConcatModel(contract="W", dropout=0.0, host_path=True)._host(x)


def test_host_tokens_cut_only_without_dropout(monkeypatch):
    """Right-padded token batches are cut to their longest real sequence only when no dropout is drawn
    (eval, or p = 0): in training with dropout the padded tensors keep the reference's RNG consumption."""
    from eegfusion import cpu_path
    import model as drop_in
    m = drop_in.ConcatModel()
    B, Lp = 2, 512
    ids = torch.zeros(B, Lp, dtype=torch.long)
    mask = torch.zeros(B, Lp, dtype=torch.long)
    mask[:, :40] = 1
    seen = []
    real_embedding = torch.nn.functional.embedding

    def spy(i, w, *a, **k):
        seen.append(i.shape[1])
        return real_embedding(i, w, *a, **k)
    monkeypatch.setattr(cpu_path.F, "embedding", spy)
    batch = {"title_input": ids, "text_mask": mask}
    with torch.no_grad():
        cpu_path._bert(m, m.engine.cfg, batch, training=False)
        cpu_path._bert(m, m.engine.cfg, batch, training=True)
    assert seen == [40, Lp]
