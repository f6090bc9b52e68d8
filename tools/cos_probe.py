"""bf16-vs-fp32 engine agreement of the attention Q/K/V weight gradients (tests/test_production_gpu.py
test_full_size_bf16_vs_fp32_engine) for several dropout rates and rng bases: tells a numerical
regression from a change of dropout realization.  Usage: python tools/cos_probe.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "eeg-multimodal_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

DEV = "cuda"


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(a @ b / (a.norm() * b.norm() + 1e-300))


def run(m, eeg, act, labels, rng0):
    m.engine.rng_counter = rng0
    for q in m.parameters():
        q.grad = None
    logits = m.forward_window(eeg, act, True)
    torch.nn.functional.cross_entropy(logits, labels).backward()
    torch.cuda.synchronize()
    names = [f"bert.encoder.layer.{i}.attention.self.{k}.weight" for i in range(12) for k in ("query", "key", "value")]
    g = dict(m.named_parameters())
    return {n: g[n].grad.detach().clone() for n in names}


def main():
    from eegfusion.modules import PriGumbelModel
    B = 256
    ps = [float(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0.0, 0.1]
    rngs = [int(x) << 20 for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1 << 20, 5 << 20]
    for p in ps:
        for rng0 in rngs:
            torch.manual_seed(2)
            m = PriGumbelModel(1.0, contract="W", eps_mode="newfrac", dropout=p, seed=980616).cuda().train()
            g = torch.Generator(device=DEV).manual_seed(B)
            eeg = torch.randn(B, 64, 256, generator=g, device=DEV)
            act = torch.randn(B, 32, generator=g, device=DEV) * 0.5
            labels = (torch.rand(B, generator=g, device=DEV) < 0.66).long()
            m.set_compute_dtype(torch.bfloat16)
            gb = run(m, eeg, act, labels, rng0)
            m.set_compute_dtype(torch.float32)
            gf = run(m, eeg, act, labels, rng0)
            cos = sorted((_cos(gb[n], gf[n]), n.split(".")[3] + "." + n.split(".")[6]) for n in gb)
            print(f"p={p} rng0={rng0}: worst {[(round(c, 5), n) for c, n in cos[:3]]}", flush=True)


if __name__ == "__main__":
    main()
