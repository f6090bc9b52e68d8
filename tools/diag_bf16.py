"""Per-parameter gradient agreement of the engine (fp32 and bf16) with the CPU oracle."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "eeg-multimodal_amd"), str(ROOT), str(ROOT / "tests")]
import torch
from goldens import det_params, w_values_dp
from oracle import fusion_oracle as O
from eegfusion.modules import PriGumbelModel

torch.manual_seed(5)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
eeg = torch.randn(B, 64, 256); act = torch.randn(B, 32) * 0.5
labels = torch.tensor([0, 1, 1, 0] * (B // 4))
noise = O.laplace_from_uniform(torch.rand(B, 2304) * 2 - 1)
gumbels = -torch.log(-torch.log(torch.rand(2, B, 2304).clamp(1e-6, 1 - 1e-6)))
dp = w_values_dp()
p = det_params("W", "prigumbel", dp)
ref = O.forward(p, dict(eeg=eeg, act=act), O.PathConfig(contract="W", variant="prigumbel", hard=False), noise=noise, gumbels=gumbels)
O.cal_loss(ref, labels)[0].backward()
for dt in (torch.float32, torch.bfloat16):
    torch.manual_seed(0)
    m = PriGumbelModel(1.0, contract="W", dropout=0.0)
    m.load_state_dict({k: v.detach() for k, v in p.items()}, strict=False)
    m = m.cuda().train().set_compute_dtype(dt)
    m.engine.injected = dict(noise=noise.cuda(), gumbels=gumbels.cuda().contiguous())
    logits = m.forward_window(eeg.cuda(), act.cuda(), False)
    torch.nn.functional.cross_entropy(logits, labels.cuda()).backward()
    torch.cuda.synchronize()
    print(dt, "logits rel", ((logits.cpu() - ref.detach()).abs().max() / ref.abs().max()).item())
    rows = []
    for n, t in m.named_parameters():
        if n not in p or p[n].grad is None or t.grad is None:
            continue
        a, b = t.grad.double().cpu().reshape(-1), p[n].grad.double().reshape(-1)
        if b.norm() == 0 or b.norm() < 1e-6 * max(1.0, a.norm().item()):
            continue
        rows.append(((a @ b / (a.norm() * b.norm() + 1e-30)).item(), (a.norm() / b.norm()).item(), n))
    rows.sort()
    for r in rows[:12]:
        print(f"  cos {r[0]:.4f} normratio {r[1]:.4f} {r[2]}")
