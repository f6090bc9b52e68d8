"""The optimized PriGumbel iteration (pass 1: encoders forward only, backward through the head and
privacy stage for the DP gradient) leaves exactly the same parameters as the reference loop
(past_acc.py:194-212: full backward in both passes, two Adam optimizers), checked on the CPU oracle
against the reference's own one-iteration deltas (tests/golden/two_optimizer_step.npz)."""
import numpy as np
import torch

from goldens import det_params, load, w_values_dp
from oracle import fusion_oracle as O


def _iteration(p, fx, optimized):
    B = fx["eeg"].shape[0]
    batch = dict(eeg=torch.from_numpy(fx["eeg"]), act=torch.from_numpy(fx["act"]))
    labels = torch.from_numpy(fx["labels"])
    dp = [p["DP"]]
    model = [v for k, v in p.items() if k != "DP"]
    mopt, dopt = torch.optim.Adam(model, lr=1e-6), torch.optim.Adam(dp, lr=1e-6)
    dopt.zero_grad()
    n1, g1 = torch.from_numpy(fx["noise1"]), torch.from_numpy(fx["gumbels1"])
    if optimized:
        with torch.no_grad():
            pooled, img, cross = O.encoders(p, batch, O.PathConfig(contract="W"))
        f = O.minmax(torch.cat((pooled, img, cross), 1))
        logits = O.head(p, O.prigumbel_gate(f, p["DP"], n1, g1, 1.0, "newfrac", False))
    else:
        logits = O.forward(p, batch, O.PathConfig(contract="W", hard=False), noise=n1, gumbels=g1)
    O.cal_loss(logits, labels)[0].backward()
    dopt.step()
    mopt.zero_grad()
    n2, g2 = torch.from_numpy(fx["noise2"]), torch.from_numpy(fx["gumbels2"])
    logits = O.forward(p, batch, O.PathConfig(contract="W", hard=True), noise=n2, gumbels=g2)
    O.cal_loss(logits, labels)[0].backward()
    mopt.step()


def test_optimized_schedule_matches_reference_deltas():
    cfg, fx = load("two_optimizer_step")
    p = det_params("W", "prigumbel", w_values_dp())
    before = {k: v.detach().clone() for k, v in p.items()}
    _iteration(p, fx, optimized=True)
    for key in fx:
        if not key.startswith("delta:"):
            continue
        n = key.split(":", 1)[1]
        d = ((p[n].detach() - before[n]) / cfg["lr"]).reshape(-1).numpy()
        ref = fx[key]
        big = np.abs(ref) > 0.05            # Adam step 1: delta/lr = -g/(|g|+eps) ~ -sign(g)
        assert np.abs(d[big] - ref[big]).max() < 2e-3, n
