"""Debug: per-(row tile, k) errors of the fused column sums of eegf_gemm_acs."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "eeg-multimodal_amd"))
import torch
from eegfusion import _lib
M, N, K = (int(x) for x in sys.argv[1:4])
torch.manual_seed(13)
dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
c = torch.zeros(M, N, device="cuda").to(torch.bfloat16)
tiles = (M + 255) // 256
part = torch.full((tiles, K), float("nan"), device="cuda")
_lib.call("eegf_gemm_acs", 1, 1, 1, 0, _lib.EPI_NONE, M, N, K, dy.data_ptr(), K, w.data_ptr(), N, c.data_ptr(), N, None,
          None, 0, 1.0, 0.0, 1.0, part.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
pref = torch.nn.functional.pad(dy.double(), (0, 0, 0, tiles * 256 - M)).view(tiles, 256, K).sum(1)
err = (part.double() - pref).abs()
bad = (err > 1e-3 * pref.abs().max()).nonzero()
print("bad entries", bad.shape[0], "of", err.numel())
kk = bad[:, 1]
print("bad tiles", sorted(set(bad[:, 0].tolist())))
print("bad k mod 32 histogram", torch.bincount(kk % 32, minlength=32).tolist())
print("bad k//32 (K-tiles) first", sorted(set((kk // 32).tolist()))[:20], "count", len(set((kk // 32).tolist())))
t0 = bad[0, 0].item() if bad.shape[0] else 0
for k in range(0, 40):
    print(k, round(part[t0, k].item(), 3), round(pref[t0, k].item(), 3))
# which 32-row chunks (with what weight) make up the bad K-tile's sums (tile t0)?
kt = (bad[0, 1].item() // 32) if bad.shape[0] else 1
x = dy[t0 * 256:(t0 + 1) * 256, kt * 32:(kt + 1) * 32].double()
chunks = x.view(8, 32, 32).sum(1)                      # [8 chunks][32 k]
# also 8-row groups
g8 = x.view(32, 8, 32).sum(1)                          # [32 groups][32 k]
sol = torch.linalg.lstsq(g8.t().cpu(), part[t0, kt * 32:(kt + 1) * 32].double().cpu().unsqueeze(1)).solution.squeeze()
print("8-row group weights", [round(v, 2) for v in sol.tolist()])
# compare against the previous K-tile's data (stale image?)
for dk in (-1, 1, 3, 4, 5):
    k2 = kt + dk
    if 0 <= k2 < K // 32:
        y = dy[t0 * 256:(t0 + 1) * 256, k2 * 32:(k2 + 1) * 32].double().sum(0)
        print("dk", dk, "maxdiff", (part[t0, kt * 32:(kt + 1) * 32].double().cpu() - y.cpu()).abs().max().item())
