"""Which hipBLASLt kernels torch picks for the step's GEMM shapes (run under rocprofv3 --kernel-trace)."""
import torch
R = 65536
dt = torch.bfloat16
for (M, N, K) in [(R, 3072, 768), (R, 768, 3072), (R, 2304, 768), (R, 3072, 3072), (R, 768, 768)]:
    A = torch.randn(M, K, device="cuda", dtype=dt)
    B = torch.randn(N, K, device="cuda", dtype=dt)
    bias = torch.randn(N, device="cuda", dtype=dt)
    for _ in range(3):
        torch.nn.functional.linear(A, B, bias)
        torch.nn.functional.linear(A, B)
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
