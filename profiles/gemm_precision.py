"""Diagnostic: fp32 GEMM accuracy of the learner's BLAS path on the GPU (rocBLAS, as learner.prefer_rocblas
selects) against float64, at the learner's weight-gradient shape (X^T dZ, 1408 x 256 each)."""
import torch

torch.backends.cuda.preferred_blas_library("cublas")
g = torch.Generator().manual_seed(0)
for M, K, N, tag in ((256, 1408, 256, "weight grad X^T dZ"), (1408, 256, 256, "forward X W")):
    a = torch.randn(M, K, generator=g, dtype=torch.float64)
    b = torch.randn(K, N, generator=g, dtype=torch.float64)
    ref = a @ b
    for name, fn in (("gpu fp32", lambda: (a.float().cuda() @ b.float().cuda()).double().cpu()),
                     ("cpu fp32", lambda: (a.float() @ b.float()).double())):
        out = fn()
        err = ((out - ref).norm() / ref.norm()).item()
        print(f"{tag} [{M}x{K}]x[{K}x{N}] {name}: Frobenius rel err {err:.2e}, max {((out - ref).abs().max() / ref.abs().max()).item():.2e}")
print("allow_tf32:", torch.backends.cuda.matmul.allow_tf32, "fp32 precision:", torch.get_float32_matmul_precision())
