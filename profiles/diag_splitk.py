"""Is the batched split-K GEMM (learner._dense_ln_fwd, MUZ_SPLITK_DENSE) deterministic?  torch.bmm of the
representation Dense_0 shape repeated and at shifted input addresses, compared bit for bit; then two fresh classic /
det learners' gradients on the same batch (run to run)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

g = torch.Generator().manual_seed(0)
M, K, N, S = 128, 3584, 256, 14
x = torch.randn(M, K, generator=g).cuda()
W = (torch.randn(K, N, generator=g) * 0.02).cuda()
ref = torch.bmm(x.view(M, S, K // S).transpose(0, 1), W.view(S, K // S, N))
same = all(torch.equal(ref, torch.bmm(x.view(M, S, K // S).transpose(0, 1), W.view(S, K // S, N))) for _ in range(5))
big = torch.empty(M * K + 64, device="cuda")
shifted = []
for off in (1, 4, 16, 33):
    xs = big[off:off + M * K].view(M, K)
    xs.copy_(x)
    shifted.append(torch.equal(ref, torch.bmm(xs.view(M, S, K // S).transpose(0, 1), W.view(S, K // S, N))))
print(f"bmm [{S}, {M}, {K // S}] x [{S}, {K // S}, {N}]: repeat bit-identical {same}; shifted inputs bit-identical "
      f"{shifted}; vs one GEMM max rel {float((ref.sum(0) - x @ W).abs().max() / (x @ W).abs().max()):.2e}", flush=True)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_learner_oracle as T  # noqa: E402

for classic in (False, True):
    params, batch, make = T._classic_setup() if classic else T._det_setup()
    grads = []
    for _ in range(2):
        lr = make()
        lr.train_step(batch)
        torch.cuda.synchronize()
        grads.append(T._grads(lr))
    diff = [k for k in grads[0] if not np.array_equal(grads[0][k], grads[1][k])]
    print(f"{'classic' if classic else 'det'}: two fresh learners, same batch: {len(diff)} of {len(grads[0])} gradients "
          f"differ bitwise {diff[:5]}", flush=True)
