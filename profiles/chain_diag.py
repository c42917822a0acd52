"""Chain kernel (learner.CHAIN_KERNEL) against the per-layer path: per-application differences of the outputs,
the min-max extremum columns (where out == 0 / 1) and the FiLM gradients -- to locate a disagreement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from oracle import nets as ON  # noqa: E402

B, K = int(sys.argv[1]) if len(sys.argv) > 1 else 128, int(sys.argv[2]) if len(sys.argv) > 2 else 10
g = torch.Generator().manual_seed(43 + B)
nets = L.MuZeroNets(ON.init_params(18, seed=4, randomize_affine=True), 18, 24, "cuda")
names, apps, scaled, heads, T = list(L.DYN_TRUNK_PARAMS), (0,) * K, (True,) * K, True, K
lat0 = torch.rand(B, 256, generator=g).cuda().requires_grad_(True)
scale = (0.3 * torch.randn(T, B, 256, generator=g)).cuda().requires_grad_(True)
shift = (0.3 * torch.randn(T, B, 256, generator=g)).cuda().requires_grad_(True)
w, wh = (torch.randn(T, B, 256, generator=g).cuda() for _ in range(2))
params = [nets.p[n] for n in names]
inputs = [lat0, scale, shift] + params
res = []
for chain in (True, False):
    L.CHAIN_KERNEL = chain
    o = L._TrunkChain.apply(lat0, scale, shift, 0.5, apps, scaled, heads, *params)
    out, raw = o
    loss = (out * w).sum() + out[-1].square().sum() + (raw * wh).sum()
    res.append((out.detach().clone(), torch.autograd.grad(loss, inputs)))
L.CHAIN_KERNEL = True
torch.cuda.synchronize()
(o1, g1), (o2, g2) = res
for i in range(T):
    z1, z2 = (o1[i] == 0), (o2[i] == 0)
    e1, e2 = (o1[i] == 1), (o2[i] == 1)
    ds = (g1[1][i] - g2[1][i]).abs()
    dh = (g1[2][i] - g2[2][i]).abs()
    bad = ds.amax(1)
    r = int(bad.argmax())
    print(f"app {i}: out diff {(o1[i] - o2[i]).abs().max().item():.2e}, min cols differ in {int((z1 != z2).any(1).sum())} rows, "
          f"max cols in {int((e1 != e2).any(1).sum())} rows; dscale diff {ds.max().item():.2e} (of {g2[1][i].abs().max().item():.2e}, "
          f"worst row {r}: {bad[r].item():.2e}, rows > 1e-4: {int((bad > 1e-4).sum())}), dshift diff {dh.max().item():.2e}")
for n, a, b in zip(["latent0", "scale", "shift"] + names, g1, g2):
    err = (a - b).abs().max().item() / max(1e-3, b.abs().max().item())
    print(f"{n}: {err:.2e}")
