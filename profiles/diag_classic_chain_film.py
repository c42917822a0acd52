"""Diagnosis: the classic chain node vs the per-step graph with the fused LayerNorm_0 + FiLM kernels on / off
(learner.FUSED_FILM): per-input max relative gradient difference, and whether the chain outputs differ."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from exploring_muzero_on_dog_amd import stochastic as ST  # noqa: E402

C, B, K = 20, 64, 5
params = ST.init_classic_params(C, seed=6)
rng = np.random.default_rng(8)
params = {k: (v + 0.1 * rng.standard_normal(v.shape).astype(np.float32)) if not k.endswith("kernel") else v
          for k, v in params.items()}
nets = L.ClassicMuZeroNets(params, C, "cuda")
g = torch.Generator().manual_seed(5)
lat0 = torch.rand(B, 256, generator=g).cuda().requires_grad_(True)
ea = torch.relu(torch.randn(K * B, 64, generator=g)).cuda().requires_grad_(True)
ec = torch.relu(torch.randn(K * B, 64, generator=g)).cuda().requires_grad_(True)
w = torch.randn(2 * K, B, 256, generator=g).cuda()
names = [n for kind in ("act", "chance") for n in L.trunk_param_names(kind)]
names += [f"dynamics/{pre}_film_{x}/{y}" for pre in ("act", "chance") for x in ("scale", "shift") for y in ("kernel", "bias")]
inputs = [lat0, ea, ec] + [nets.p[n] for n in names]
film = [torch.stack([nets._dense(f"dynamics/{pre}_film_{x}", e).reshape(K, B, -1)
                     for pre, e in (("act", ea), ("chance", ec))], 1).reshape(2 * K, B, -1) for x in ("scale", "shift")]
seq, lat = [], lat0
for k in range(K):
    after = nets._film_trunk("act", 0, lat, None, film=(film[0][2 * k], film[1][2 * k]))
    nxt = nets._film_trunk("chance", 2, after, None, film=(film[0][2 * k + 1], film[1][2 * k + 1]))
    lat = (nxt * 0.5).detach() + nxt * 0.5
    seq += [after, lat]
ref = torch.stack(seq)
g2 = torch.autograd.grad((ref * w).sum() + ref[-1].square().sum(), inputs, retain_graph=True)
outs = {}
for fused in (True, False):
    L.FUSED_FILM = fused
    out = L._TrunkChain.apply(lat0, film[0], film[1], 0.5, (0, 1) * K, (False, True) * K, False,
                              *(nets.p[n] for n in names[:2 * L._NP]))
    g1 = torch.autograd.grad((out * w).sum() + out[-1].square().sum(), inputs, retain_graph=True)
    torch.cuda.synchronize()
    outs[fused] = (out.detach().clone(), [x.clone() for x in g1])
    errs = [((a - b).abs().max().item() / max(1e-3, b.abs().max().item()), n)
            for n, a, b in zip(["latent0", "act_embed", "chance_embed"] + names, g1, g2)]
    print(f"FUSED_FILM={fused}: forward max |d| {(out - ref).abs().max().item():.3e}; worst gradients:",
          sorted(errs, reverse=True)[:4], flush=True)
o1, o0 = outs[True], outs[False]
print("fused vs unfused: forward identical", torch.equal(o1[0], o0[0]), "max |d|", (o1[0] - o0[0]).abs().max().item())
print("fused vs unfused gradients max |d|:", max((a - b).abs().max().item() for a, b in zip(o1[1], o0[1])))
