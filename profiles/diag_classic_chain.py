"""Diagnostic: tests/test_gpu_learner.py::test_classic_chain_node_matches_per_step_autograd with the fused
dense kernels on / off (which input's gradient moves, and by how much)."""
import sys

sys.path.insert(0, ".")
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from exploring_muzero_on_dog_amd import stochastic as ST  # noqa: E402

L.prefer_rocblas()
for fused in (False, True):
    L.FUSED_DENSE = fused
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
    names += [f"dynamics/{pre}_film_{x}/{y}" for pre in ("act", "chance") for x in ("scale", "shift")
              for y in ("kernel", "bias")]
    inputs = [lat0, ea, ec] + [nets.p[n] for n in names]
    film = [torch.stack([nets._dense(f"dynamics/{pre}_film_{x}", e).reshape(K, B, -1)
                         for pre, e in (("act", ea), ("chance", ec))], 1).reshape(2 * K, B, -1) for x in ("scale", "shift")]
    out = L._TrunkChain.apply(lat0, film[0], film[1], 0.5, (0, 1) * K, (False, True) * K, False,
                              *(nets.p[n] for n in names[:2 * L._NP]))
    g1 = torch.autograd.grad((out * w).sum() + out[-1].square().sum(), inputs, retain_graph=True)
    seq, lat = [], lat0
    for k in range(K):
        if "--shared-film" in sys.argv:
            after = nets._film_trunk("act", 0, lat, None, film=(film[0][2 * k], film[1][2 * k]))
            nxt = nets._film_trunk("chance", 2, after, None, film=(film[0][2 * k + 1], film[1][2 * k + 1]))
        else:
            after = nets._film_trunk("act", 0, lat, ea[k * B:(k + 1) * B])
            nxt = nets._film_trunk("chance", 2, after, ec[k * B:(k + 1) * B])
        lat = (nxt * 0.5).detach() + nxt * 0.5
        seq += [after, lat]
    ref = torch.stack(seq)
    g2 = torch.autograd.grad((ref * w).sum() + ref[-1].square().sum(), inputs)
    torch.cuda.synchronize()
    print(f"fused={fused}: forward max diff {(out - ref).abs().max().item():.3e}; per-step rows with range < 1e-3: "
          f"{int(((ref.amax(-1) - ref.amin(-1)) < 1e-3).sum())}")
    errs = sorted(((a - b).abs().max().item() / max(1e-3, b.abs().max().item()), n)
                  for n, a, b in zip(["latent0", "act_embed", "chance_embed"] + names, g1, g2))[::-1]
    print("  worst:", ", ".join(f"{n} {e:.2e}" for e, n in errs[:6]))
