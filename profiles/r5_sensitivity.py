"""Round-5 diagnosis, step 3: where is the classic learner's gradient sensitive to last-bit forward differences?

Takes the per-layer learner path (CHAIN_KERNEL, RESBLOCK_STACK, RESBLOCK_NODE off: within 1.6e-6 of the float64
oracle) and adds a relative perturbation of `eps` (default 3e-7, the kernels' measured forward difference) to ONE
forward tensor at a time -- value only, the gradient passes through unchanged -- then logs the gradient error
against the float64 restatement.  A site whose perturbation moves the error from ~1e-6 to ~1e-4 is downstream of a
discontinuity (a ReLU / argmax decision within eps of its threshold).

usage: python profiles/r5_sensitivity.py [det] [eps]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "profiles"))
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from oracle import learner_grad as OG  # noqa: E402
import r5_classic_grad_diag as D  # noqa: E402

SITE = {"name": None, "seed": 0, "eps": 3e-7}


def perturb(t, tag):
    """t + eps * |t| * noise (a constant: the gradient is unchanged) when `tag` is the active site."""
    name = SITE["name"]
    if name is None or not tag.startswith(name):
        return t
    g = torch.Generator(device=t.device).manual_seed(SITE["seed"] * 1000 + len(tag))
    noise = torch.randn(t.shape, generator=g, device=t.device, dtype=t.dtype)
    return t + (t.detach().abs() * SITE["eps"] * noise)


def install(classic):
    oc = L._TrunkChain.apply

    def chain(*args):
        out = oc(*args)
        if isinstance(out, tuple):
            return tuple(perturb(o, f"chain/{i}") for i, o in enumerate(out))
        if classic:   # rows interleaved: act_0 (afterstate), chance_0 (state), ...
            ev = perturb(out[0::2], "chain/after")
            od = perturb(out[1::2], "chain/state")
            return torch.stack([ev, od], 1).reshape(out.shape)
        return perturb(out, "chain/state")
    L._TrunkChain.apply = staticmethod(chain)
    odm = L._DenseMinmax.apply
    L._DenseMinmax.apply = staticmethod(lambda *a: perturb(odm(*a), "repr/latent"))
    od = L._DenseLN.apply
    L._DenseLN.apply = staticmethod(lambda *a: perturb(od(*a), "denseln"))
    orr = L._ResBlockLN.apply
    L._ResBlockLN.apply = staticmethod(lambda *a: perturb(orr(*a), "resblock"))
    ode = L._Dense.apply
    L._Dense.apply = staticmethod(lambda *a: perturb(ode(*a), "dense"))


def main():
    det = "det" in sys.argv[1:]
    for a in sys.argv[1:]:
        try:
            SITE["eps"] = float(a)
        except ValueError:
            pass
    params, C, batch, make = D.det_setup() if det else D.classic_setup()
    b = {k: v.detach().cpu().numpy() for k, v in batch.items()}
    _, _, ref = OG.loss_and_grads(params, b, unroll_steps=10, classic=not det)
    for s in ("CHAIN_KERNEL", "RESBLOCK_STACK", "RESBLOCK_NODE"):
        setattr(L, s, False)
    install(not det)
    sites = [None, "chain/after", "chain/state", "chain", "repr/latent", "denseln", "resblock", "dense"]
    for name in sites:
        for seed in ((0,) if name is None else (1, 2)):
            SITE["name"], SITE["seed"] = name, seed
            learner = make()
            learner.train_step(batch)
            torch.cuda.synchronize()
            g = {k: p.grad.detach().double().cpu().numpy() for k, p in learner.nets.p.items()}
            e = {k: float(np.linalg.norm(g[k] - ref[k])) / max(float(np.linalg.norm(ref[k])), 1e-12) for k in ref}
            worst = sorted(e, key=lambda k: -e[k])[:3]
            print(f"[{'none' if name is None else name} eps {SITE['eps']:.0e} seed {seed}] Frobenius worst: " +
                  ", ".join(f"{k} {e[k]:.2e}" for k in worst), flush=True)
            del learner


if __name__ == "__main__":
    main()
