"""Round-5 diagnosis, step 2: the classic learner's _TrunkChain and _ResStack nodes, kernel vs per-layer path.

Runs one classic (or det) loss forward + backward with the default switches while capturing every _TrunkChain /
_ResStack call's inputs and the gradient that reaches its output, then re-runs each captured node twice on the
same inputs and output gradient -- once through csrc/learner_chain.hip (CHAIN_KERNEL / RESBLOCK_STACK) and once
through the per-layer launches (both off) -- and logs, per output / input gradient, the largest relative
difference and the rows where it sits, plus the forward values of those rows.

usage: python profiles/r5_chain_vs_layers.py [det]
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
import r5_classic_grad_diag as D  # noqa: E402

CAPT = []


def wrap(cls, kind):
    orig = cls.apply

    def apply(*args):
        out = orig(*args)
        rec = dict(kind=kind, args=args, grads=None)
        o = out if isinstance(out, tuple) else (out,)

        def hook_for(i):
            def h(g):
                if rec["grads"] is None:
                    rec["grads"] = [None] * len(o)
                rec["grads"][i] = g.detach().clone()
            return h
        for i, t in enumerate(o):
            t.register_hook(hook_for(i))
        CAPT.append(rec)
        return out
    cls.apply = staticmethod(apply)
    return orig


def rerun(kind, orig, args, grads, kernel):
    """-> (outputs, input grads) of one node on the captured inputs, kernel path or per-layer path."""
    L.CHAIN_KERNEL = kernel
    with torch.enable_grad():
        if kind == "chain":
            lat, sc, sh, gs, apps, scaled, heads, *P = args
            lat, sc, sh = (t.detach().clone().requires_grad_(True) for t in (lat, sc, sh))
            P = [p.detach().clone().requires_grad_(True) for p in P]
            out = orig(lat, sc, sh, gs, apps, scaled, heads, *P)
            ins = [lat, sc, sh] + P
        else:
            x, owners, *P = args
            x = x.detach().clone().requires_grad_(True)
            P = [p.detach().clone().requires_grad_(True) for p in P]
            if kernel:
                out = orig(x, None, *P)
            else:         # the per-layer form of nb ResBlocks (_dense_ln_fwd pairs through autograd, RESBLOCK_NODE off)
                h = x
                for b in range(len(P) // 8):
                    Wa, ba, ga, bea, Wb, bb, gb, beb = P[8 * b:8 * b + 8]
                    ya = L._DenseLN.apply(h, Wa, ba, ga, bea, None, L.LN_RELU, None)
                    h = L._DenseLN.apply(ya, Wb, bb, gb, beb, h, L.LN_RESID_RELU, None)
                out = h
            ins = [x] + P
        o = out if isinstance(out, tuple) else (out,)
        gl = [(t, g) for t, g in zip(o, grads) if g is not None]
        dins = torch.autograd.grad([t for t, _ in gl], ins, [g for _, g in gl], allow_unused=True)
    return [t.detach() for t in o], dins


def rel(a, b):
    d = (a.double() - b.double()).abs()
    return float(d.max()) / max(float(b.double().abs().max()), 1e-30), d


def main():
    det = len(sys.argv) > 1 and sys.argv[1] == "det"
    params, C, batch, make = D.det_setup() if det else D.classic_setup()
    o_chain = wrap(L._TrunkChain, "chain")
    o_stack = wrap(L._ResStack, "stack")
    learner = make()
    learner.sink = None          # plain autograd gradients (GradSink is checked separately)
    learner.train_step(batch)
    torch.cuda.synchronize()
    L._TrunkChain.apply, L._ResStack.apply = staticmethod(o_chain), staticmethod(o_stack)
    for n, rec in enumerate(CAPT):
        kind, orig = rec["kind"], (o_chain if rec["kind"] == "chain" else o_stack)
        if rec["grads"] is None:
            print(f"node {n} ({kind}): no gradient reached it")
            continue
        ok, dk = rerun(kind, orig, rec["args"], rec["grads"], True)
        ol, dl = rerun(kind, orig, rec["args"], rec["grads"], False)
        L.CHAIN_KERNEL = True
        shape = tuple(ok[0].shape)
        e, d = rel(ok[0], ol[0])
        line = f"node {n} ({kind}, out {shape}): forward rel {e:.2e}"
        flat = d.reshape(-1, d.shape[-1]).amax(-1)
        worst = torch.topk(flat, min(4, flat.numel())).indices.tolist()
        line += f" worst rows {worst} ({', '.join(f'{float(flat[r]):.1e}' for r in worst)})"
        names = ["x"] if kind == "stack" else ["latent0", "scale", "shift"]
        errs = []
        for i, (a, b) in enumerate(zip(dk, dl)):
            if a is None or b is None:
                continue
            ee, dd = rel(a, b)
            nm = names[i] if i < len(names) else f"P{i - len(names)}"
            errs.append((ee, nm, dd))
        errs.sort(key=lambda t: -t[0])
        line += "; grads rel: " + ", ".join(f"{nm} {ee:.2e}" for ee, nm, _ in errs[:6])
        print(line, flush=True)
        ee, nm, dd = errs[0]
        if ee > 1e-5 and dd.dim() >= 2:
            rows = dd.reshape(-1, dd.shape[-1]).amax(-1)
            top = torch.topk(rows, min(6, rows.numel()))
            print(f"   worst grad {nm}: rows {top.indices.tolist()} |d| {[f'{v:.1e}' for v in top.values.tolist()]}; "
                  f"rows above 1e-3 x max: {int((rows > 1e-3 * float(rows.max() / max(ee, 1e-30))).sum())}", flush=True)


if __name__ == "__main__":
    main()
