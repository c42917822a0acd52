"""Strict search / self-play parity checks shared by the GPU tests.

The GPU side and the oracle side see identical network outputs in these tests (the oracle calls the GPU's
own root / recurrent kernels), so only the tree arithmetic's summation order differs.  The bar:

  * every game agrees on the action, its root value within TOL (the north star's 1e-5 fp32) and its action
    weights within TOL + DQ x gain, where `gain` (from the oracle) is the Q-rescale gain of the final
    weights: they are a softmax over logits + visit_scale x value_scale x (q - lo) / (hi - lo), so q's
    last-ulp differences (DQ = 4 fp32 ulps at 1) reach the weights multiplied by
    K = visit_scale x value_scale / (hi - lo) (oracle/mctx_gumbel.py);
  * the only excuse for a differing action is a near-tie the oracle itself recorded for that search:
    `margin`, the smallest top-2 gap over all of the search's argmax decisions divided by that decision's
    rounding bound (1e-5 relative + DQ x the decision's own gain), <= TIE = 1.  How many games needed the
    excuse is logged (so far: none);
  * self-play: every game's record is identical up to its first differing turn (exact integers, floats as
    above), that turn must be an oracle-recorded near-tie, and without one the whole record is identical.

Each check appends one line to gpurun_out/parity.log (copied into profiles/ as the tracked record)."""
import os

import numpy as np

TIE = 1.0
TOL = 1e-5
DQ = 4.8e-7
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def log(line):
    print(line)
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "parity.log"), "a") as f:
        f.write(line + "\n")


def search_parity(label, ga, gw, grv, a, w, orv, margin, gain=None, tol=TOL, tie=TIE):
    """One batched search: GPU (ga, gw, grv) vs oracle (a, w, orv) with the oracle's per-game margins and
    final-weights gains (None: the weights carry no rescale, e.g. visit fractions)."""
    B = len(a)
    tied = np.asarray(margin) <= tie
    agree = np.asarray(ga) == np.asarray(a)
    dw = np.abs(np.asarray(gw) - np.asarray(w)).max(-1)
    dv = np.abs(np.asarray(grv) - np.asarray(orv))
    g = np.zeros(B) if gain is None else np.asarray(gain)
    wtol = tol + DQ * g
    over = agree & (dw > tol)      # beyond the literal 1e-5: only the Q-rescale allowance admits these
    log(f"{label}: B={B} action agreement {agree.mean():.4f} ({int(agree.sum())}/{B}), differing games excused "
        f"as oracle near-ties {int((~agree).sum())}; agreeing games: max|dw| {dw[agree].max():.2e} "
        f"(max |dw| / its bound {(dw / wtol)[agree].max():.3f}), max|dv| {dv[agree].max():.2e}; "
        f"|dw| > {tol:g} in {int(over.sum())} games (largest gain among them "
        f"{(g[over].max() if over.any() else 0.0):.3g}); bit-identical weights in {int((dw[agree] == 0).sum())}")
    bad = np.flatnonzero(~agree & ~tied)
    assert bad.size == 0, f"{label}: games {bad[:8]} chose differently without a near-tie (margins {np.asarray(margin)[bad[:8]]})"
    assert (dw[agree] <= wtol[agree]).all(), f"{label}: action_weights differ beyond tol + DQ x gain"
    assert dv[agree].max() <= tol, f"{label}: root value differs by {dv[agree].max():.2e} > {tol}"
    return agree.mean()


def selfplay_parity(label, buf, ref, exact_keys, float_keys=("val", "pol"), tol=TOL, tie=TIE):
    """Trajectory buffers of the GPU engine (buf) vs the oracle loop (ref, with ref['margin'] / ref['gain']
    [n, T] recorded per MCTS turn)."""
    n = len(ref["idx"])
    diverged, max_d = [], 0.0
    over, over_gain, turns, exact = 0, 0.0, 0, 0   # turns with a float beyond the literal 1e-5 / bit-identical
    for i in range(n):
        L, Lg = int(ref["idx"][i]), int(buf["idx"][i])
        m = min(L, Lg)
        diff = np.flatnonzero(buf["act"][i, :m] != ref["act"][i, :m])
        t_star = int(diff[0]) if diff.size else (m if L != Lg else L)
        if t_star < L:
            assert ref["margin"][i, t_star] <= tie, \
                f"{label}: game {i} diverges at turn {t_star} without a near-tie (margin {ref['margin'][i, t_star]:.3e})"
            diverged.append((i, t_star))
        for k in exact_keys:
            assert np.array_equal(buf[k][i, :t_star], ref[k][i, :t_star]), (label, k, i)
        for k in float_keys:
            d = np.abs(buf[k][i, :t_star] - ref[k][i, :t_star])
            d = d.reshape(t_star, -1).max(-1) if t_star else d
            # the policy target carries the final Q-rescale gain, the root value does not
            bound = tol + (DQ * ref["gain"][i, :t_star] if k == "pol" and "gain" in ref else 0.0)
            if t_star:
                max_d = max(max_d, float(d.max()))
                if k == "pol":
                    o = d > tol
                    over += int(o.sum())
                    turns += t_star
                    exact += int((d == 0).sum())
                    if o.any() and "gain" in ref:
                        over_gain = max(over_gain, float(ref["gain"][i, :t_star][o].max()))
            assert (d <= bound).all(), f"{label}: game {i} {k} differs by {d.max():.2e} beyond its bound"
    log(f"{label}: {n - len(diverged)}/{n} games identical; diverged at oracle near-ties {diverged}; "
        f"max float |d| {max_d:.2e}; policy turns |d| > {tol:g}: {over} of {turns} (largest gain among them "
        f"{over_gain:.3g}), bit-identical {exact}; env-steps {int(ref['idx'].sum())}")
    return diverged
