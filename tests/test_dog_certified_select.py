"""Soundness of k_dog_search's certified interior argmax (csrc/dog_search.hip wselect_certified), on the CPU.

The kernel picks mctx's interior action (softmax(prior + completed Q) - N / (1 + sum N), oracle/mctx_gumbel.py
interior_action_selection) from the visited children and the unvisited child of the largest prior, with the softmax
denominator bounded instead of summed, and falls back to the exact 806-exponential path when the bound cannot
separate the best candidate.  The GPU tests compare whole searches bit for bit, but their nodes almost never come
near a tie (the exact path ran 0 times in 902,542 self-play selections).  Here the certification is restated
line for line (float32 where the kernel computes in float, float64 where it does) and run on random and adversarial
nodes -- duplicated / one-ulp-apart priors, ties between visited children, extreme logits -- against the oracle's
own exact selection: whenever it certifies, it must pick the exact argmax.  Test infrastructure, not the product."""
import numpy as np

from oracle import mctx_gumbel as G

F32 = np.float32
A = 806
TINY = np.finfo(np.float32).tiny


def exact_cq(prior, q, visits, raw, value_scale=0.5, maxvisit_init=50.0):
    """qtransform_completed_by_mix_value for one node (oracle/mctx_gumbel.py:178-209, one row)."""
    prior_probs = G.softmax(prior[None])[0]
    pp = np.maximum(F32(TINY), prior_probs)
    visited = visits > 0
    sum_probs = G.row_sum(np.where(visited, pp, F32(0.0))[None])[0]
    denom = np.where(visited, sum_probs, F32(1.0))
    weighted_q = G.row_sum(np.where(visited, (pp * q / denom).astype(F32), F32(0.0))[None])[0]
    sv = visits.sum()
    value = F32((raw + F32(sv) * weighted_q) / F32(sv + 1))
    cq = np.where(visited, q, value).astype(F32)
    lo, hi = cq.min(), cq.max()
    cq = ((cq - lo) / np.maximum(hi - lo, F32(1e-8))).astype(F32)
    scale = F32(F32(maxvisit_init) + F32(visits.max())) * F32(value_scale)
    return (scale * cq).astype(F32)


def exact_pick(prior, cq, visits):
    probs = G.softmax((prior + cq).astype(F32)[None])[0]
    score = (probs - visits.astype(F32) / F32(1 + visits.sum())).astype(F32)
    return int(np.argmax(score))


def certified_pick(prior, cq, visits):
    """wselect_certified restated: -1 when it declines (the kernel then runs the exact path)."""
    visited = np.flatnonzero(visits > 0)
    unv = np.flatnonzero(visits == 0)
    pm = prior.max()
    es = G.lane_tree_sum(G.exp_cr(prior - pm))
    order = unv[np.lexsort((unv, -prior[unv].astype(np.float64)))]    # (value desc, index asc)
    ui, u1 = int(order[0]), prior[order[0]]
    u2 = prior[order[1]] if len(order) > 1 else F32(-np.inf)
    K = cq[ui]                                                       # every unvisited child's completed Q
    zU = F32(u1 + K)
    z = (prior[visited] + cq[visited]).astype(F32)
    zm = max(F32(z.max()) if len(z) else F32(-np.inf), zU)
    ez = G.exp_cr((z - zm).astype(F32))
    sez = F32(ez.sum(dtype=np.float64))
    sep = F32(G.exp_cr((prior[visited] - pm).astype(F32)).sum(dtype=np.float64))
    f = np.exp(float(K) + float(pm) - float(zm))
    zsa = float(sez) + f * max(float(es) - float(sep), 0.0)
    c0 = 4.0 * (abs(float(zm)) + abs(float(K)) + abs(float(pm)) + 1.0)
    err = zsa * (2.0 ** -23 * (c0 + 900.0) + 2.0 ** -17) + f * float(es) * 2.0 ** -17
    if not (zsa - err > 0.0) or not (err < 0.01 * zsa):
        return -1
    zlo = F32(F32(zsa - err) * F32(1 - 2.0 ** -22))
    zhi = F32(F32(zsa + err) * F32(1 + 2.0 ** -22))
    n = (visits[visited].astype(F32) / F32(1 + visits.sum())).astype(F32)
    q_hi = (ez / zlo).astype(F32)
    slack = (F32(2.0 ** -20) * (q_hi + n)).astype(F32)
    lo = ((ez / zhi - n) - slack).astype(F32)
    hi = ((q_hi - n) + slack).astype(F32)
    bi, blo = A, F32(-np.inf)
    for k, a in enumerate(visited):                                 # (value desc, index asc)
        if lo[k] > blo or (lo[k] == blo and a < bi):
            bi, blo = int(a), lo[k]
    ezU = G.exp_cr(F32(zU - zm))
    loU = F32(ezU / zhi - F32(2.0 ** -20) * F32(ezU / zlo))
    hiU = F32(ezU / zlo + F32(2.0 ** -20) * F32(ezU / zlo))
    pick_u = loU > blo or bi >= A
    if pick_u:
        bi, blo = ui, loU
        if not loU > F32(2.0 ** -100):
            return -1
        if u2 != -np.inf and not ezU > F32(G.exp_cr(F32(F32(u2 + K) - zm)) * F32(1 + 2.0 ** -21)):
            return -1
    others = [hi[k] for k, a in enumerate(visited) if a != bi]
    hub = max(others + ([] if pick_u else [hiU]), default=F32(-np.inf))
    return bi if blo > hub else -1


def make_node(rng, kind):
    prior = rng.normal(0, rng.choice([0.5, 2.0, 8.0]), A).astype(F32)
    if kind == "dup":          # the largest prior repeated, some one ulp apart
        m = prior.max()
        idx = rng.choice(A, 6, replace=False)
        prior[idx[:3]] = m
        prior[idx[3:]] = np.nextafter(m, F32(-np.inf))
    if kind == "peaked":       # one dominant logit (the deep dives of random-init networks)
        prior[rng.integers(A)] += F32(rng.uniform(5, 30))
    nv = int(rng.integers(0, 12))
    vis_idx = rng.choice(A, nv, replace=False)
    if kind == "dup" and nv:
        vis_idx[0] = int(np.argmax(prior))
    visits = np.zeros(A, np.int32)
    visits[vis_idx] = rng.integers(1, 20, nv)
    q = rng.uniform(-1, 1, A).astype(F32)
    if kind == "tie" and nv >= 2:   # two visited children with the same q, prior and count
        q[vis_idx[1]] = q[vis_idx[0]]
        prior[vis_idx[1]] = prior[vis_idx[0]]
        visits[vis_idx[1]] = visits[vis_idx[0]]
    raw = F32(rng.uniform(-1, 1))
    return prior, q, visits, raw


def test_certified_pick_is_the_exact_argmax():
    rng = np.random.default_rng(12)
    counts = {}
    for kind in ("random", "dup", "peaked", "tie"):
        cert = 0
        n = 1000
        for _ in range(n):
            prior, q, visits, raw = make_node(rng, kind)
            cq = exact_cq(prior, q, visits, raw)
            want = exact_pick(prior, cq, visits)
            got = certified_pick(prior, cq, visits)
            if got >= 0:
                cert += 1
                assert got == want, (kind, got, want)
        counts[kind] = cert / n
    print("certified fraction:", counts)
    assert counts["random"] > 0.9 and counts["peaked"] > 0.9
