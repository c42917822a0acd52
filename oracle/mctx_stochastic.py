"""CPU oracle: Stochastic MuZero search of mctx 0.0.6 (TEST INFRASTRUCTURE ONLY).

mctx 0.0.6 (``uv.lock:655`` of the reference) is not vendored; this restates its published
``stochastic_muzero_policy`` (policies.py) with ``_make_stochastic_recurrent_fn``,
``_make_stochastic_action_selection_fn``, ``_mask_tree``, ``muzero_action_selection`` and
``qtransform_by_parent_and_siblings`` as called by MuZero_Classic_MADN/muzero_classic_madn.py:464-517
(qtransform_by_parent_and_siblings, dirichlet 0.25 / 0.3, pb_c 1.25 / 19652, temperature).

Only the branch a node actually uses is evaluated (mctx computes the decision AND the chance function
for every expansion and keeps one per lane; the other output is never read).

Randomness, all explicit so both sides see the same numbers (the reference uses jax threefry:
parity of the random SOURCE is unpinned):
  * ``dirichlet`` [B, A]: the root noise sample;
  * the 1e-7 tie-break uniform of muzero_action_selection: ``tiebreak_uniform`` (the engine's
    counter RNG, restated bit-exactly);
  * ``gumbel`` [B, A]: the Gumbel draws of the final ``jax.random.categorical``.
Parity status: UNPINNED (no reference test covers mctx).
"""
from __future__ import annotations

import numpy as np

from .selfplay import M64, _mix64

F32 = np.float32
FMIN = np.finfo(np.float32).min
TINY = np.finfo(np.float32).tiny


def tiebreak_uniform(seed, gid, turn, sim, depth, a):
    """csrc/stochastic.hip:tiebreak_uniform: U[0,1) on a 24-bit grid from a counter hash."""
    h = _mix64((seed & M64) ^ _mix64(((gid & 0xFFFFFFFF) << 32) | (turn & 0xFFFFFFFF))
               ^ _mix64(((sim & 0xFFFF) << 16) | (depth & 0xFFFF)) ^ (((a + 1) * 0x9E6C63D0676A9A99) & M64))
    return np.float32((h >> 40) * (1.0 / 16777216.0))


def _softmax(x):
    x = np.asarray(x, F32)
    m = np.max(x)
    e = np.exp(x - m).astype(F32)
    return (e / e.sum(dtype=F32)).astype(F32)


class _Tree:
    def __init__(self, N, Ap, L):
        self.visits = np.zeros(N, np.int32)
        self.raw = np.zeros(N, F32)
        self.value = np.zeros(N, F32)
        self.is_dec = np.zeros(N, bool)
        self.emb = np.zeros((N, L), F32)
        self.info = np.zeros((N, 2), F32)
        self.parent = np.full(N, -1, np.int32)
        self.afp = np.full(N, -1, np.int32)
        self.c_index = np.full((N, Ap), -1, np.int32)
        self.c_prior = np.zeros((N, Ap), F32)
        self.c_value = np.zeros((N, Ap), F32)
        self.c_visits = np.zeros((N, Ap), np.int32)
        self.c_reward = np.zeros((N, Ap), F32)
        self.c_disc = np.zeros((N, Ap), F32)

    def qvalues(self, n):
        return (self.c_reward[n] + self.c_disc[n] * self.c_value[n]).astype(F32)

    def update_node(self, n, prior, value, is_dec, emb, info):
        self.c_prior[n] = prior
        self.raw[n] = value
        self.value[n] = value
        self.visits[n] += 1
        self.is_dec[n] = is_dec
        self.emb[n] = emb
        self.info[n] = info


def qtransform_by_parent_and_siblings(t: _Tree, n, eps=1e-8, with_gain=False):
    q = t.qvalues(n)
    vis = t.c_visits[n]
    nv = t.value[n]
    safe = np.where(vis > 0, q, nv)
    lo = min(nv, safe.min())
    hi = max(nv, safe.max())
    comp = np.where(vis > 0, q, lo)
    out = ((comp - lo) / max(F32(hi - lo), F32(eps))).astype(F32)
    if with_gain:       # d out / d q (near-tie instrumentation, see mctx_gumbel.top2_margin)
        return out, (0.0 if hi == lo else 1.0 / float(max(F32(hi - lo), F32(eps))))
    return out


def _margin(x, gain=0.0):
    """Normalised top-2 gap of one argmax decision (see mctx_gumbel.top2_margin); test instrumentation."""
    from oracle.mctx_gumbel import top2_margin
    return float(top2_margin(np.asarray(x)[None], gain)[0])


def decision_select(t: _Tree, n, depth, root_invalid, tb, margins=None):
    """muzero_action_selection (action_selection.py) with the root mask at depth 0."""
    vc = t.c_visits[n]
    nvis = t.visits[n]
    pb_c = F32(1.25) + F32(np.log(F32((F32(nvis) + F32(19652.0) + F32(1.0)) / F32(19652.0))))
    probs = _softmax(t.c_prior[n])
    policy = (F32(np.sqrt(F32(nvis))) * pb_c * probs / (vc + 1).astype(F32)).astype(F32)
    cq, gain = qtransform_by_parent_and_siblings(t, n, with_gain=True)
    score = (cq + policy + F32(1e-7) * tb).astype(F32)
    if depth == 0:
        score = np.where(root_invalid, -np.inf, score)
    if margins is not None:
        margins.append(_margin(score, gain))
    return int(np.argmax(score))


def chance_select(t: _Tree, n, A, margins=None):
    p = _softmax(t.c_prior[n, A:])
    x = p / (t.c_visits[n, A:] + 1).astype(F32)
    if margins is not None:
        margins.append(_margin(x))
    return int(np.argmax(x)) + A


def stochastic_muzero_policy(params, root_logits, root_value, root_emb, decision_fn, chance_fn, num_simulations,
                             invalid, dirichlet, gumbel, max_depth=None, temperature=1.0, seed=0, turn=0, gids=None,
                             num_chance=6, dirichlet_fraction=0.25, trace=None):
    """Batched over B games (per-game trees, batched network calls).

    decision_fn(params, action[b], emb[b,256]) -> (chance_logits, afterstate_value, afterstate, reward, discount)
    chance_fn(params, chance[b], afterstate[b,256]) -> (action_logits, value, next_state)
    Returns (action [B], action_weights [B, A], root_value_clipped [B], trees).  With a dict `trace`,
    trace['margin'][b] is the smallest relative top-2 gap of every argmax decision of game b's search."""
    B, A = root_logits.shape
    C = num_chance
    Ap = A + C
    S = num_simulations
    D = S if max_depth is None else max_depth
    L = root_emb.shape[1]
    gids = np.arange(B) if gids is None else np.asarray(gids)
    # root noise (policies.py: _add_dirichlet_noise, _get_logits_from_probs, _mask_invalid_actions)
    probs = np.stack([_softmax(root_logits[b]) for b in range(B)])
    noisy = (F32(1 - dirichlet_fraction) * probs + F32(dirichlet_fraction) * dirichlet.astype(F32)).astype(F32)
    logits = np.log(np.maximum(noisy, TINY)).astype(F32)
    logits = (logits - logits.max(-1, keepdims=True)).astype(F32)
    logits = np.where(invalid, FMIN, logits).astype(F32)
    root_prior = np.concatenate([logits, np.full((B, C), -np.inf, F32)], -1)
    root_invalid = np.concatenate([invalid.astype(bool), np.ones((B, C), bool)], -1)
    trees = [_Tree(S + 1, Ap, L) for _ in range(B)]
    margins = [[] if trace is not None else None for _ in range(B)]
    for b, t in enumerate(trees):
        t.update_node(0, root_prior[b], F32(root_value[b]), True, root_emb[b], (0.0, 0.0))
    for sim in range(S):
        parents, actions, nexts = [], [], []
        for b, t in enumerate(trees):
            node, depth = 0, 0
            while True:
                if t.is_dec[node]:
                    tb = np.array([tiebreak_uniform(seed, int(gids[b]), turn, sim, depth, a) for a in range(Ap)], F32)
                    a = decision_select(t, node, depth, root_invalid[b], tb, margins[b])
                else:
                    a = chance_select(t, node, A, margins[b])
                nxt = t.c_index[node, a]
                depth += 1
                if nxt == -1 or depth >= D:
                    break
                node = nxt
            parents.append(node)
            actions.append(a)
            nexts.append(int(t.c_index[node, a]) if t.c_index[node, a] != -1 else sim + 1)
        dec = [b for b in range(B) if trees[b].is_dec[parents[b]]]
        cha = [b for b in range(B) if not trees[b].is_dec[parents[b]]]
        if dec:
            cl, av, after, r, d = decision_fn(params, np.array([actions[b] for b in dec]),
                                              np.stack([trees[b].emb[parents[b]] for b in dec]))
            for j, b in enumerate(dec):
                t, p, a, nn = trees[b], parents[b], actions[b], nexts[b]
                prior = np.concatenate([np.full(A, -np.inf, F32), cl[j].astype(F32)])
                t.update_node(nn, prior, F32(av[j]), False, after[j], (r[j], d[j]))
                t.c_reward[p, a], t.c_disc[p, a] = F32(0.0), F32(1.0)
                t.c_index[p, a], t.parent[nn], t.afp[nn] = nn, p, a
        if cha:
            lg, v, nxt_state = chance_fn(params, np.array([actions[b] - A for b in cha]),
                                         np.stack([trees[b].emb[parents[b]] for b in cha]))
            for j, b in enumerate(cha):
                t, p, a, nn = trees[b], parents[b], actions[b], nexts[b]
                prior = np.concatenate([lg[j].astype(F32), np.full(C, -np.inf, F32)])
                t.update_node(nn, prior, F32(v[j]), True, nxt_state[j], (0.0, 0.0))
                t.c_reward[p, a], t.c_disc[p, a] = t.info[p, 0], t.info[p, 1]
                t.c_index[p, a], t.parent[nn], t.afp[nn] = nn, p, a
        for b, t in enumerate(trees):          # search.py backward
            idx = nexts[b]
            leaf = F32(t.value[idx])
            while idx != 0:
                p = t.parent[idx]
                cnt = t.visits[p]
                a = t.afp[idx]
                leaf = F32(t.c_reward[p, a] + t.c_disc[p, a] * leaf)
                t.value[p] = F32((t.value[p] * F32(cnt) + leaf) / (F32(cnt) + F32(1.0)))
                t.visits[p] = cnt + 1
                t.c_value[p, a] = t.value[idx]
                t.c_visits[p, a] += 1
                idx = p
    # _mask_tree(decision) + summary + _apply_temperature + categorical
    action = np.zeros(B, np.int32)
    weights = np.zeros((B, A), F32)
    rv = np.zeros(B, F32)
    for b, t in enumerate(trees):
        vc = t.c_visits[0, :A].astype(F32)
        tot = vc.sum(dtype=F32)
        w = (vc / max(tot, F32(1.0))).astype(F32) if tot > 0 else np.full(A, F32(1.0 / A), F32)
        weights[b] = w
        with np.errstate(divide="ignore"):
            lw = np.log(w).astype(F32)
        lw = ((lw - lw.max()) / max(TINY, F32(temperature))).astype(F32)
        if margins[b] is not None:
            margins[b].append(_margin(lw + gumbel[b].astype(F32)))
        action[b] = int(np.argmax(lw + gumbel[b].astype(F32)))
        rv[b] = np.clip(t.value[0], -1.0, 1.0)
    if trace is not None:
        trace["margin"] = np.array([min(m) if m else np.inf for m in margins])
    return action, weights, rv, trees
