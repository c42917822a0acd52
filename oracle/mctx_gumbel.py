"""CPU oracle: Gumbel MuZero search of mctx 0.0.6, batched in NumPy (TEST INFRASTRUCTURE ONLY).

mctx 0.0.6 (``uv.lock:655`` of the reference) is NOT vendored in /root/reference; this file
restates its published algorithm:
  mctx/_src/policies.py      gumbel_muzero_policy, _mask_invalid_actions
  mctx/_src/search.py        search, simulate, expand, backward, update_tree_node,
                             instantiate_tree_from_root
  mctx/_src/action_selection.py  gumbel_muzero_root/interior_action_selection, masked_argmax
  mctx/_src/qtransforms.py   qtransform_completed_by_mix_value (+ _compute_mixed_value,
                             _complete_qvalues, _rescale_qvalues)
  mctx/_src/seq_halving.py   score_considered, get_sequence_of_considered_visits
  mctx/_src/tree.py          Tree.qvalues, Tree.summary
and anchors on the reference call site MuZero_det_MADN/muzero_deterministic_madn.py:663-704
(qtransform_completed_by_mix_value(value_scale=0.5), max_num_considered_actions=16 default,
gumbel_scale=temperature).  Parity vs mctx itself: UNPINNED (no reference test covers it).

The Gumbel noise is an explicit input (the reference draws it with jax threefry, which is
not restated); given the noise the search is deterministic.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
UNVISITED = -1
NO_PARENT = -1
TINY = np.finfo(np.float32).tiny
FMIN = np.finfo(np.float32).min


# ---------------------------------------------------------------- seq_halving.py
def get_sequence_of_considered_visits(max_num_considered_actions, num_simulations):
    if max_num_considered_actions <= 1:
        return tuple(range(num_simulations))
    log2max = int(math.ceil(math.log2(max_num_considered_actions)))
    sequence = []
    visits = [0] * max_num_considered_actions
    num_considered = max_num_considered_actions
    while len(sequence) < num_simulations:
        num_extra_visits = max(1, int(num_simulations / (log2max * num_considered)))
        for _ in range(num_extra_visits):
            sequence.extend(visits[:num_considered])
            for i in range(num_considered):
                visits[i] += 1
        num_considered = max(2, num_considered // 2)
    return tuple(sequence[:num_simulations])


def get_table_of_considered_visits(max_num_considered_actions, num_simulations):
    return np.array([get_sequence_of_considered_visits(m, num_simulations)
                     for m in range(max_num_considered_actions + 1)], dtype=np.int32)


def score_considered(considered_visit, gumbel, logits, normalized_qvalues, visit_counts):
    low_logit = F32(-1e9)
    logits = logits - logits.max(-1, keepdims=True)
    penalty = np.where(visit_counts == considered_visit, F32(0.0), F32(-np.inf))
    return (np.maximum(low_logit, gumbel + logits + normalized_qvalues) + penalty).astype(F32)


# ---------------------------------------------------------------- helpers
def exp_cr(x):
    """float32 exp, correctly rounded: evaluated in float64 and rounded once.  numpy's own float32 exp is up to
    a few ulp off (and its SIMD kernels differ between host CPUs); jax's is another polynomial.  The device
    search (csrc/search.hip exp_cr) rounds the same float64 exp, so the tree arithmetic compares bit for bit."""
    return np.exp(np.asarray(x, F32).astype(np.float64)).astype(F32)


LANES = 32   # lanes per game of the wide-action device search (csrc/dog_search.hip)


def lane_tree_sum(x):
    """float32 sum over the last axis in the order of the wide-action device search (A > 128, DOG's 806):
    lane l of a game's 32 lanes adds its entries l, l + 32, l + 64, ... in turn, then the 32 lane sums are
    combined as a balanced binary tree in lane order (((s0 + s1) + (s2 + s3)) + ...) -- the DPP / permlane
    butterfly of csrc/nn.hpp row_reduce, whose every step adds a commutative pair."""
    x = np.asarray(x, F32)
    A = x.shape[-1]
    pad = (-A) % LANES
    xp = np.concatenate([x, np.full(x.shape[:-1] + (pad,), F32(-0.0))], -1) if pad else x
    cols = xp.reshape(x.shape[:-1] + (-1, LANES))          # [..., j, lane]
    s = cols[..., 0, :].copy()
    for j in range(1, cols.shape[-2]):
        s = (s + cols[..., j, :]).astype(F32)
    while s.shape[-1] > 1:
        s = (s[..., 0::2] + s[..., 1::2]).astype(F32)
    return s[..., 0]


def row_sum(x, keepdims=False):
    """Sum over the action axis: numpy's own (pairwise) order up to 128 actions -- the det / classic kernels
    restate it (csrc/search.hip row_sum24) -- and the wide search's lane order beyond."""
    x = np.asarray(x, F32)
    out = x.sum(-1).astype(F32) if x.shape[-1] <= 128 else lane_tree_sum(x)
    return out[..., None] if keepdims else out


def softmax(x):
    x = x.astype(F32)
    u = exp_cr(x - x.max(-1, keepdims=True))
    return (u / row_sum(u, keepdims=True)).astype(F32)


def mask_invalid_actions(logits, invalid):
    logits = (logits - logits.max(-1, keepdims=True)).astype(F32)
    return np.where(invalid, FMIN, logits).astype(F32)


def masked_argmax(x, invalid):
    x = np.where(invalid, -np.inf, x) if invalid is not None else x
    return np.argmax(x, -1).astype(np.int32)


# Near-tie instrumentation for the parity tests (not part of mctx).  Two fp32 implementations of the same
# tree arithmetic that sum in different orders agree on every value in [-1, 1] to a few ulps; the Q-value
# rescale (q - lo) / (hi - lo) multiplies that by the gain K = visit_scale * value_scale / (hi - lo), which
# is large when the children's values are nearly equal (and 0 when they are exactly equal: the rescale then
# maps every entry to 0 on both sides).  A decision whose top-2 gap is below
# TIE_REL * max(1, |top|) + DQ * K could legitimately go either way; margin = gap / that bound (<= 1: tie).
TIE_REL = 1e-5
DQ = 4.8e-7            # 4 fp32 ulps at 1


def top2_margin(x, gain=0.0):
    """Top-2 gap of each row's argmax decision over its uncertainty bound (see above); inf when only one
    entry is finite."""
    x = np.asarray(x, np.float64)
    srt = np.sort(np.where(np.isfinite(x), x, -np.inf), -1)
    with np.errstate(invalid="ignore"):
        bound = TIE_REL * np.maximum(1.0, np.abs(srt[:, -1])) + DQ * np.asarray(gain, np.float64)
        m = (srt[:, -1] - srt[:, -2]) / bound
    return np.where(np.isfinite(m), m, np.inf)


def _note(trace, mask, x, gain=0.0):
    """Fold the decision margins of the rows in `mask` into trace['margin'] (per game minimum)."""
    if trace is None:
        return
    m = top2_margin(x, gain)
    trace["margin"] = np.where(mask, np.minimum(trace["margin"], m), trace["margin"])


class Tree:
    def __init__(self, B, S, A, E):
        N = S + 1
        self.node_visits = np.zeros((B, N), np.int32)
        self.raw_values = np.zeros((B, N), F32)
        self.node_values = np.zeros((B, N), F32)
        self.parents = np.full((B, N), NO_PARENT, np.int32)
        self.action_from_parent = np.full((B, N), NO_PARENT, np.int32)
        self.children_index = np.full((B, N, A), UNVISITED, np.int32)
        self.children_prior_logits = np.zeros((B, N, A), F32)
        self.children_values = np.zeros((B, N, A), F32)
        self.children_visits = np.zeros((B, N, A), np.int32)
        self.children_rewards = np.zeros((B, N, A), F32)
        self.children_discounts = np.zeros((B, N, A), F32)
        self.embeddings = np.zeros((B, N, E), F32)
        self.B = B

    def qvalues(self, node):
        b = np.arange(self.B)
        return (self.children_rewards[b, node] + self.children_discounts[b, node] * self.children_values[b, node]
                ).astype(F32)


def update_tree_node(t: Tree, node, prior_logits, value, embedding):
    b = np.arange(t.B)
    t.children_prior_logits[b, node] = prior_logits
    t.raw_values[b, node] = value
    t.node_values[b, node] = value
    t.node_visits[b, node] = t.node_visits[b, node] + 1
    t.embeddings[b, node] = embedding


# ---------------------------------------------------------------- qtransforms.py
def qtransform_completed_by_mix_value(t: Tree, node, value_scale=0.5, maxvisit_init=50.0, rescale_values=True,
                                      use_mixed_value=True, epsilon=1e-8, with_gain=False):
    b = np.arange(t.B)
    q = t.qvalues(node)
    visits = t.children_visits[b, node]
    raw = t.raw_values[b, node]
    prior_probs = softmax(t.children_prior_logits[b, node])
    if use_mixed_value:
        sum_visits = visits.sum(-1)
        pp = np.maximum(F32(TINY), prior_probs)
        visited = visits > 0
        sum_probs = row_sum(np.where(visited, pp, F32(0.0)))
        denom = np.where(visited, sum_probs[:, None], F32(1.0))
        weighted_q = row_sum(np.where(visited, (pp * q / denom).astype(F32), F32(0.0)))
        value = ((raw + sum_visits.astype(F32) * weighted_q) / (sum_visits + 1).astype(F32)).astype(F32)
    else:
        value = raw
    cq = np.where(visits > 0, q, value[:, None]).astype(F32)
    span = np.ones(t.B, F32)
    if rescale_values:
        lo = cq.min(-1, keepdims=True)
        hi = cq.max(-1, keepdims=True)
        span = np.maximum(hi - lo, F32(epsilon))[:, 0]
        cq = ((cq - lo) / np.maximum(hi - lo, F32(epsilon))).astype(F32)
    maxvisit = visits.max(-1)
    visit_scale = (F32(maxvisit_init) + maxvisit.astype(F32)).astype(F32)
    out = (visit_scale[:, None] * F32(value_scale) * cq).astype(F32)
    if with_gain:      # d out / d q: how much the rescale amplifies rounding in q (near-tie instrumentation);
        # an exactly flat row (hi == lo: every entry the same completed value) carries no amplified difference
        flat = (cq.max(-1) == cq.min(-1)) if not rescale_values else (span <= F32(epsilon)) & (hi == lo)[:, 0]
        return out, np.where(flat, 0.0, visit_scale.astype(np.float64) * value_scale / span)
    return out


# ---------------------------------------------------------------- action_selection.py
def root_action_selection(t: Tree, node, root_invalid, gumbel, table, max_num_considered=16, trace=None,
                          active=None):
    b = np.arange(t.B)
    visits = t.children_visits[b, node]
    prior = t.children_prior_logits[b, node]
    cq, gain = qtransform_completed_by_mix_value(t, node, with_gain=True)
    num_valid = (1 - root_invalid.astype(np.int32)).sum(-1)
    num_considered = np.minimum(max_num_considered, num_valid)
    sim_index = visits.sum(-1)
    considered_visit = table[num_considered, sim_index]
    score = score_considered(considered_visit[:, None], gumbel, prior, cq, visits)
    if active is not None:
        _note(trace, active, np.where(root_invalid, -np.inf, score), gain)
    return masked_argmax(score, root_invalid)


def interior_action_selection(t: Tree, node, trace=None, active=None):
    b = np.arange(t.B)
    visits = t.children_visits[b, node]
    prior = t.children_prior_logits[b, node]
    cq, gain = qtransform_completed_by_mix_value(t, node, with_gain=True)
    probs = softmax(prior + cq)
    to_argmax = probs - visits.astype(F32) / (1 + visits.sum(-1, keepdims=True)).astype(F32)
    if active is not None:
        _note(trace, active, to_argmax, gain)
    return np.argmax(to_argmax, -1).astype(np.int32)


# ---------------------------------------------------------------- search.py
def simulate(t: Tree, root_invalid, gumbel, table, max_depth, trace=None):
    B = t.B
    b = np.arange(B)
    node_index = np.full(B, NO_PARENT, np.int32)
    action = np.full(B, NO_PARENT, np.int32)
    next_node = np.zeros(B, np.int32)
    depth = np.zeros(B, F32)
    cont = np.ones(B, bool)
    while cont.any():
        ni = np.where(cont, next_node, node_index)
        root_a = root_action_selection(t, ni, root_invalid, gumbel, table, trace=trace,
                                       active=cont & (depth == 0))
        int_a = interior_action_selection(t, ni, trace=trace, active=cont & (depth != 0))
        a = np.where(depth == 0, root_a, int_a)
        nn = t.children_index[b, ni, a]
        d = depth + 1
        c2 = (nn != UNVISITED) & (d < max_depth)
        node_index = np.where(cont, ni, node_index)
        action = np.where(cont, a, action)
        next_node = np.where(cont, nn, next_node)
        depth = np.where(cont, d, depth)
        cont = np.where(cont, c2, cont)
    return node_index, action


def expand(params, t: Tree, recurrent_fn, parent, action, next_node):
    b = np.arange(t.B)
    emb = t.embeddings[b, parent]
    reward, discount, prior, value, nemb = recurrent_fn(params, action, emb)
    update_tree_node(t, next_node, prior, value, nemb)
    t.children_index[b, parent, action] = next_node
    t.children_rewards[b, parent, action] = reward
    t.children_discounts[b, parent, action] = discount
    t.parents[b, next_node] = parent
    t.action_from_parent[b, next_node] = action


def backward(t: Tree, leaf):
    b = np.arange(t.B)
    leaf_value = t.node_values[b, leaf].copy()
    index = leaf.copy()
    while (index != 0).any():
        act = index != 0
        ib = b[act]
        idx = index[act]
        parent = t.parents[ib, idx]
        count = t.node_visits[ib, parent]
        a = t.action_from_parent[ib, idx]
        reward = t.children_rewards[ib, parent, a]
        lv = (reward + t.children_discounts[ib, parent, a] * leaf_value[act]).astype(F32)
        parent_value = ((t.node_values[ib, parent] * count.astype(F32) + lv) / (count.astype(F32) + F32(1.0))
                        ).astype(F32)
        child_value = t.node_values[ib, idx]
        child_count = t.children_visits[ib, parent, a] + 1
        t.node_values[ib, parent] = parent_value
        t.node_visits[ib, parent] = count + 1
        t.children_values[ib, parent, a] = child_value
        t.children_visits[ib, parent, a] = child_count
        leaf_value[act] = lv
        index[act] = parent


def gumbel_muzero_policy(params, root_logits, root_value, root_embedding, recurrent_fn, num_simulations,
                         invalid_actions, gumbel, max_depth=None, max_num_considered_actions=16, trace=None):
    """mctx.gumbel_muzero_policy with explicit (already gumbel_scale-scaled) Gumbel noise.

    Returns (action [B], action_weights [B, A], root_value [B] = summary().value, tree).  With a dict `trace`,
    trace['margin'][b] is the smallest normalised top-2 gap (top2_margin) of every argmax decision game b's
    search took (root and interior selections of every simulation, and the final action), and
    trace['gain'][b] the Q-rescale gain of the final action weights: a game whose margin is > 1 cannot
    legitimately choose differently under another fp32 summation order."""
    B, A = root_logits.shape
    E = root_embedding.shape[-1]
    S = num_simulations
    if max_depth is None:
        max_depth = S
    invalid = np.asarray(invalid_actions, bool)
    logits = mask_invalid_actions(root_logits.astype(F32), invalid)
    gumbel = np.asarray(gumbel, F32)
    table = get_table_of_considered_visits(max_num_considered_actions, S)
    t = Tree(B, S, A, E)
    if trace is not None:
        trace["margin"] = np.full(B, np.inf)
    update_tree_node(t, np.zeros(B, np.int32), logits, root_value.astype(F32), root_embedding.astype(F32))
    for sim in range(S):
        parent, action = simulate(t, invalid, gumbel, table, max_depth, trace)
        nn = t.children_index[np.arange(B), parent, action]
        nn = np.where(nn == UNVISITED, sim + 1, nn).astype(np.int32)
        expand(params, t, recurrent_fn, parent, action, nn)
        backward(t, nn)
    root = np.zeros(B, np.int32)
    visits = t.children_visits[:, 0].astype(F32)
    considered_visit = visits.max(-1, keepdims=True)
    cq, gain = qtransform_completed_by_mix_value(t, root, with_gain=True)
    to_argmax = score_considered(considered_visit, gumbel, logits, cq, visits)
    _note(trace, np.ones(B, bool), np.where(invalid, -np.inf, to_argmax), gain)
    if trace is not None:
        trace["gain"] = gain    # the action weights softmax(logits + cq) inherit q's rounding times this
    action = masked_argmax(to_argmax, invalid)
    weights = softmax(mask_invalid_actions((logits + cq).astype(F32), invalid))
    return action, weights, t.node_values[:, 0].copy(), t
