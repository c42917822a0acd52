"""CPU oracle: gradients of the two MuZero learners' losses (TEST INFRASTRUCTURE ONLY).

A float64 restatement of the reference losses written in the reference's own step order, with torch
autograd standing in for jax.value_and_grad (the arithmetic is restated here, independently of the
package's learner):
  * det  ``loss_fn``            MuZero_det_MADN/train_with_reward.py:24-146 (scan over K+1 steps, lax.cond
                                 on k < K, ``next_latent = stop_gradient(0.5 x) + 0.5 x`` at line 105 AFTER
                                 dynamics_net returned its reward / discount logits, so those heads read the
                                 unscaled next latent, muzero_deterministic_madn.py:437-455);
  * classic ``loss_fn_stochastic`` MuZero_Classic_MADN/train_stochastic.py:34-181 (action_dynamics ->
                                 afterstate (unscaled) -> chance_dynamics -> next state scaled at line 119).
Networks: the Flax modules as oracle/nets.py / oracle/classic_nets.py restate them -- LayerNorm with the fast
variance max(0, E[x^2] - E[x]^2), 'SAME' Conv1D, one_hot(-1) = 0 -- and the min-max latent scaling with
jnp.min / jnp.max, whose gradient JAX splits evenly over tied entries (reduce_min / reduce_max JVP);
torch.amin / amax do the same.
Parity: unpinned (flax / jax / optax are not vendored); oracle/learner.py holds the fp32 NumPy losses and the
optax AdamW restatement these gradients feed.
"""
from __future__ import annotations

import numpy as np
import torch

EPS_LN = 1e-6
SCALES_DET = dict(value=4.0, policy=1.0, discount=1.0, reward=1.0)                 # train_with_reward.py:323-326
SCALES_CLASSIC = dict(value=4.0, policy=2.0, chance=0.5, discount=1.0, reward=1.0)  # train_stochastic.py:374-378


class _Net:
    def __init__(self, params: dict, dtype=torch.float64, record: bool = False):
        self.rec = [] if record else None
        self.p = {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=True) for k, v in params.items()}
        self.dt = dtype

    def dense(self, name, x):
        return x @ self.p[f"{name}/kernel"] + self.p[f"{name}/bias"]

    def ln(self, name, x):
        mean = x.mean(-1, keepdim=True)
        var = torch.clamp((x * x).mean(-1, keepdim=True) - mean * mean, min=0.0)
        return (x - mean) * (torch.rsqrt(var + EPS_LN) * self.p[f"{name}/scale"]) + self.p[f"{name}/bias"]

    def conv(self, name, x):
        k = self.p[f"{name}/kernel"]
        K, Cin, Cout = k.shape
        pl = (K - 1) // 2
        W = x.shape[1]
        xp = torch.nn.functional.pad(x, (0, 0, pl, K - 1 - pl))
        cols = torch.cat([xp[:, d:d + W, :] for d in range(K)], -1)
        return cols @ k.reshape(K * Cin, Cout) + self.p[f"{name}/bias"]

    def resblock(self, name, x):
        y = self.relu(self.ln(f"{name}/LayerNorm_0", self.dense(f"{name}/Dense_0", x)))
        y = self.ln(f"{name}/LayerNorm_1", self.dense(f"{name}/Dense_1", y))
        return self.relu(x + y)

    def relu(self, x):
        if self.rec is not None:    # decision_margins: distance of every ReLU input to the kink, per batch row
            self.rec.append(("relu", x.detach().reshape(x.shape[0], -1).abs()))
        return torch.relu(x)

    def _mm(self, x):
        if self.rec is not None:    # decision_margins: gap of the two largest / smallest entries over the range
            s = torch.sort(x.detach(), -1)[0]
            gap = torch.minimum(s[:, -1] - s[:, -2], s[:, 1] - s[:, 0]) / (s[:, -1] - s[:, 0]).clamp_min(1e-30)
            self.rec.append(("minmax", gap[:, None]))
        return self.minmax(x)

    @staticmethod
    def minmax(x):
        lo = torch.amin(x, -1, keepdim=True)
        hi = torch.amax(x, -1, keepdim=True)
        return (x - lo) / (hi - lo + 1e-8)

    def one_hot(self, a, n):
        a = torch.as_tensor(np.asarray(a)).long()
        return (a[:, None] == torch.arange(n)[None, :]).to(self.dt)

    # RepresentationNetwork2 (muzero_deterministic_madn.py:75-141)
    def representation(self, obs):
        r = "representation"
        x = torch.as_tensor(np.asarray(obs, np.float32)).to(self.dt)
        sp, g = x[:, :6, :].transpose(1, 2), x[:, 6:, 0]
        for i in range(3):
            sp = self.relu(self.ln(f"{r}/LayerNorm_{i}", self.conv(f"{r}/Conv_{i}", sp)))
        flat = self.relu(self.ln(f"{r}/LayerNorm_3", self.dense(f"{r}/Dense_0", sp.reshape(sp.shape[0], -1))))
        g = self.relu(self.ln(f"{r}/LayerNorm_4", self.dense(f"{r}/Dense_1", g)))
        g = self.relu(self.ln(f"{r}/LayerNorm_5", self.dense(f"{r}/Dense_2", g)))
        h = self.relu(self.ln(f"{r}/LayerNorm_6", self.dense(f"{r}/Dense_3", torch.cat([flat, g], -1))))
        for b in range(6):
            h = self.resblock(f"{r}/ResBlock_{b}", h)
        if f"{r}/LayerNorm_7/scale" in self.p:     # the DOG RepresentationNetwork (MuZero_DOG/muzero_dog.py:80-81)
            return self.ln(f"{r}/LayerNorm_7", self.dense(f"{r}/Dense_4", h))
        return self._mm(self.dense(f"{r}/Dense_4", h))

    # PredictionNetwork4 (muzero_deterministic_madn.py:549-583; classic 192-226)
    def prediction(self, latent):
        p = "prediction"
        x = self.ln(f"{p}/LayerNorm_0", latent)
        for b in range(2):
            x = self.resblock(f"{p}/ResBlock_{b}", x)
        pol = self.relu(self.ln(f"{p}/LayerNorm_1", self.dense(f"{p}/Dense_0", x)))
        pol = self.relu(self.ln(f"{p}/LayerNorm_2", self.dense(f"{p}/Dense_1", pol)))
        v = self.relu(self.ln(f"{p}/LayerNorm_3", self.dense(f"{p}/Dense_3", x)))
        v = self.relu(self.dense(f"{p}/Dense_4", v))
        return self.dense(f"{p}/Dense_2", pol), torch.tanh(self.dense(f"{p}/Dense_5", v))

    # DynamicsNetwork4 (muzero_deterministic_madn.py:391-457)
    def dynamics(self, latent, action, A=None):
        d = "dynamics"
        A = self.p[f"{d}/Dense_0/kernel"].shape[0] if A is None else A     # 24 det, 806 DOG
        oh = self.one_hot(action, A)
        e = self.relu(self.dense(f"{d}/Dense_0", oh))
        x = self.ln(f"{d}/LayerNorm_0", latent) * (1.0 + self.dense(f"{d}/Dense_1", e)) + self.dense(f"{d}/Dense_2", e)
        x = self.relu(self.ln(f"{d}/LayerNorm_1", self.dense(f"{d}/Dense_3", x)))
        x = self.relu(self.ln(f"{d}/LayerNorm_2", self.dense(f"{d}/Dense_4", x)))
        for b in range(2):
            x = self.resblock(f"{d}/ResBlock_{b}", x)
        nxt = self._mm(latent + self.dense(f"{d}/Dense_5", x))
        ri = torch.cat([nxt, oh], -1)
        rl = self.dense(f"{d}/reward_head", self.relu(self.dense(f"{d}/Dense_6", ri)))
        dl = self.dense(f"{d}/discount_head", self.relu(self.dense(f"{d}/Dense_7", ri)))
        return nxt, rl, dl

    # StochasticDynamicsNetwork4 (muzero_classic_madn.py:314-408)
    def _film_trunk(self, pre, rb0, x_in, e):
        d = "dynamics"
        x = self.ln(f"{d}/{pre}_input_ln", x_in) * (1.0 + self.dense(f"{d}/{pre}_film_scale", e)) + \
            self.dense(f"{d}/{pre}_film_shift", e)
        x = self.relu(self.ln(f"{d}/{pre}_ln1", self.dense(f"{d}/{pre}_dense1", x)))
        x = self.relu(self.ln(f"{d}/{pre}_ln2", self.dense(f"{d}/{pre}_dense2", x)))
        for r in range(rb0, rb0 + 2):
            x = self.resblock(f"{d}/ResBlock_{r}", x)
        return self._mm(x_in + self.dense(f"{d}/{pre}_proj", x))

    def action_dynamics(self, latent, action, A=4):
        d = "dynamics"
        oh = self.one_hot(action, A)
        after = self._film_trunk("act", 0, latent, self.relu(self.dense(f"{d}/act_embed", oh)))
        rl = self.dense(f"{d}/reward_head", self.relu(self.dense(f"{d}/reward_dense", torch.cat([after, oh], -1))))
        dl = self.dense(f"{d}/discount_head", self.relu(self.ln(f"{d}/discount_ln", self.dense(f"{d}/discount_dense", latent))))
        return after, rl, self.dense(f"{d}/chance_head", after), dl

    def chance_dynamics(self, after, chance, C=6):
        e = self.relu(self.dense("dynamics/chance_embed", self.one_hot(chance, C)))
        return self._film_trunk("chance", 2, after, e)


def _t(x, dt):
    return torch.as_tensor(np.asarray(x)).to(dt)


def _ce_int(logits, labels):
    """optax.softmax_cross_entropy_with_integer_labels."""
    return -torch.log_softmax(logits, -1).gather(1, torch.as_tensor(np.asarray(labels)).long()[:, None])[:, 0]


def _scaled(x, s=0.5):
    """jax.lax.stop_gradient(x * s) + x * s (train_with_reward.py:105, train_stochastic.py:119)."""
    return (x * s).detach() + x * s


def det_loss(net: _Net, batch: dict, unroll_steps: int = 10):
    """train_with_reward.py:24-146 -> (total, (value, policy, discount, reward)) as float64 tensors."""
    dt = net.dt
    latent = net.representation(batch["observations"])
    B, K = np.asarray(batch["actions"]).shape
    acts = np.concatenate([np.asarray(batch["actions"]), np.zeros((B, 1), np.int32)], 1)
    disc_t = np.concatenate([np.asarray(batch["discount_targets"]), np.ones((B, 1), np.int32)], 1)
    rew_t = np.concatenate([np.asarray(batch["rewards"]), np.ones((B, 1), np.int32)], 1)
    sc = SCALES_DET
    total = torch.zeros((), dtype=dt)
    sums = [torch.zeros((), dtype=dt) for _ in range(4)]
    for k in range(K + 1):
        mask = _t(batch["masks"], dt)[:, k]
        logits, v = net.prediction(latent)
        l_value = torch.mean(mask * (_t(batch["target_values"], dt)[:, k] - v[:, 0]) ** 2)
        l_policy = torch.mean(mask * -(_t(batch["policies"], dt)[:, k] * torch.log_softmax(logits, -1)).sum(-1))
        step = (1.0 / unroll_steps) * (sc["value"] * l_value + sc["policy"] * l_policy)
        l_disc = l_rew = torch.zeros((), dtype=dt)
        nxt = latent
        if k < K:
            nxt, rl, dl = net.dynamics(latent, acts[:, k])
            rc = torch.as_tensor(rew_t[:, k])
            ce = _ce_int(rl, rew_t[:, k])
            neu = (rc == 1).to(dt)
            n_neu = torch.clamp((mask * neu).sum(), min=1.0)
            n_non = torch.clamp((mask * (1 - neu)).sum(), min=1.0)
            l_rew = 0.1 * (mask * neu * ce).sum() / n_neu + 1.0 * (mask * (1 - neu) * ce).sum() / n_non
            dc = torch.as_tensor(disc_t[:, k])
            ce = _ce_int(dl, disc_t[:, k])
            term = (dc == 1).to(dt)
            n_nt = torch.clamp((mask * (1 - term)).sum(), min=1.0)
            n_t = torch.clamp((mask * term).sum(), min=1.0)
            l_disc = 0.1 * (mask * (1 - term) * ce).sum() / n_nt + 1.0 * (mask * term * ce).sum() / n_t
        latent = _scaled(nxt)
        total = total + step + (1.0 / unroll_steps) * (sc["discount"] * l_disc + sc["reward"] * l_rew)
        for i, x in enumerate((l_value, l_policy, l_disc, l_rew)):
            sums[i] = sums[i] + x
    return total, tuple(sums)


def _balanced(ce, is_rare, mask, n_valid, w_rare=1.0, w_common=0.1):
    """train_stochastic.py:25-31."""
    masked_rare = mask * is_rare
    n_rare = torch.clamp(masked_rare.sum(), min=1.0)
    n_common = torch.clamp(n_valid - n_rare, min=1.0)
    return w_rare * (masked_rare * ce).sum() / n_rare + w_common * ((mask - masked_rare) * ce).sum() / n_common


def classic_loss(net: _Net, batch: dict, unroll_steps: int = 10):
    """train_stochastic.py:34-181 -> (total, (value, policy, chance, discount, reward))."""
    dt = net.dt
    latent = net.representation(batch["observations"])
    B, K = np.asarray(batch["actions"]).shape
    acts = np.concatenate([np.asarray(batch["actions"]), np.zeros((B, 1), np.int32)], 1)
    dice = np.concatenate([np.asarray(batch["dice_outcomes"])[:, 1:], np.zeros((B, 2), np.int32)], 1)
    probs = np.concatenate([np.asarray(batch["dice_probs"], np.float32), np.full((B, 1, 6), 1.0 / 6.0, np.float32)], 1)
    disc_t = np.concatenate([np.asarray(batch["discount_targets"]), np.ones((B, 1), np.int32)], 1)
    rew_t = np.concatenate([np.asarray(batch["rewards"]), np.ones((B, 1), np.int32)], 1)
    sc = SCALES_CLASSIC
    total = torch.zeros((), dtype=dt)
    sums = [torch.zeros((), dtype=dt) for _ in range(5)]
    for k in range(K + 1):
        mask = _t(batch["masks"], dt)[:, k]
        logits, v = net.prediction(latent)
        l_policy = torch.mean(mask * -(_t(batch["policies"], dt)[:, k] * torch.log_softmax(logits, -1)).sum(-1))
        l_value = torch.mean(mask * (_t(batch["target_values"], dt)[:, k] - v[:, 0]) ** 2)
        n_valid = mask.sum()
        tp = _t(probs[:, k], dt)
        l_chance = l_disc = l_rew = torch.zeros((), dtype=dt)
        nxt = latent
        if k < K:
            after, rl, cl, dl = net.action_dynamics(latent, acts[:, k])
            rc, dc = torch.as_tensor(rew_t[:, k]), torch.as_tensor(disc_t[:, k])
            l_rew = _balanced(_ce_int(rl, rew_t[:, k]), (rc != 1).to(dt), mask, n_valid)
            l_disc = _balanced(_ce_int(dl, disc_t[:, k]), (dc == 1).to(dt), mask, n_valid)
            nonu = (((tp - 1.0 / 6.0) ** 2).sum(-1) > 1e-6).to(dt)
            l_chance = _balanced(-(tp * torch.log_softmax(cl, -1)).sum(-1), nonu, mask, n_valid)
            nxt = net.chance_dynamics(after, dice[:, k])
        latent = _scaled(nxt)
        total = total + (1.0 / unroll_steps) * (sc["value"] * l_value + sc["policy"] * l_policy +
                                                sc["chance"] * l_chance + sc["discount"] * l_disc +
                                                sc["reward"] * l_rew)
        for i, x in enumerate((l_value, l_policy, l_chance, l_disc, l_rew)):
            sums[i] = sums[i] + x
    return total, tuple(sums)


def loss_and_grads(params: dict, batch: dict, unroll_steps: int = 10, classic: bool = False,
                   dtype=torch.float64):
    """jax.value_and_grad(loss_fn[_stochastic], has_aux=True)(params, batch) restated:
    -> (total float, parts tuple of floats, grads {name: float64 ndarray})."""
    net = _Net(params, dtype)
    total, parts = (classic_loss if classic else det_loss)(net, batch, unroll_steps)
    total.backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach().numpy() for k, p in net.p.items()}
    return float(total.detach()), tuple(float(x.detach()) for x in parts), grads


def decision_margins(params: dict, batch: dict, unroll_steps: int = 10, classic: bool = False):
    """The loss's discontinuities, measured in float64: -> (dist [B], sites).  dist[b] = the smallest distance of batch
    row b's forward (every unroll step) to a decision -- a ReLU input's |x| (the kink), or a min-max row's gap between
    its two largest (smallest) entries over its range (the argmax / argmin that takes the extremum's gradient).  A
    fp32 forward that differs from float64 by more than that may take the other side, which moves the gradient by
    a fixed quantum (one ReLU element's or one extremum's whole contribution): the learner gradient test exempts
    such rows, logged (tests/test_gpu_learner_oracle.py).  sites = [(distance, kind, call #, row, column)] sorted,
    the 3 closest of every call."""
    net = _Net(params, torch.float64, record=True)
    with torch.no_grad():
        (classic_loss if classic else det_loss)(net, batch, unroll_steps)
    B = np.asarray(batch["actions"]).shape[0]
    dist = np.full(B, np.inf)
    sites = []
    for call, (kind, t) in enumerate(net.rec):
        m, idx = t.min(1)
        dist = np.minimum(dist, m.numpy())
        for r in torch.argsort(m)[:3].tolist():
            sites.append((float(m[r]), kind, call, r, int(idx[r])))
    sites.sort()
    return dist, sites

