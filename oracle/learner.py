"""CPU oracle: the det-MADN learner's loss and optimizer update (TEST INFRASTRUCTURE ONLY).

NumPy restatement of MuZero_det_MADN/train_with_reward.py:
  * loss_fn 24-141: K+1 unroll steps from the representation of the root observation; value MSE x4 and
    policy cross-entropy per step, class-balanced reward / discount cross-entropies per dynamics step
    (0.1 x neutral + 1.0 x non-neutral rewards; 0.1 x non-terminal + 1.0 x terminal discounts), each step
    scaled by 1 / unroll_steps; the latent carried with the 0.5 gradient scaling (a forward identity);
  * optimizer 361-372: clip_by_global_norm(5.0) -> adamw(piecewise_constant lr, weight_decay 1e-4)
    with optax 0.2 defaults (b1 0.9, b2 0.999, eps 1e-8), restated from its published algorithm.
The forward passes are oracle/nets.py.  Parity: unpinned (no reference test; optax is not vendored).
"""
from __future__ import annotations

import numpy as np

from . import nets as ON

F32 = np.float32
VALUE_SCALING, POLICY_SCALING, DISCOUNT_SCALING, REWARD_SCALING = 4.0, 1.0, 1.0, 1.0


def _log_softmax(x):
    x = x.astype(np.float64)
    m = x.max(-1, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(-1, keepdims=True))


def _ce_int(logits, labels):
    return -np.take_along_axis(_log_softmax(logits), labels[:, None].astype(np.int64), -1)[:, 0]


def loss_fn(params, batch, unroll_steps=10):
    """-> (total_loss, (value_loss, policy_loss, discount_loss, reward_loss)) in float64 from fp32 nets."""
    latent = ON.representation(params, batch["observations"])
    K = batch["actions"].shape[1]
    B = latent.shape[0]
    acts = np.concatenate([batch["actions"], np.zeros((B, 1), np.int32)], 1)
    disc_t = np.concatenate([batch["discount_targets"], np.ones((B, 1), np.int32)], 1)
    rew_t = np.concatenate([batch["rewards"], np.ones((B, 1), np.int32)], 1)
    total = 0.0
    sums = [0.0, 0.0, 0.0, 0.0]
    for k in range(K + 1):
        mask = batch["masks"][:, k].astype(np.float64)
        logits, v = ON.prediction(params, latent)
        l_value = np.mean(mask * (batch["target_values"][:, k] - v[:, 0].astype(np.float64)) ** 2)
        l_policy = np.mean(mask * -(batch["policies"][:, k].astype(np.float64) * _log_softmax(logits)).sum(-1))
        step = (1.0 / unroll_steps) * (VALUE_SCALING * l_value + POLICY_SCALING * l_policy)
        l_disc = l_rew = 0.0
        if k < K:
            nxt, rl, dl = ON.dynamics(params, latent, acts[:, k])
            rc = rew_t[:, k]
            ce = _ce_int(rl, rc)
            neu = rc == 1
            n_neu = max(np.sum(mask * neu), 1.0)
            n_non = max(np.sum(mask * ~neu), 1.0)
            l_rew = 0.1 * np.sum(mask * np.where(neu, ce, 0.0)) / n_neu + 1.0 * np.sum(mask * np.where(~neu, ce, 0.0)) / n_non
            dc = disc_t[:, k]
            ce = _ce_int(dl, dc)
            term = dc == 1
            n_nt = max(np.sum(mask * ~term), 1.0)
            n_t = max(np.sum(mask * term), 1.0)
            l_disc = 0.1 * np.sum(mask * np.where(~term, ce, 0.0)) / n_nt + 1.0 * np.sum(mask * np.where(term, ce, 0.0)) / n_t
            latent = nxt
        total += step + (1.0 / unroll_steps) * DISCOUNT_SCALING * l_disc + (1.0 / unroll_steps) * REWARD_SCALING * l_rew
        for i, x in enumerate((l_value, l_policy, l_disc, l_rew)):
            sums[i] += x
    return total, tuple(sums)


def lr_schedule(step, lr0=0.005, steps_per_iteration=2500):
    """optax.piecewise_constant_schedule of train_with_reward.py:361-368."""
    lr = lr0
    for boundary, scale in ((30, 0.2), (60, 0.2), (85, 0.5)):
        if step >= boundary * steps_per_iteration:
            lr *= scale
    return lr


class AdamW:
    """optax.chain(clip_by_global_norm(5.0), adamw(schedule, weight_decay=1e-4)) on a dict of arrays."""

    def __init__(self, params, max_norm=5.0, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4, schedule=lr_schedule):
        self.mu = {k: np.zeros_like(v, F32) for k, v in params.items()}
        self.nu = {k: np.zeros_like(v, F32) for k, v in params.items()}
        self.count = 0
        self.max_norm, self.b1, self.b2, self.eps, self.wd, self.schedule = max_norm, b1, b2, eps, wd, schedule

    def update(self, params, grads):
        g_norm = np.float32(np.sqrt(sum(np.sum(np.square(g.astype(F32)), dtype=F32) for g in grads.values())))
        trigger = g_norm < self.max_norm
        lr = F32(self.schedule(self.count))
        self.count += 1
        c1 = F32(1.0 - self.b1 ** self.count)
        c2 = F32(1.0 - self.b2 ** self.count)
        out = {}
        for k, p in params.items():
            g = grads[k].astype(F32)
            if not trigger:
                g = (g / g_norm * F32(self.max_norm)).astype(F32)
            self.mu[k] = (F32(1 - self.b1) * g + F32(self.b1) * self.mu[k]).astype(F32)
            self.nu[k] = (F32(1 - self.b2) * (g * g) + F32(self.b2) * self.nu[k]).astype(F32)
            u = (self.mu[k] / c1) / (np.sqrt(self.nu[k] / c2) + F32(self.eps))
            u = u + F32(self.wd) * p
            out[k] = (p - lr * u).astype(F32)
        return out


# ---- classic MADN: train_stochastic.py:25-180 -----------------------------------------------------------
def _softmax_ce(logits, probs):
    return -(probs.astype(np.float64) * _log_softmax(logits)).sum(-1)


def balanced_loss(ce, is_rare, mask, n_valid, w_rare=1.0, w_common=0.1):
    masked_rare = mask * is_rare
    n_rare = max(np.sum(masked_rare), 1.0)
    n_common = max(n_valid - n_rare, 1.0)
    return w_rare * np.sum(masked_rare * ce) / n_rare + w_common * np.sum((mask - masked_rare) * ce) / n_common


def loss_fn_stochastic(params, batch, unroll_steps=10):
    from . import classic_nets as CN
    latent = ON.representation(params, batch["observations"])
    K = batch["actions"].shape[1]
    B = latent.shape[0]
    acts = np.concatenate([batch["actions"], np.zeros((B, 1), np.int32)], 1)
    dice = np.concatenate([batch["dice_outcomes"][:, 1:], np.zeros((B, 2), np.int32)], 1)
    probs = np.concatenate([batch["dice_probs"], np.full((B, 1, 6), 1.0 / 6.0, np.float32)], 1)
    disc_t = np.concatenate([batch["discount_targets"], np.ones((B, 1), np.int32)], 1)
    rew_t = np.concatenate([batch["rewards"], np.ones((B, 1), np.int32)], 1)
    total = 0.0
    sums = [0.0] * 5
    for k in range(K + 1):
        mask = batch["masks"][:, k].astype(np.float64)
        logits, v = ON.prediction(params, latent)
        l_policy = np.mean(mask * -(batch["policies"][:, k].astype(np.float64) * _log_softmax(logits)).sum(-1))
        l_value = np.mean(mask * (batch["target_values"][:, k] - v[:, 0].astype(np.float64)) ** 2)
        l_chance = l_disc = l_rew = 0.0
        if k < K:
            n_valid = np.sum(mask)
            after, rl, cl, dl = CN.action_dynamics(params, latent, acts[:, k])
            rc, dc, tp = rew_t[:, k], disc_t[:, k], probs[:, k]
            l_rew = balanced_loss(_ce_int(rl, rc), (rc != 1).astype(np.float64), mask, n_valid)
            l_disc = balanced_loss(_ce_int(dl, dc), (dc == 1).astype(np.float64), mask, n_valid)
            nonu = (((tp.astype(np.float64) - 1.0 / 6.0) ** 2).sum(-1) > 1e-6).astype(np.float64)
            l_chance = balanced_loss(_softmax_ce(cl, tp), nonu, mask, n_valid)
            latent = CN.chance_dynamics(params, after, dice[:, k])
        total += (1.0 / unroll_steps) * (4.0 * l_value + 2.0 * l_policy + 0.5 * l_chance + 1.0 * l_disc + 1.0 * l_rew)
        for i, x in enumerate((l_value, l_policy, l_chance, l_disc, l_rew)):
            sums[i] += x
    return total, tuple(sums)
