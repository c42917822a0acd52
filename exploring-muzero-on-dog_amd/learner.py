"""Learner for det-MADN MuZero: train_step of MuZero_det_MADN/train_with_reward.py in torch (autograd).

The learner sits beside the self-play hot path (SURVEY §8f "next"): it consumes batches straight from
the device replay ring (replay.VectorizedReplayBuffer.sample_batch -> device tensors, no host copy) and
hands new weights back to the self-play engine as one packed arena (``push_to``).  Reference functions
mirrored:

  repr_net / dynamics_net / pred_net   muzero_deterministic_madn.py:75-141, 391-457, 549-583 (Flax
                                       semantics: fast-variance LayerNorm eps 1e-6, 'SAME' Conv1D,
                                       one_hot of an out-of-range action = 0, min-max latent scaling)
  loss_fn                              train_with_reward.py:24-141
  train_step                           train_with_reward.py:148-162
  optimizer                            train_with_reward.py:361-372: clip_by_global_norm(5.0) ->
                                       adamw(piecewise-constant lr 0.005, x0.2 @ it 30, x0.2 @ 60,
                                       x0.5 @ 85 of 2500 steps, weight decay 1e-4), optax semantics
  test_training loop                   train_with_reward.py:167-311 (``train_loop``)

Parameters are kept under the Flax path names of nets.param_shapes, so the same dict packs into the
self-play kernels' arena (nets.DeviceNet).  Everything is fp32.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import nets as N

EPS_LN = 1e-6
VALUE_SCALING, POLICY_SCALING, DISCOUNT_SCALING, REWARD_SCALING = 4.0, 1.0, 1.0, 1.0


class MuZeroNets:
    """Flax-named fp32 parameters of (RepresentationNetwork2, DynamicsNetwork4, PredictionNetwork4)."""

    def __init__(self, params: dict, obs_channels: int, num_actions: int = 24, device="cuda",
                 dtype=torch.float32):
        self.C, self.A = int(obs_channels), int(num_actions)
        shapes = N.param_shapes(self.C, self.A)
        if set(shapes) != set(params):
            raise ValueError("parameter names differ from nets.param_shapes")
        self.p = {k: torch.tensor(np.asarray(params[k]).reshape(shapes[k]), dtype=dtype, device=device,
                                  requires_grad=True) for k in shapes}

    def parameters(self):
        return list(self.p.values())

    def numpy(self) -> dict:
        return {k: v.detach().float().cpu().numpy() for k, v in self.p.items()}

    # ---- layers (oracle/nets.py restates the same Flax semantics) ----------------------------------
    def _dense(self, name, x):
        return x @ self.p[f"{name}/kernel"] + self.p[f"{name}/bias"]

    def _ln(self, name, x):
        mean = x.mean(-1, keepdim=True)
        mean2 = (x * x).mean(-1, keepdim=True)
        var = torch.clamp(mean2 - mean * mean, min=0.0)
        return (x - mean) * (torch.rsqrt(var + EPS_LN) * self.p[f"{name}/scale"]) + self.p[f"{name}/bias"]

    def _conv(self, name, x):
        """Flax Conv 'SAME', stride 1, NWC input [B, W, Cin] -> [B, W, Cout]."""
        k = self.p[f"{name}/kernel"]            # (K, Cin, Cout)
        K = k.shape[0]
        pl = (K - 1) // 2
        y = F.conv1d(F.pad(x.transpose(1, 2), (pl, K - 1 - pl)), k.permute(2, 1, 0), self.p[f"{name}/bias"])
        return y.transpose(1, 2)

    def _rb(self, name, x):
        y = F.relu(self._ln(f"{name}/LayerNorm_0", self._dense(f"{name}/Dense_0", x)))
        y = self._ln(f"{name}/LayerNorm_1", self._dense(f"{name}/Dense_1", y))
        return F.relu(x + y)

    @staticmethod
    def _minmax(x):
        lo = x.min(-1, keepdim=True).values
        hi = x.max(-1, keepdim=True).values
        return (x - lo) / (hi - lo + 1e-8)

    # ---- networks ------------------------------------------------------------------------------------
    def representation(self, obs):
        r = "representation"
        sp = obs[:, :6, :].transpose(1, 2)
        g = obs[:, 6:, 0]
        for i in range(3):
            sp = F.relu(self._ln(f"{r}/LayerNorm_{i}", self._conv(f"{r}/Conv_{i}", sp)))
        flat = F.relu(self._ln(f"{r}/LayerNorm_3", self._dense(f"{r}/Dense_0", sp.reshape(sp.shape[0], -1))))
        g = F.relu(self._ln(f"{r}/LayerNorm_4", self._dense(f"{r}/Dense_1", g)))
        g = F.relu(self._ln(f"{r}/LayerNorm_5", self._dense(f"{r}/Dense_2", g)))
        h = F.relu(self._ln(f"{r}/LayerNorm_6", self._dense(f"{r}/Dense_3", torch.cat([flat, g], -1))))
        for b in range(6):
            h = self._rb(f"{r}/ResBlock_{b}", h)
        return self._minmax(self._dense(f"{r}/Dense_4", h))

    def dynamics(self, latent, action):
        d = "dynamics"
        oh = (action.long()[:, None] == torch.arange(self.A, device=latent.device)[None, :]).to(latent.dtype)
        e = F.relu(self._dense(f"{d}/Dense_0", oh))
        x = self._ln(f"{d}/LayerNorm_0", latent) * (1.0 + self._dense(f"{d}/Dense_1", e)) + self._dense(f"{d}/Dense_2", e)
        x = F.relu(self._ln(f"{d}/LayerNorm_1", self._dense(f"{d}/Dense_3", x)))
        x = F.relu(self._ln(f"{d}/LayerNorm_2", self._dense(f"{d}/Dense_4", x)))
        for b in range(2):
            x = self._rb(f"{d}/ResBlock_{b}", x)
        nxt = self._minmax(latent + self._dense(f"{d}/Dense_5", x))
        ri = torch.cat([nxt, oh], -1)
        rl = self._dense(f"{d}/reward_head", F.relu(self._dense(f"{d}/Dense_6", ri)))
        dl = self._dense(f"{d}/discount_head", F.relu(self._dense(f"{d}/Dense_7", ri)))
        return nxt, rl, dl

    def prediction(self, latent):
        p = "prediction"
        x = self._ln(f"{p}/LayerNorm_0", latent)
        for b in range(2):
            x = self._rb(f"{p}/ResBlock_{b}", x)
        pol = F.relu(self._ln(f"{p}/LayerNorm_1", self._dense(f"{p}/Dense_0", x)))
        pol = F.relu(self._ln(f"{p}/LayerNorm_2", self._dense(f"{p}/Dense_1", pol)))
        logits = self._dense(f"{p}/Dense_2", pol)
        v = F.relu(self._ln(f"{p}/LayerNorm_3", self._dense(f"{p}/Dense_3", x)))
        v = F.relu(self._dense(f"{p}/Dense_4", v))
        return logits, torch.tanh(self._dense(f"{p}/Dense_5", v))


def _balanced_ce(logits, labels, mask, special, w_special, w_other):
    """Per-class balanced cross-entropy (train_with_reward.py:54-86)."""
    ce = F.cross_entropy(logits, labels.long(), reduction="none")
    is_s = labels == special
    n_s = torch.clamp((mask * is_s).sum(), min=1.0)
    n_o = torch.clamp((mask * ~is_s).sum(), min=1.0)
    return (w_special * (mask * torch.where(is_s, ce, torch.zeros_like(ce))).sum() / n_s +
            w_other * (mask * torch.where(~is_s, ce, torch.zeros_like(ce))).sum() / n_o)


def loss_fn(nets: MuZeroNets, batch: dict, unroll_steps: int = 10, grad_scale: float = 0.5):
    """train_with_reward.py:24-141 -> (total_loss, (value_loss, policy_loss, discount_loss, reward_loss)).
    grad_scale: the gradient share carried through the unrolled latent (0.5 in the reference, line 106;
    the forward value does not depend on it)."""
    obs = batch["observations"].to(nets.p["prediction/Dense_5/bias"].dtype)
    latent = nets.representation(obs)
    B, K = batch["actions"].shape
    dev = obs.device
    acts = torch.cat([batch["actions"], torch.zeros((B, 1), dtype=batch["actions"].dtype, device=dev)], 1)
    ones = torch.ones((B, 1), dtype=torch.int32, device=dev)
    disc_t = torch.cat([batch["discount_targets"].int(), ones], 1)
    rew_t = torch.cat([batch["rewards"].int(), ones], 1)
    total = torch.zeros((), dtype=obs.dtype, device=dev)
    sums = [torch.zeros((), dtype=obs.dtype, device=dev) for _ in range(4)]
    for k in range(K + 1):
        mask = batch["masks"][:, k].to(obs.dtype)
        logits, v = nets.prediction(latent)
        l_value = torch.mean(mask * (batch["target_values"][:, k].to(obs.dtype) - v[:, 0]) ** 2)
        l_policy = torch.mean(mask * -(batch["policies"][:, k].to(obs.dtype) * F.log_softmax(logits, -1)).sum(-1))
        step = (1.0 / unroll_steps) * (VALUE_SCALING * l_value + POLICY_SCALING * l_policy)
        if k < K:
            nxt, rl, dl = nets.dynamics(latent, acts[:, k])
            l_rew = _balanced_ce(rl, rew_t[:, k], mask, 1, 0.1, 1.0)        # neutral 0.1, win/lose 1.0
            l_disc = _balanced_ce(dl, disc_t[:, k], mask, 1, 1.0, 0.1)      # terminal 1.0, other 0.1
        else:
            nxt, l_rew, l_disc = latent, torch.zeros((), dtype=obs.dtype, device=dev), \
                torch.zeros((), dtype=obs.dtype, device=dev)
        total = total + step + (1.0 / unroll_steps) * DISCOUNT_SCALING * l_disc + \
            (1.0 / unroll_steps) * REWARD_SCALING * l_rew
        latent = (nxt * (1.0 - grad_scale)).detach() + nxt * grad_scale   # gradient scaling (forward identity)
        for i, x in enumerate((l_value, l_policy, l_disc, l_rew)):
            sums[i] = sums[i] + x
    return total, tuple(sums)


def lr_schedule(step: int, lr0: float = 0.005, steps_per_iteration: int = 2500) -> float:
    """optax.piecewise_constant_schedule (train_with_reward.py:361-368)."""
    lr = lr0
    for boundary, scale in ((30, 0.2), (60, 0.2), (85, 0.5)):
        if step >= boundary * steps_per_iteration:
            lr *= scale
    return lr


class AdamW:
    """optax.chain(clip_by_global_norm(5.0), adamw(schedule, b1 0.9, b2 0.999, eps 1e-8, weight_decay 1e-4))."""

    def __init__(self, params: list, max_norm=5.0, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4, schedule=lr_schedule):
        self.params = params
        self.mu = [torch.zeros_like(p) for p in params]
        self.nu = [torch.zeros_like(p) for p in params]
        self.count = 0
        self.max_norm, self.b1, self.b2, self.eps, self.wd, self.schedule = max_norm, b1, b2, eps, wd, schedule

    @torch.no_grad()
    def step(self):
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        g_norm = torch.sqrt(sum(torch.sum(g * g) for g in grads))
        lr = self.schedule(self.count)
        self.count += 1
        c1, c2 = 1.0 - self.b1 ** self.count, 1.0 - self.b2 ** self.count
        for p, g, m, v in zip(self.params, grads, self.mu, self.nu):
            g = torch.where(g_norm < self.max_norm, g, g / g_norm * self.max_norm)
            m.mul_(self.b1).add_((1 - self.b1) * g)
            v.mul_(self.b2).add_((1 - self.b2) * (g * g))
            u = (m / c1) / (torch.sqrt(v / c2) + self.eps) + self.wd * p
            p.sub_(lr * u)
        return g_norm


class Learner:
    """train_step (train_with_reward.py:148-162) on batches sampled from the device ring."""

    def __init__(self, params: dict, obs_channels: int, num_actions: int = 24, unroll_steps: int = 10,
                 device="cuda", **opt):
        self.nets = MuZeroNets(params, obs_channels, num_actions, device)
        self.opt = AdamW(self.nets.parameters(), **opt)
        self.unroll_steps = int(unroll_steps)

    def train_step(self, batch: dict) -> dict:
        for p in self.nets.parameters():
            p.grad = None
        loss, (v, pl, d, r) = loss_fn(self.nets, batch, self.unroll_steps)
        loss.backward()
        self.opt.step()
        return {"total_loss": loss.detach(), "v_loss": v.detach(), "p_loss": pl.detach(), "d_loss": d.detach(),
                "r_loss": r.detach()}

    def push_to(self, net: "N.DeviceNet"):
        """Pack the current parameters into the self-play engine's arena (same layout) in place."""
        fresh = N.DeviceNet(self.nets.numpy(), net.C, net.A, device=net.buffer.device)
        net.buffer.copy_(fresh.buffer)
        net.prepare()


def train_loop(learner: Learner, engine, ring, iterations: int, train_steps: int, games_per_iteration: int,
               temperature_schedule=(2.0, 1.5, 1.0, 0.8, 0.6), seed: int = 42, warmup_calls: int = 3):
    """test_training (train_with_reward.py:167-311) with the device engine: streamed self-play into the
    ring, train_steps sampled batches per iteration, new weights pushed to the engine each iteration."""
    def temp(it):
        ph = min(int(it / max(iterations, 1) * len(temperature_schedule)), len(temperature_schedule) - 1)
        return temperature_schedule[ph]

    for n in range(warmup_calls):
        ring.save_games_from_buffers(engine.play_stream(games_per_iteration, seed * n, temp(0)))
    history = []
    for it in range(iterations):
        ring.save_games_from_buffers(engine.play_stream(games_per_iteration, seed + it ** 3, temp(it)))
        for _ in range(train_steps):
            losses = learner.train_step(ring.sample_batch())
        learner.push_to(engine.net)
        history.append({k: float(v) for k, v in losses.items()})
    return history
