"""CPU oracle: classic-MADN Stochastic MuZero networks in NumPy fp32 (TEST INFRASTRUCTURE ONLY).

Restates MuZero_Classic_MADN/muzero_classic_madn.py:
  RepresentationNetwork2 69-135 (identical to the det file's, reused from oracle.nets),
  PredictionNetwork4 192-226 (A = 4, reused from oracle.nets),
  StochasticDynamicsNetwork4 314-408 (action_dynamics 329-371, chance_dynamics 373-408),
  decision_recurrent_fn 414-432, chance_recurrent_fn 434-451, root_inference_fn 453-462.
Flax semantics as in oracle.nets.  Parameter paths: the module's explicit names
(``dynamics/act_embed/kernel`` ...); the four anonymous ResBlocks are ``ResBlock_0..1`` (action
dynamics) and ``ResBlock_2..3`` (chance dynamics).
Parity status: UNPINNED (flax absent, no classic checkpoints in the reference).
"""
from __future__ import annotations

import numpy as np

from .nets import (F32, LATENT, SUPPORT, _resblock_shapes, dense, layer_norm, minmax, one_hot, pred_param_shapes,
                   prediction, relu, repr_param_shapes, representation, resblock, softmax, sub)

A_CLASSIC = 4
CHANCE = 6


def sdyn_param_shapes(A: int = A_CLASSIC, C: int = CHANCE) -> dict:
    s = {}
    dense_l = {"act_embed": (A, 64), "act_film_scale": (64, LATENT), "act_film_shift": (64, LATENT),
               "act_dense1": (LATENT, LATENT), "act_dense2": (LATENT, LATENT), "act_proj": (LATENT, LATENT),
               "reward_dense": (LATENT + A, 64), "reward_head": (64, 3), "discount_dense": (LATENT, 32),
               "discount_head": (32, 3), "chance_head": (LATENT, C),
               "chance_embed": (C, 64), "chance_film_scale": (64, LATENT), "chance_film_shift": (64, LATENT),
               "chance_dense1": (LATENT, LATENT), "chance_dense2": (LATENT, LATENT), "chance_proj": (LATENT, LATENT)}
    for name, (i, o) in dense_l.items():
        s[f"{name}/kernel"] = (i, o)
        s[f"{name}/bias"] = (o,)
    for name, n in {"act_input_ln": LATENT, "act_ln1": LATENT, "act_ln2": LATENT, "discount_ln": 32,
                    "chance_input_ln": LATENT, "chance_ln1": LATENT, "chance_ln2": LATENT}.items():
        s[f"{name}/scale"] = (n,)
        s[f"{name}/bias"] = (n,)
    for r in range(4):
        _resblock_shapes(s, f"ResBlock_{r}")
    return s


def param_shapes(C_obs: int, A: int = A_CLASSIC) -> dict:
    out = {}
    for net, shapes in (("representation", repr_param_shapes(C_obs)), ("dynamics", sdyn_param_shapes(A)),
                        ("prediction", pred_param_shapes(A))):
        for k, v in shapes.items():
            out[f"{net}/{k}"] = v
    return out


def init_params(C_obs: int = 11, seed: int = 0, randomize_affine: bool = False) -> dict:
    """Same recipe as oracle.nets.init_params (lecun-normal kernels, zero / unit affine)."""
    rng = np.random.default_rng(seed)
    p = {}
    for k, shp in param_shapes(C_obs).items():
        if k.endswith("kernel"):
            fan_in = int(np.prod(shp[:-1]))
            std = np.sqrt(1.0 / fan_in) / 0.87962566103423978
            p[k] = (np.clip(rng.standard_normal(shp), -2.0, 2.0) * std).astype(F32)
        elif k.endswith("scale"):
            p[k] = (np.ones(shp) + (0.1 * rng.standard_normal(shp) if randomize_affine else 0.0)).astype(F32)
        else:
            p[k] = (0.05 * rng.standard_normal(shp) if randomize_affine else np.zeros(shp)).astype(F32)
    return p


def _film_trunk(p, pre, rb0, x_in, e):
    """LN(input) * (1 + scale(e)) + shift(e) -> dense1/LN/relu -> dense2/LN/relu -> 2 ResBlocks -> proj,
    + input skip, min-max over features (lines 339-360 / 381-406)."""
    ln = layer_norm(p, f"{pre}_input_ln", x_in)
    x = (ln * (F32(1.0) + dense(p, f"{pre}_film_scale", e)) + dense(p, f"{pre}_film_shift", e)).astype(F32)
    x = relu(layer_norm(p, f"{pre}_ln1", dense(p, f"{pre}_dense1", x)))
    x = relu(layer_norm(p, f"{pre}_ln2", dense(p, f"{pre}_dense2", x)))
    for r in range(rb0, rb0 + 2):
        x = resblock(p, f"ResBlock_{r}", x)
    x = dense(p, f"{pre}_proj", x)
    return minmax((x_in + x).astype(F32))


def action_dynamics(params, latent, action, A: int = A_CLASSIC):
    """StochasticDynamicsNetwork4.action_dynamics (329-371)
    -> (afterstate, reward_logits [B,3], chance_logits [B,6], discount_logits [B,3])."""
    p = sub(params, "dynamics")
    oh = one_hot(action, A)
    e = relu(dense(p, "act_embed", oh))
    after = _film_trunk(p, "act", 0, latent.astype(F32), e)
    rl = dense(p, "reward_head", relu(dense(p, "reward_dense", np.concatenate([after, oh], -1))))
    dl = dense(p, "discount_head", relu(layer_norm(p, "discount_ln", dense(p, "discount_dense", latent))))
    cl = dense(p, "chance_head", after)
    return after, rl, cl, dl


def chance_dynamics(params, afterstate, chance, C: int = CHANCE):
    """StochasticDynamicsNetwork4.chance_dynamics (373-408) -> next_state."""
    p = sub(params, "dynamics")
    e = relu(dense(p, "chance_embed", one_hot(chance, C)))
    return _film_trunk(p, "chance", 2, afterstate.astype(F32), e)


def root_inference(params, obs):
    """root_inference_fn (453-462) -> (prior_logits [B,4], value [B], embedding)."""
    emb = representation(params, obs)
    logits, v = prediction(params, emb)
    return logits, v[:, 0], emb


def decision_recurrent(params, action, emb):
    """decision_recurrent_fn (414-432) -> (chance_logits, afterstate_value, afterstate, reward, discount);
    the reference concatenates reward / discount to the afterstate (258 floats)."""
    after, rl, cl, dl = action_dynamics(params, emb, action)
    reward = (softmax(rl) * SUPPORT).sum(-1).astype(F32)
    discount = (softmax(dl) * SUPPORT).sum(-1).astype(F32)
    _, v = prediction(params, after)
    return cl, v[:, 0], after, reward, discount


def chance_recurrent(params, chance, afterstate):
    """chance_recurrent_fn (434-451) -> (action_logits, value, next_embedding); reward / discount come
    from the afterstate's extra floats."""
    nxt = chance_dynamics(params, afterstate, chance)
    logits, v = prediction(params, nxt)
    return logits, v[:, 0], nxt
