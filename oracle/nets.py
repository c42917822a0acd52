"""CPU oracle: det-MADN MuZero networks in NumPy fp32 (TEST INFRASTRUCTURE ONLY).

Restates the three active Flax modules of MuZero_det_MADN/muzero_deterministic_madn.py:
  ResBlock 12-24, RepresentationNetwork2 75-141, DynamicsNetwork4 391-457,
  PredictionNetwork4 549-583, root_inference_fn 621-630, recurrent_inference_fn 632-661.
Flax 0.12.1 semantics (not vendored in the reference, restated from its public source):
  Dense y = x @ W + b (W[in, out]); Conv 1-D 'SAME' pads (k-1)//2 left; LayerNorm eps 1e-6
  with the fast variance  var = max(0, E[x^2] - E[x]^2),  y = (x - mean) * (rsqrt(var+eps)*scale) + bias.
Parity status: UNPINNED (flax is absent and the reference's .pkl checkpoints are missing);
the GPU kernels are checked against this restatement within a stated fp32 tolerance.

Parameters are a flat dict keyed by Flax paths, e.g. ``dynamics/ResBlock_0/Dense_1/kernel``.
"""
from __future__ import annotations

import numpy as np

LATENT = 256
EPS_LN = 1e-6
F32 = np.float32


# ---------------------------------------------------------------- parameter layout
def repr_param_shapes(C: int, head: str = "minmax") -> dict:
    """RepresentationNetwork2 parameter shapes for an observation of C channels (head "layernorm": the DOG
    RepresentationNetwork, MuZero_DOG/muzero_dog.py:25-83, whose last Dense is followed by LayerNorm_7)."""
    s = {}
    s["Conv_0/kernel"] = (3, 6, 32)
    s["Conv_0/bias"] = (32,)
    s["Conv_1/kernel"] = (3, 32, 64)
    s["Conv_1/bias"] = (64,)
    s["Conv_2/kernel"] = (5, 64, 64)
    s["Conv_2/bias"] = (64,)
    for i, n in enumerate([32, 64, 64, 256, 64, 64, 256]):
        s[f"LayerNorm_{i}/scale"] = (n,)
        s[f"LayerNorm_{i}/bias"] = (n,)
    for name, (i, o) in {"Dense_0": (56 * 64, 256), "Dense_1": (C - 6, 64), "Dense_2": (64, 64),
                         "Dense_3": (320, 256), "Dense_4": (256, 256)}.items():
        s[f"{name}/kernel"] = (i, o)
        s[f"{name}/bias"] = (o,)
    for r in range(6):
        _resblock_shapes(s, f"ResBlock_{r}")
    if head == "layernorm":
        s["LayerNorm_7/scale"] = (LATENT,)
        s["LayerNorm_7/bias"] = (LATENT,)
    return s


def _resblock_shapes(s, pre):
    for d in range(2):
        s[f"{pre}/Dense_{d}/kernel"] = (LATENT, LATENT)
        s[f"{pre}/Dense_{d}/bias"] = (LATENT,)
        s[f"{pre}/LayerNorm_{d}/scale"] = (LATENT,)
        s[f"{pre}/LayerNorm_{d}/bias"] = (LATENT,)


def dyn_param_shapes(A: int = 24) -> dict:
    """DynamicsNetwork4 parameter shapes."""
    s = {}
    dense = {"Dense_0": (A, 64), "Dense_1": (64, 256), "Dense_2": (64, 256), "Dense_3": (256, 256),
             "Dense_4": (256, 256), "Dense_5": (256, 256), "Dense_6": (256 + A, 64), "reward_head": (64, 3),
             "Dense_7": (256 + A, 64), "discount_head": (64, 3)}
    for name, (i, o) in dense.items():
        s[f"{name}/kernel"] = (i, o)
        s[f"{name}/bias"] = (o,)
    for i in range(3):
        s[f"LayerNorm_{i}/scale"] = (LATENT,)
        s[f"LayerNorm_{i}/bias"] = (LATENT,)
    for r in range(2):
        _resblock_shapes(s, f"ResBlock_{r}")
    return s


def pred_param_shapes(A: int = 24) -> dict:
    """PredictionNetwork4 parameter shapes."""
    s = {}
    dense = {"Dense_0": (256, 256), "Dense_1": (256, 128), "Dense_2": (128, A), "Dense_3": (256, 128),
             "Dense_4": (128, 64), "Dense_5": (64, 1)}
    for name, (i, o) in dense.items():
        s[f"{name}/kernel"] = (i, o)
        s[f"{name}/bias"] = (o,)
    for i, n in enumerate([256, 256, 128, 128]):
        s[f"LayerNorm_{i}/scale"] = (n,)
        s[f"LayerNorm_{i}/bias"] = (n,)
    for r in range(2):
        _resblock_shapes(s, f"ResBlock_{r}")
    return s


def param_shapes(C: int, A: int = 24, head: str = "minmax") -> dict:
    out = {}
    for net, shapes in (("representation", repr_param_shapes(C, head)), ("dynamics", dyn_param_shapes(A)),
                        ("prediction", pred_param_shapes(A))):
        for k, v in shapes.items():
            out[f"{net}/{k}"] = v
    return out


def init_params(C: int, A: int = 24, seed: int = 0, randomize_affine: bool = False, head: str = "minmax") -> dict:
    """Seeded Flax-default-like init: lecun_normal (truncated) kernels, zero biases, unit LN scale.

    ``randomize_affine`` also draws non-trivial biases / LN scales+biases so parity tests
    exercise every parameter.  (The reference's jax threefry init is not reproducible here.)"""
    rng = np.random.default_rng(seed)
    p = {}
    for k, shp in param_shapes(C, A, head).items():
        if k.endswith("kernel"):
            fan_in = int(np.prod(shp[:-1]))
            std = np.sqrt(1.0 / fan_in) / 0.87962566103423978
            w = rng.standard_normal(shp)
            w = np.clip(w, -2.0, 2.0)
            p[k] = (w * std).astype(F32)
        elif k.endswith("scale"):
            p[k] = (np.ones(shp) + (0.1 * rng.standard_normal(shp) if randomize_affine else 0.0)).astype(F32)
        else:
            p[k] = (0.05 * rng.standard_normal(shp) if randomize_affine else np.zeros(shp)).astype(F32)
    return p


def sub(params: dict, prefix: str) -> dict:
    n = len(prefix) + 1
    return {k[n:]: v for k, v in params.items() if k.startswith(prefix + "/")}


# ---------------------------------------------------------------- layers
def dense(p, name, x):
    return (x.astype(F32) @ p[f"{name}/kernel"] + p[f"{name}/bias"]).astype(F32)


def layer_norm(p, name, x):
    x = x.astype(F32)
    mean = x.mean(-1, keepdims=True, dtype=F32)
    mean2 = (x * x).mean(-1, keepdims=True, dtype=F32)
    var = np.maximum(F32(0.0), mean2 - mean * mean)
    mul = (F32(1.0) / np.sqrt(var + F32(EPS_LN))).astype(F32) * p[f"{name}/scale"]
    return ((x - mean) * mul + p[f"{name}/bias"]).astype(F32)


def relu(x):
    return np.maximum(x, F32(0.0))


def conv1d_same(p, name, x):
    """Flax Conv, 1-D NWC, padding 'SAME', stride 1 (cross-correlation)."""
    k = p[f"{name}/kernel"]        # (K, Cin, Cout)
    K = k.shape[0]
    pl = (K - 1) // 2
    pr = K - 1 - pl
    B, W, Cin = x.shape
    xp = np.zeros((B, W + K - 1, Cin), F32)
    xp[:, pl:pl + W] = x
    cols = np.concatenate([xp[:, d:d + W, :] for d in range(K)], axis=-1)   # (B, W, K*Cin)
    return (cols @ k.reshape(K * Cin, -1) + p[f"{name}/bias"]).astype(F32)


def resblock(p, name, x):
    r = x
    y = relu(layer_norm(p, f"{name}/LayerNorm_0", dense(p, f"{name}/Dense_0", x)))
    y = layer_norm(p, f"{name}/LayerNorm_1", dense(p, f"{name}/Dense_1", y))
    return relu(r + y)


def minmax(x):
    lo = x.min(-1, keepdims=True)
    hi = x.max(-1, keepdims=True)
    return ((x - lo) / (hi - lo + F32(1e-8))).astype(F32)


# ---------------------------------------------------------------- networks
def representation(params: dict, obs: np.ndarray) -> np.ndarray:
    """RepresentationNetwork2 (muzero_deterministic_madn.py:75-141). obs [B, C, 56] -> [B, 256].  With a
    ``representation/LayerNorm_7`` entry it is the DOG RepresentationNetwork (MuZero_DOG/muzero_dog.py:25-83):
    the same trunk, LayerNorm instead of min-max after the last Dense (80-81)."""
    p = sub(params, "representation")
    x = obs.astype(F32)
    sp = np.transpose(x[:, :6, :], (0, 2, 1))            # (B, 56, 6)
    g = x[:, 6:, 0]                                      # (B, C-6)
    sp = relu(layer_norm(p, "LayerNorm_0", conv1d_same(p, "Conv_0", sp)))
    sp = relu(layer_norm(p, "LayerNorm_1", conv1d_same(p, "Conv_1", sp)))
    sp = relu(layer_norm(p, "LayerNorm_2", conv1d_same(p, "Conv_2", sp)))
    flat = sp.reshape(sp.shape[0], -1)
    flat = relu(layer_norm(p, "LayerNorm_3", dense(p, "Dense_0", flat)))
    g = relu(layer_norm(p, "LayerNorm_4", dense(p, "Dense_1", g)))
    g = relu(layer_norm(p, "LayerNorm_5", dense(p, "Dense_2", g)))
    h = relu(layer_norm(p, "LayerNorm_6", dense(p, "Dense_3", np.concatenate([flat, g], -1))))
    for r in range(6):
        h = resblock(p, f"ResBlock_{r}", h)
    if "LayerNorm_7/scale" in p:
        return layer_norm(p, "LayerNorm_7", dense(p, "Dense_4", h))
    return minmax(dense(p, "Dense_4", h))


def one_hot(a, n):
    a = np.asarray(a)
    out = np.zeros(a.shape + (n,), F32)
    ok = (a >= 0) & (a < n)
    out[ok, a[ok]] = 1.0      # jax.nn.one_hot: out-of-range (e.g. -1) -> all-zero row
    return out


def dynamics(params: dict, latent: np.ndarray, action: np.ndarray, A: int | None = None):
    """DynamicsNetwork4 (muzero_deterministic_madn.py:391-457) -> (next_latent, reward_logits, discount_logits).
    A (the one-hot width) defaults to the parameters' own (Dense_0's input rows)."""
    p = sub(params, "dynamics")
    A = p["Dense_0/kernel"].shape[0] if A is None else A
    oh = one_hot(action, A)
    e = relu(dense(p, "Dense_0", oh))
    ln = layer_norm(p, "LayerNorm_0", latent)
    scale = dense(p, "Dense_1", e)
    shift = dense(p, "Dense_2", e)
    x = (ln * (F32(1.0) + scale) + shift).astype(F32)
    x = relu(layer_norm(p, "LayerNorm_1", dense(p, "Dense_3", x)))
    x = relu(layer_norm(p, "LayerNorm_2", dense(p, "Dense_4", x)))
    for r in range(2):
        x = resblock(p, f"ResBlock_{r}", x)
    x = dense(p, "Dense_5", x)
    nxt = minmax((latent + x).astype(F32))
    ri = np.concatenate([nxt, oh], -1)
    rl = dense(p, "reward_head", relu(dense(p, "Dense_6", ri)))
    dl = dense(p, "discount_head", relu(dense(p, "Dense_7", ri)))
    return nxt, rl, dl


def prediction(params: dict, latent: np.ndarray):
    """PredictionNetwork4 (muzero_deterministic_madn.py:549-583) -> (policy_logits [B,A], value [B,1])."""
    p = sub(params, "prediction")
    x = layer_norm(p, "LayerNorm_0", latent)
    for r in range(2):
        x = resblock(p, f"ResBlock_{r}", x)
    pol = relu(layer_norm(p, "LayerNorm_1", dense(p, "Dense_0", x)))
    pol = relu(layer_norm(p, "LayerNorm_2", dense(p, "Dense_1", pol)))
    logits = dense(p, "Dense_2", pol)
    v = relu(layer_norm(p, "LayerNorm_3", dense(p, "Dense_3", x)))
    v = relu(dense(p, "Dense_4", v))
    v = np.tanh(dense(p, "Dense_5", v)).astype(F32)
    return logits, v


def softmax(x, axis=-1):
    x = x.astype(F32)
    u = np.exp(x - x.max(axis, keepdims=True))
    return (u / u.sum(axis, keepdims=True)).astype(F32)


SUPPORT = np.array([-1.0, 0.0, 1.0], F32)


def root_inference(params, obs):
    """root_inference_fn (muzero_deterministic_madn.py:621-630) -> (prior_logits, value, embedding)."""
    emb = representation(params, obs)
    logits, v = prediction(params, emb)
    return logits, v[:, 0], emb


def recurrent_inference(params, action, emb):
    """recurrent_inference_fn (muzero_deterministic_madn.py:632-661)
    -> (reward, discount, prior_logits, value, next_embedding)."""
    nxt, rl, dl = dynamics(params, emb, action)
    logits, v = prediction(params, nxt)
    reward = (softmax(rl) * SUPPORT).sum(-1).astype(F32)
    discount = (softmax(dl) * SUPPORT).sum(-1).astype(F32)
    return reward, discount, logits, v[:, 0], nxt
