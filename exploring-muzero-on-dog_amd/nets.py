"""MuZero networks of MuZero_det_MADN/muzero_deterministic_madn.py on the GPU.

Host side of the fused fp32 MFMA network kernels (csrc/nets.hip, csrc/nn.hpp):
  * parameter init / layout follow the Flax module tree (paths such as
    ``dynamics/ResBlock_0/Dense_1/kernel``), so checkpoints map 1:1 (init_muzero_params,
    lines 706-748);
  * ``DeviceNet`` packs the dense kernels into the MFMA B-fragment layout documented in
    include/muz.h, uploads everything as one device buffer and fills ``muz_net_w``;
  * ``root_inference_fn`` / ``recurrent_inference_fn`` mirror lines 621-661.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import lib as _L
from .lib import MuzNetW  # struct layout of include/muz.h

LATENT = 256


# ---------------------------------------------------------------------------------- parameters
def _resblock_shapes(s, pre):
    for d in range(2):
        s[f"{pre}/Dense_{d}/kernel"] = (LATENT, LATENT)
        s[f"{pre}/Dense_{d}/bias"] = (LATENT,)
        s[f"{pre}/LayerNorm_{d}/scale"] = (LATENT,)
        s[f"{pre}/LayerNorm_{d}/bias"] = (LATENT,)


def param_shapes(obs_channels: int, num_actions: int = 24) -> dict:
    """Flax parameter tree of (RepresentationNetwork2, DynamicsNetwork4, PredictionNetwork4), flattened."""
    C, A = obs_channels, num_actions
    s = {}
    r = "representation"
    s[f"{r}/Conv_0/kernel"], s[f"{r}/Conv_0/bias"] = (3, 6, 32), (32,)
    s[f"{r}/Conv_1/kernel"], s[f"{r}/Conv_1/bias"] = (3, 32, 64), (64,)
    s[f"{r}/Conv_2/kernel"], s[f"{r}/Conv_2/bias"] = (5, 64, 64), (64,)
    for i, n in enumerate([32, 64, 64, 256, 64, 64, 256]):
        s[f"{r}/LayerNorm_{i}/scale"] = s[f"{r}/LayerNorm_{i}/bias"] = (n,)
    for name, (i, o) in {"Dense_0": (56 * 64, 256), "Dense_1": (C - 6, 64), "Dense_2": (64, 64),
                         "Dense_3": (320, 256), "Dense_4": (256, 256)}.items():
        s[f"{r}/{name}/kernel"], s[f"{r}/{name}/bias"] = (i, o), (o,)
    for b in range(6):
        _resblock_shapes(s, f"{r}/ResBlock_{b}")
    d = "dynamics"
    for name, (i, o) in {"Dense_0": (A, 64), "Dense_1": (64, 256), "Dense_2": (64, 256), "Dense_3": (256, 256),
                         "Dense_4": (256, 256), "Dense_5": (256, 256), "Dense_6": (256 + A, 64),
                         "reward_head": (64, 3), "Dense_7": (256 + A, 64), "discount_head": (64, 3)}.items():
        s[f"{d}/{name}/kernel"], s[f"{d}/{name}/bias"] = (i, o), (o,)
    for i in range(3):
        s[f"{d}/LayerNorm_{i}/scale"] = s[f"{d}/LayerNorm_{i}/bias"] = (LATENT,)
    for b in range(2):
        _resblock_shapes(s, f"{d}/ResBlock_{b}")
    p = "prediction"
    for name, (i, o) in {"Dense_0": (256, 256), "Dense_1": (256, 128), "Dense_2": (128, A), "Dense_3": (256, 128),
                         "Dense_4": (128, 64), "Dense_5": (64, 1)}.items():
        s[f"{p}/{name}/kernel"], s[f"{p}/{name}/bias"] = (i, o), (o,)
    for i, n in enumerate([256, 256, 128, 128]):
        s[f"{p}/LayerNorm_{i}/scale"] = s[f"{p}/LayerNorm_{i}/bias"] = (n,)
    for b in range(2):
        _resblock_shapes(s, f"{p}/ResBlock_{b}")
    return s


def init_muzero_params(seed: int, obs_channels: int, num_actions: int = 24) -> dict:
    """init_muzero_params (lines 706-748) with Flax defaults: lecun_normal kernels (truncated at 2 std),
    zero biases, unit LayerNorm scales.  Seeded NumPy draws (jax threefry is not reproduced)."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, shp in param_shapes(obs_channels, num_actions).items():
        if k.endswith("kernel"):
            fan_in = int(np.prod(shp[:-1]))
            std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
            out[k] = (np.clip(rng.standard_normal(shp), -2.0, 2.0) * std).astype(np.float32)
        elif k.endswith("scale"):
            out[k] = np.ones(shp, np.float32)
        else:
            out[k] = np.zeros(shp, np.float32)
    return out


# ---------------------------------------------------------------------------------- packing
def nt_for(N: int, nw: int) -> int:
    """16-column MFMA tiles per wave for a layer of N outputs split over nw waves (csrc/nn.hpp:nt_for)."""
    return -(-N // (16 * nw))


def pack_dense(W: np.ndarray, nw: int, nt: int) -> np.ndarray:
    """MFMA 16x16x4 B-fragment packing (layout documented in include/muz.h):
    out[w][kb][lane][t][j] = W[kb*16 + 4*(lane>>4) + j][(w*nt + t)*16 + (lane&15)]."""
    W = np.asarray(W, np.float32)
    K, N = W.shape
    KB = (K + 15) // 16
    Np = nw * nt * 16
    if N > Np:
        raise ValueError(f"N={N} does not fit {nw} groups x {nt} tiles")
    Wp = np.zeros((KB * 16, Np), np.float32)
    Wp[:K, :N] = W
    arr = Wp.reshape(KB, 4, 4, nw, nt, 16).transpose(3, 0, 1, 5, 4, 2)
    return np.ascontiguousarray(arr).reshape(-1)


class _Packer:
    """Builds one device buffer of packed parameters and fills a ctypes weight table from a nested spec
    (leaf = offset in floats, (w, b) pair = muz_dense / muz_ln, list = array field, dict = sub-struct)."""

    def __init__(self, params: dict, obs_channels: int, num_actions: int):
        self.C, self.A = int(obs_channels), int(num_actions)
        self.waves = _L.load().muz_tile_waves()   # column groups of the packed 16-row layers (csrc/nn.hpp kWaves)
        self._chunks = []
        self._off = 0
        self.params = {k: np.asarray(v, np.float32) for k, v in params.items()}

    def _put(self, arr) -> int:
        a = np.ascontiguousarray(np.asarray(arr, np.float32).reshape(-1))
        pad = (-a.size) % 4          # keep every array 16-byte aligned for f32x4 loads
        if pad:
            a = np.concatenate([a, np.zeros(pad, np.float32)])
        off = self._off
        self._chunks.append(a)
        self._off += a.size
        return off

    def _dense_k(self, k, b):
        return (self._put(pack_dense(k, self.waves, nt_for(k.shape[1], self.waves))), self._put(b))

    def _dense(self, name):
        return self._dense_k(self.params[f"{name}/kernel"], self.params[f"{name}/bias"])

    def _plain(self, name):
        return (self._put(self.params[f"{name}/kernel"]), self._put(self.params[f"{name}/bias"]))

    def _ln(self, name):
        return (self._put(self.params[f"{name}/scale"]), self._put(self.params[f"{name}/bias"]))

    def _rb(self, pre):
        return dict(d0=self._dense(f"{pre}/Dense_0"), ln0=self._ln(f"{pre}/LayerNorm_0"), d1=self._dense(f"{pre}/Dense_1"),
                    ln1=self._ln(f"{pre}/LayerNorm_1"))

    def _repr_spec(self):
        P, put, r = self.params, self._put, "representation"
        return dict(
            conv0=(put(P[f"{r}/Conv_0/kernel"]), put(P[f"{r}/Conv_0/bias"])), ln0=self._ln(f"{r}/LayerNorm_0"),
            # the conv kernels as 4 column groups of one 16-channel tile each (k_repr_conv: one group per wave)
            conv1=(put(pack_dense(P[f"{r}/Conv_1/kernel"].reshape(96, 64), 4, 1)), put(P[f"{r}/Conv_1/bias"])),
            ln1=self._ln(f"{r}/LayerNorm_1"),
            conv2=(put(pack_dense(P[f"{r}/Conv_2/kernel"].reshape(320, 64), 4, 1)), put(P[f"{r}/Conv_2/bias"])),
            ln2=self._ln(f"{r}/LayerNorm_2"), d0=self._dense(f"{r}/Dense_0"), ln3=self._ln(f"{r}/LayerNorm_3"),
            d1=self._dense(f"{r}/Dense_1"), ln4=self._ln(f"{r}/LayerNorm_4"), d2=self._dense(f"{r}/Dense_2"),
            ln5=self._ln(f"{r}/LayerNorm_5"), d3=self._dense(f"{r}/Dense_3"), ln6=self._ln(f"{r}/LayerNorm_6"),
            rb=[self._rb(f"{r}/ResBlock_{i}") for i in range(6)], d4=self._dense(f"{r}/Dense_4"))

    def _pred_spec(self):
        P, p = self.params, "prediction"
        return dict(
            ln0=self._ln(f"{p}/LayerNorm_0"), rb=[self._rb(f"{p}/ResBlock_{i}") for i in range(2)],
            d03=self._dense_k(np.concatenate([P[f"{p}/Dense_0/kernel"], P[f"{p}/Dense_3/kernel"]], 1),
                              np.concatenate([P[f"{p}/Dense_0/bias"], P[f"{p}/Dense_3/bias"]])),
            ln1=self._ln(f"{p}/LayerNorm_1"), d1=self._dense(f"{p}/Dense_1"), ln2=self._ln(f"{p}/LayerNorm_2"),
            d2=self._dense(f"{p}/Dense_2"), ln3=self._ln(f"{p}/LayerNorm_3"), d4=self._dense(f"{p}/Dense_4"),
            d5=self._plain(f"{p}/Dense_5"))

    def _dyn_spec(self):
        """DynamicsNetwork4 (lines 391-457); the FiLM table [A + 1][512] is derived on the device (prepare)."""
        P, put, A, d = self.params, self._put, self.A, "dynamics"
        k6, k7 = P[f"{d}/Dense_6/kernel"], P[f"{d}/Dense_7/kernel"]
        return dict(
            d0=self._plain(f"{d}/Dense_0"), ln0=self._ln(f"{d}/LayerNorm_0"),
            d12=self._dense_k(np.concatenate([P[f"{d}/Dense_1/kernel"], P[f"{d}/Dense_2/kernel"]], 1),
                              np.concatenate([P[f"{d}/Dense_1/bias"], P[f"{d}/Dense_2/bias"]])),
            d3=self._dense(f"{d}/Dense_3"), ln1=self._ln(f"{d}/LayerNorm_1"), d4=self._dense(f"{d}/Dense_4"),
            ln2=self._ln(f"{d}/LayerNorm_2"), rb=[self._rb(f"{d}/ResBlock_{i}") for i in range(2)],
            d5=self._dense(f"{d}/Dense_5"),
            d67=self._dense_k(np.concatenate([k6[:LATENT], k7[:LATENT]], 1),
                              np.concatenate([P[f"{d}/Dense_6/bias"], P[f"{d}/Dense_7/bias"]])),
            d67_onehot=put(np.concatenate([k6[LATENT:LATENT + A], k7[LATENT:LATENT + A]], 1)),
            reward_head=self._plain(f"{d}/reward_head"), discount_head=self._plain(f"{d}/discount_head"),
            film=put(np.zeros((A + 1) * 2 * LATENT, np.float32)))

    def _upload(self, w, spec, device):
        host = np.concatenate(self._chunks) if self._chunks else np.zeros(4, np.float32)
        self.buffer = torch.from_numpy(host).to(device)
        self._fill(w, spec, self.buffer.data_ptr())
        self.w = w

    @staticmethod
    def _fill(struct, spec, base):
        for name, val in spec.items():
            field = getattr(struct, name)
            if isinstance(val, int):
                setattr(struct, name, base + 4 * val)
            elif isinstance(val, tuple):
                field.__setattr__(field._fields_[0][0], base + 4 * val[0])
                field.__setattr__(field._fields_[1][0], base + 4 * val[1])
            elif isinstance(val, list):
                for i, sub in enumerate(val):
                    if isinstance(sub, tuple):     # array of muz_dense / muz_ln
                        f = field[i]
                        f.__setattr__(f._fields_[0][0], base + 4 * sub[0])
                        f.__setattr__(f._fields_[1][0], base + 4 * sub[1])
                    else:
                        _Packer._fill(field[i], sub, base)
            elif isinstance(val, dict):
                _Packer._fill(field, val, base)
            else:
                raise TypeError(name)


class DeviceNet(_Packer):
    """Packed device copy of a det-MADN parameter dict + the ``muz_net_w`` table the kernels read."""

    def __init__(self, params: dict, obs_channels: int, num_actions: int = 24, device="cuda"):
        super().__init__(params, obs_channels, num_actions)
        w = MuzNetW()
        w.obs_channels, w.num_actions = self.C, self.A
        spec = {"repr": self._repr_spec(), "dyn": self._dyn_spec(), "pred": self._pred_spec()}
        self._upload(w, spec, device)
        self.prepare()

    def prepare(self):
        """Re-derive the per-action FiLM table from the packed weights (after they change in place, e.g.
        a parameter broadcast from the learner)."""
        with torch.cuda.device(self.buffer.device):
            _L.check(_L.load().muz_net_prepare(ctypes.byref(self.w), _L.stream_ptr()), "muz_net_prepare")


# ---------------------------------------------------------------------------------- inference
def root_inference_fn(net: DeviceNet, observation: torch.Tensor, scratch: torch.Tensor | None = None):
    """root_inference_fn (lines 621-630): obs [B, C, 56] -> (prior_logits [B, A], value [B], embedding [B, 256])."""
    lib = _L.load()
    obs = observation.to(dtype=torch.float32).contiguous()
    B = obs.shape[0]
    if obs.shape[1] != net.C or obs.shape[2] != 56:
        raise ValueError(f"observation shape {tuple(obs.shape)} != (B, {net.C}, 56)")
    dev = obs.device
    need = lib.muz_nets_root_scratch_bytes(B)
    if scratch is None or scratch.numel() * scratch.element_size() < need:
        scratch = torch.empty(need // 4, dtype=torch.float32, device=dev)
    logits = torch.empty((B, net.A), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    emb = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    _L.check(lib.muz_nets_root(net.w, _L.ptr(obs), B, _L.ptr(scratch), _L.nbytes(scratch), _L.ptr(logits),
                               _L.ptr(value), _L.ptr(emb), _L.stream_ptr()), "muz_nets_root")
    return logits, value, emb


def recurrent_inference_fn(net: DeviceNet, action: torch.Tensor, embedding: torch.Tensor):
    """recurrent_inference_fn (lines 632-661) -> (reward, discount, prior_logits, value, next_embedding)."""
    lib = _L.load()
    emb = embedding.to(dtype=torch.float32).contiguous()
    act = action.to(device=emb.device, dtype=torch.int32).contiguous()
    B = emb.shape[0]
    dev = emb.device
    reward = torch.empty((B,), dtype=torch.float32, device=dev)
    discount = torch.empty((B,), dtype=torch.float32, device=dev)
    logits = torch.empty((B, net.A), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    nxt = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    _L.check(lib.muz_nets_recurrent(net.w, _L.ptr(act), _L.ptr(emb), B, _L.ptr(reward), _L.ptr(discount),
                                    _L.ptr(logits), _L.ptr(value), _L.ptr(nxt), _L.stream_ptr()),
             "muz_nets_recurrent")
    return reward, discount, logits, value, nxt


# ---------------------------------------------------------------------------------- reference params
_NET_CACHE: dict = {}


def rng_key_to_seed(rng_key) -> int:
    """The reference's ``rng_key`` argument -> this engine's 64-bit counter-RNG seed.  Accepts an int or a
    jax-style uint32[2] key (key data as a list / NumPy / torch array).  jax's threefry streams are not
    reproduced: the key only selects the engine's own noise stream, deterministically."""
    if isinstance(rng_key, (int, np.integer)):
        return int(rng_key) & ((1 << 64) - 1)
    k = np.asarray(rng_key.cpu() if isinstance(rng_key, torch.Tensor) else rng_key).astype(np.uint64).ravel()
    if k.size != 2:
        raise ValueError(f"rng_key must be an int or a uint32[2] key, got shape {k.shape}")
    return int((int(k[0]) << 32) | int(k[1]))


def as_device_net(params, obs_channels: int | None = None, device="cuda") -> DeviceNet:
    """The reference's ``params`` argument -> a DeviceNet (packed once, cached per params object).

    Accepts what the reference passes around -- init_muzero_params' nested Flax tree
    (``{"representation": {"params": ...}, "dynamics": ..., "prediction": ...}``,
    muzero_deterministic_madn.py:706-748), a flat ``"net/Layer/param"`` dict, or a DeviceNet.  The channel
    count is read from the representation's Dense_1 kernel (C - 6 inputs) when not given."""
    if isinstance(params, DeviceNet):
        return params
    fp = params_fingerprint(params)
    hit = _NET_CACHE.get(id(params))
    if hit is not None and hit[0] is params and hit[2] == fp and str(hit[1].buffer.device) == str(torch.device(device)):
        return hit[1]
    from . import checkpoint as CK
    flat = params if all(isinstance(k, str) and "/" in k for k in params) else CK.muzero_tree_to_flat_any(params)
    flat = {k: np.asarray(v.detach().cpu() if isinstance(v, torch.Tensor) else v, np.float32) for k, v in flat.items()}
    C = int(flat["representation/Dense_1/kernel"].shape[0]) + 6 if obs_channels is None else int(obs_channels)
    A = int(flat["prediction/Dense_2/kernel"].shape[1])
    net = DeviceNet(flat, C, A, device=device)
    prev = next(iter(_NET_CACHE.values()), None)
    if prev is not None and (prev[1].C, prev[1].A) == (C, A) and prev[1].buffer.shape == net.buffer.shape \
            and prev[1].buffer.device == net.buffer.device:
        # same shapes: the new weights go into the live DeviceNet, so engines cached on it (game_agent.cached_engine)
        # keep their state, workspace and buffers across a training loop's iterations
        prev[1].buffer.copy_(net.buffer)
        prev[1].prepare()
        net = prev[1]
    _NET_CACHE.clear()          # one live weight set per process is what the reference's loops use
    _NET_CACHE[id(params)] = (params, net, fp)
    return net


_VERSIONED = {}    # id(tree) -> (tree, version()): trees whose owner updates the leaves in place


def register_versioned_params(tree, version):
    """``tree``'s leaves are updated in place by an owner that counts its updates (training.OptState: the
    learner's steps): params_fingerprint of that tree is then the count, not an inference from the values."""
    _VERSIONED[id(tree)] = (tree, version)


def params_fingerprint(params) -> tuple:
    """Content fingerprint of a parameter tree, so an in-place update of the same dict / arrays between
    calls invalidates as_device_net's cache: a tree registered by its owner (register_versioned_params: the
    learner's live tree) by the owner's update count; otherwise per NumPy leaf a CRC32 of its bytes (~10 ms for
    the 11 MB det tree), the torch leaves (e.g. a learner's live parameters, which the fused AdamW kernel updates through
    raw pointers, so torch's version counters do not move) by their L2 norms, all in one multi-tensor kernel
    and one device-to-host copy."""
    hit = _VERSIONED.get(id(params))
    if hit is not None and hit[0] is params:
        return (("version", int(hit[1]())),)
    import zlib
    out, tens = [], []

    def walk(t, pre):
        if isinstance(t, dict):
            for k in sorted(t):
                walk(t[k], f"{pre}/{k}")
        elif isinstance(t, torch.Tensor):
            out.append((pre, tuple(t.shape), t.data_ptr()))
            tens.append(t.detach())
        else:
            a = np.ascontiguousarray(np.asarray(t))
            out.append((pre, zlib.crc32(a.view(np.uint8).reshape(-1)), a.shape))
    walk(params, "")
    if tens:
        norms = torch.stack([n.double() for n in torch._foreach_norm(tens)]).cpu().numpy()
        out.append(("norms", norms.tobytes()))
    return tuple(out)
