"""MuZero_DOG/muzero_dog.py on the GPU: the DOG MuZero slice.

The reference defines the DOG ``RepresentationNetwork`` (muzero_dog.py:25-83: RepresentationNetwork2's trunk with a
LayerNorm after its last Dense) and leaves ``DynamicsNetwork`` / ``PredictionNetwork`` / ``root_inference_fn`` /
``recurrent_inference_fn`` (85-99), DOG's ``encode_board`` (DOG/dog.py:1264-1272) and the self-play loop
(MuZero_DOG/game_agent.py:52-57) as ``pass``.  SURVEY §8(d): "MCTS with the det-MADN-shaped nets at A=806".  Here:

* ``encode_board``: a 34-channel observation (csrc/dog_muzero.hip k_dog_encode; oracle/dog_muzero.py states it);
* ``init_muzero_params``: RepresentationNetwork + DynamicsNetwork4 / PredictionNetwork4 of the det file at A = 806
  (Flax paths as the det tree, plus ``representation/LayerNorm_7``);
* ``DeviceDogNet`` packs them for the fused fp32 MFMA kernels (``muz_dog_net_w``);
* ``root_inference_fn`` / ``recurrent_inference_fn`` with the mctx contract;
* ``run_muzero_mcts`` (muzero_dog.py:101-137): gumbel_muzero_policy at A = 806 (csrc/dog_search.hip).

Parity: the env under it is pinned (oracle/dog.py); everything above it is builder-defined (parity unpinned),
restated by oracle/dog_muzero.py and checked against it (tests/test_gpu_dog_muzero.py).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import dog as DOG
from . import lib as _L
from . import nets as N

NUM_ACTIONS = 806
NUM_CHANNELS = 34
LATENT = N.LATENT
CHUNKS = ((0, 256), (256, 512), (512, 768), (768, 806))   # PredictionNetwork4 Dense_2 column chunks (muz.h)


def param_shapes() -> dict:
    """Flax parameter tree of the slice, flattened: det shapes at C = 34, A = 806, plus the repr's LayerNorm_7."""
    s = N.param_shapes(NUM_CHANNELS, NUM_ACTIONS)
    s["representation/LayerNorm_7/scale"] = s["representation/LayerNorm_7/bias"] = (LATENT,)
    return s


def init_muzero_params(seed: int = 0) -> dict:
    """init_muzero_params (muzero_dog.py:139-181) with Flax defaults (lecun_normal kernels, zero biases, unit LN
    scales), seeded NumPy draws (jax threefry is not reproduced)."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, shp in param_shapes().items():
        if k.endswith("kernel"):
            fan_in = int(np.prod(shp[:-1]))
            std = np.sqrt(1.0 / fan_in) / 0.87962566103423978
            out[k] = (np.clip(rng.standard_normal(shp), -2.0, 2.0) * std).astype(np.float32)
        elif k.endswith("scale"):
            out[k] = np.ones(shp, np.float32)
        else:
            out[k] = np.zeros(shp, np.float32)
    return out


class DeviceDogNet(N._Packer):
    """Packed device copy of the slice's parameters + the ``muz_dog_net_w`` table the kernels read."""

    def __init__(self, params: dict, device="cuda"):
        super().__init__(params, NUM_CHANNELS, NUM_ACTIONS)
        P, p = self.params, "prediction"
        w = _L.MuzDogNetW()
        w.obs_channels, w.num_actions = self.C, self.A
        pred = self._pred_spec_no_logits()
        k2, b2 = P[f"{p}/Dense_2/kernel"], P[f"{p}/Dense_2/bias"]
        logits = []
        for lo, hi in CHUNKS:
            kc, bc = k2[:, lo:hi], b2[lo:hi]
            # chunks 0-2 packed for 256 columns (dense16<NT256>), the last for its 38 (dense16<nt_for(38)>)
            logits.append((self._put(N.pack_dense(kc, self.waves, N.nt_for(hi - lo, self.waves))), self._put(bc)))
        pred["d2"] = logits[0]
        spec = {"repr": self._repr_spec(), "repr_ln7": self._ln("representation/LayerNorm_7"),
                "dyn": self._dyn_spec(), "pred": pred, "logits": logits}
        self._upload(w, spec, device)
        self.prepare()

    def _pred_spec_no_logits(self):
        P, p = self.params, "prediction"
        return dict(
            ln0=self._ln(f"{p}/LayerNorm_0"), rb=[self._rb(f"{p}/ResBlock_{i}") for i in range(2)],
            d03=self._dense_k(np.concatenate([P[f"{p}/Dense_0/kernel"], P[f"{p}/Dense_3/kernel"]], 1),
                              np.concatenate([P[f"{p}/Dense_0/bias"], P[f"{p}/Dense_3/bias"]])),
            ln1=self._ln(f"{p}/LayerNorm_1"), d1=self._dense(f"{p}/Dense_1"), ln2=self._ln(f"{p}/LayerNorm_2"),
            ln3=self._ln(f"{p}/LayerNorm_3"), d4=self._dense(f"{p}/Dense_4"), d5=self._plain(f"{p}/Dense_5"))

    def prepare(self):
        with torch.cuda.device(self.buffer.device):
            _L.check(_L.load().muz_dog_net_prepare(ctypes.byref(self.w), _L.stream_ptr()), "muz_dog_net_prepare")


_NET_CACHE = []


def as_device_net(params, device="cuda") -> DeviceDogNet:
    """A flat ``net/Layer/param`` dict or a Flax tree (or a DeviceDogNet) -> DeviceDogNet.  New weights go into the
    DeviceDogNet of the previous call in place (same arena layout), so an engine cached on it (game_agent_dog.
    play_n_games_v3) keeps its buffers -- the reference's train loop passes a fresh params tree every iteration."""
    if isinstance(params, DeviceDogNet):
        return params
    flat = params if all(isinstance(k, str) and "/" in k for k in params) else _flat(params)
    flat = {k: np.asarray(v.detach().cpu() if isinstance(v, torch.Tensor) else v, np.float32) for k, v in flat.items()}
    net = DeviceDogNet(flat, device=device)
    prev = _NET_CACHE[0] if _NET_CACHE else None
    if prev is not None and prev.buffer.shape == net.buffer.shape and prev.buffer.device == net.buffer.device:
        prev.buffer.copy_(net.buffer)
        prev.prepare()
        return prev
    _NET_CACHE[:] = [net]
    return net


def _flat(tree) -> dict:
    from . import checkpoint as CK
    return CK.muzero_tree_to_flat_any(tree)


def encode_board(env: DOG.DOGState, out: torch.Tensor | None = None) -> torch.Tensor:
    """Batched encode_board (DOG/dog.py:1264-1272 is `pass`; oracle/dog_muzero.py states this one): fp32 [B, 34, 56]."""
    out = torch.empty((env.batch, NUM_CHANNELS, 56), dtype=torch.float32, device=env.board.device) \
        if out is None else out
    _L.check(_L.load().muz_dog_encode(env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr()), "muz_dog_encode")
    return out


def root_inference_fn(net: DeviceDogNet, observation: torch.Tensor, scratch: torch.Tensor | None = None):
    """obs [B, 34, 56] -> (prior_logits [B, 806], value [B], embedding [B, 256])."""
    lib = _L.load()
    obs = observation.to(dtype=torch.float32).contiguous()
    B = obs.shape[0]
    if tuple(obs.shape[1:]) != (NUM_CHANNELS, 56):
        raise ValueError(f"observation shape {tuple(obs.shape)} != (B, {NUM_CHANNELS}, 56)")
    dev = obs.device
    need = lib.muz_nets_root_scratch_bytes(B)
    if scratch is None or _L.nbytes(scratch) < need:
        scratch = torch.empty(need // 4, dtype=torch.float32, device=dev)
    logits = torch.empty((B, NUM_ACTIONS), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    emb = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    _L.check(lib.muz_dog_nets_root(net.w, _L.ptr(obs), B, _L.ptr(scratch), _L.nbytes(scratch), _L.ptr(logits),
                                   _L.ptr(value), _L.ptr(emb), _L.stream_ptr()), "muz_dog_nets_root")
    return logits, value, emb


def recurrent_inference_fn(net: DeviceDogNet, action: torch.Tensor, embedding: torch.Tensor):
    """(action [B], embedding [B, 256]) -> (reward, discount, prior_logits [B, 806], value, next_embedding)."""
    lib = _L.load()
    emb = embedding.to(dtype=torch.float32).contiguous()
    act = action.to(device=emb.device, dtype=torch.int32).contiguous()
    B, dev = emb.shape[0], emb.device
    reward = torch.empty((B,), dtype=torch.float32, device=dev)
    discount = torch.empty((B,), dtype=torch.float32, device=dev)
    logits = torch.empty((B, NUM_ACTIONS), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    nxt = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    _L.check(lib.muz_dog_nets_recurrent(net.w, _L.ptr(act), _L.ptr(emb), B, _L.ptr(reward), _L.ptr(discount),
                                        _L.ptr(logits), _L.ptr(value), _L.ptr(nxt), _L.stream_ptr()),
             "muz_dog_nets_recurrent")
    return reward, discount, logits, value, nxt


# ---------------------------------------------------------------------------------- search (muzero_dog.py:101-137)
class SearchWorkspace:
    """Device workspace for B DOG searches: children arrays [B][S+1][832] x 6 + node embeddings (+ root scratch)."""

    def __init__(self, batch: int, num_simulations: int, device="cuda"):
        from . import mcts as M
        lib = _L.load()
        self.batch, self.S = batch, num_simulations
        nbytes = lib.muz_dog_search_workspace_bytes(batch, M.make_cfg(num_simulations, 1))
        self.tree = torch.empty((nbytes,), dtype=torch.uint8, device=device)
        self.scratch = torch.empty(lib.muz_nets_root_scratch_bytes(batch) // 4, dtype=torch.float32, device=device)

    def fits(self, batch, S):
        return batch <= self.batch and S <= self.S


def gumbel_muzero_policy(net: DeviceDogNet, root_logits, root_value, root_embedding, legal_words, num_simulations,
                         max_depth, temperature=1.0, gumbel=None, seed=0, turn=0,
                         workspace: SearchWorkspace | None = None):
    """mctx.gumbel_muzero_policy at A = 806 as muzero_dog.py:122-133 calls it (qtransform_completed_by_mix_value
    with value_scale=0.5, max_num_considered_actions=16, gumbel_scale=temperature).  ``legal_words``: int32 [B, 26]
    (dog.legal_mask); ``gumbel``: explicit scaled noise [B, 806] or None for the device stream of (seed, game, turn).
    Returns (PolicyOutput, root_value = search_tree.summary().value)."""
    from . import mcts as M
    lib = _L.load()
    B, dev = root_logits.shape[0], root_logits.device
    if workspace is None or not workspace.fits(B, num_simulations):
        workspace = SearchWorkspace(B, num_simulations, dev)
    cfg = M.make_cfg(num_simulations, max_depth, temperature, seed=seed, turn=turn)
    action = torch.empty((B,), dtype=torch.int32, device=dev)
    weights = torch.empty((B, NUM_ACTIONS), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    g = None if gumbel is None else gumbel.to(device=dev, dtype=torch.float32).contiguous()
    lw = legal_words.to(device=dev, dtype=torch.int32).contiguous()
    if tuple(lw.shape) != (B, DOG.MASK_WORDS):
        raise ValueError(f"legal_words shape {tuple(lw.shape)} != ({B}, {DOG.MASK_WORDS})")
    _L.check(lib.muz_dog_gumbel_search(net.w, cfg, _L.ptr(root_logits.contiguous()), _L.ptr(root_value.contiguous()),
                                       _L.ptr(root_embedding.contiguous()), _L.ptr(lw), _L.ptr(g), B,
                                       _L.ptr(workspace.tree), _L.nbytes(workspace.tree), _L.ptr(action),
                                       _L.ptr(weights), _L.ptr(value), _L.stream_ptr()), "muz_dog_gumbel_search")
    from .mcts import PolicyOutput
    return PolicyOutput(action, weights), value


def invalid_to_words(invalid_actions) -> torch.Tensor:
    """bool [B, 806] invalid mask (the reference's ``~valid_actions``) -> int32 legal words [B, 26]."""
    inv = invalid_actions if isinstance(invalid_actions, torch.Tensor) else torch.from_numpy(
        np.asarray(invalid_actions, dtype=bool))
    inv = inv.reshape(inv.shape[0], -1).to(torch.bool)
    B, A = inv.shape
    leg = torch.zeros((B, DOG.MASK_WORDS * 32), dtype=torch.int64, device=inv.device)
    leg[:, :A] = (~inv).to(torch.int64)
    sh = torch.arange(32, device=inv.device, dtype=torch.int64)
    w = (leg.reshape(B, DOG.MASK_WORDS, 32) << sh).sum(-1)
    return (w - ((w >> 31) << 32)).to(torch.int32)     # as signed int32 words


def run_muzero_mcts(params, rng_key, observations, invalid_actions, num_simulations, max_depth, temperature):
    """run_muzero_mcts (MuZero_DOG/muzero_dog.py:101-137), reference signature: root inference + Gumbel search at
    A = 806.  ``params``: the slice's flat parameter dict or a DeviceDogNet; ``rng_key``: int or uint32[2] key;
    ``observations`` [B, 34, 56]; ``invalid_actions`` bool [B, 806].  Returns (PolicyOutput, root_value)."""
    dev = torch.device("cuda")
    net = as_device_net(params, device=dev)
    obs = observations if isinstance(observations, torch.Tensor) else torch.from_numpy(np.asarray(observations))
    logits, value, emb = root_inference_fn(net, obs.to(device=dev, dtype=torch.float32))
    return gumbel_muzero_policy(net, logits, value, emb, invalid_to_words(invalid_actions).to(dev), num_simulations,
                                max_depth, temperature, seed=N.rng_key_to_seed(rng_key))
