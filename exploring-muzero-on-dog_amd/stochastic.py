"""Stochastic MuZero for classic MADN on the GPU (host mirror of MuZero_Classic_MADN/muzero_classic_madn.py).

* ``DeviceClassicNet`` packs a flat parameter dict (Flax paths, see oracle/classic_nets.py) into the
  ``muz_classic_net_w`` table and fills the FiLM tables (``muz_classic_net_prepare``);
* ``root_inference_fn`` (453-462), ``decision_recurrent_fn`` (414-432), ``chance_recurrent_fn`` (434-451);
* ``run_stochastic_muzero_mcts`` (464-517, reference signature) / ``stochastic_muzero_mcts`` (device-native):
  ``mctx.stochastic_muzero_policy`` as one HIP launch.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import lib as _L
from .nets import LATENT, _Packer

A_CLASSIC = 4
CHANCE = 6


class DeviceClassicNet(_Packer):
    def __init__(self, params: dict, obs_channels: int, device="cuda"):
        super().__init__(params, obs_channels, A_CLASSIC)
        P, put, A, d = self.params, self._put, self.A, "dynamics"
        w = _L.MuzClassicNetW()
        w.obs_channels, w.num_actions = self.C, self.A
        rd = P[f"{d}/reward_dense/kernel"]

        def cat(n1, n2):
            return self._dense_k(np.concatenate([P[f"{d}/{n1}/kernel"], P[f"{d}/{n2}/kernel"]], 1),
                                 np.concatenate([P[f"{d}/{n1}/bias"], P[f"{d}/{n2}/bias"]]))

        spec = {"repr": self._repr_spec(), "pred": self._pred_spec()}
        spec["sdyn"] = dict(
            act_embed=self._plain(f"{d}/act_embed"), act_input_ln=self._ln(f"{d}/act_input_ln"),
            act_film=cat("act_film_scale", "act_film_shift"),
            act_dense1=self._dense(f"{d}/act_dense1"), act_ln1=self._ln(f"{d}/act_ln1"),
            act_dense2=self._dense(f"{d}/act_dense2"), act_ln2=self._ln(f"{d}/act_ln2"),
            act_rb=[self._rb(f"{d}/ResBlock_{i}") for i in range(2)], act_proj=self._dense(f"{d}/act_proj"),
            rc=self._dense_k(np.concatenate([rd[:LATENT], P[f"{d}/chance_head/kernel"]], 1),
                             np.concatenate([P[f"{d}/reward_dense/bias"], P[f"{d}/chance_head/bias"]])),
            reward_onehot=put(rd[LATENT:LATENT + A]), reward_head=self._plain(f"{d}/reward_head"),
            discount_dense=self._dense(f"{d}/discount_dense"), discount_ln=self._ln(f"{d}/discount_ln"),
            discount_head=self._plain(f"{d}/discount_head"),
            chance_embed=self._plain(f"{d}/chance_embed"), chance_input_ln=self._ln(f"{d}/chance_input_ln"),
            chance_film=cat("chance_film_scale", "chance_film_shift"),
            chance_dense1=self._dense(f"{d}/chance_dense1"), chance_ln1=self._ln(f"{d}/chance_ln1"),
            chance_dense2=self._dense(f"{d}/chance_dense2"), chance_ln2=self._ln(f"{d}/chance_ln2"),
            chance_rb=[self._rb(f"{d}/ResBlock_{i}") for i in range(2, 4)],
            chance_proj=self._dense(f"{d}/chance_proj"),
            act_film_tab=put(np.zeros((A + 1) * 2 * LATENT, np.float32)),
            chance_film_tab=put(np.zeros((CHANCE + 1) * 2 * LATENT, np.float32)))
        self._upload(w, spec, device)
        self.prepare()

    def prepare(self):
        """Re-derive the action / chance FiLM tables from the packed weights."""
        with torch.cuda.device(self.buffer.device):
            _L.check(_L.load().muz_classic_net_prepare(ctypes.byref(self.w), _L.stream_ptr()),
                     "muz_classic_net_prepare")


def classic_param_shapes(obs_channels: int, num_actions: int = A_CLASSIC, chance_outcomes: int = 6) -> dict:
    """Flax tree of (RepresentationNetwork2, StochasticDynamicsNetwork4, PredictionNetwork4) for classic
    MADN (MuZero_Classic_MADN/muzero_classic_madn.py:69-135, 314-408, 192-226), flattened."""
    from .nets import _resblock_shapes, param_shapes
    A, C, L = num_actions, chance_outcomes, LATENT
    det = param_shapes(obs_channels, A)
    dense_l = {"act_embed": (A, 64), "act_film_scale": (64, L), "act_film_shift": (64, L), "act_dense1": (L, L),
               "act_dense2": (L, L), "act_proj": (L, L), "reward_dense": (L + A, 64), "reward_head": (64, 3),
               "discount_dense": (L, 32), "discount_head": (32, 3), "chance_head": (L, C), "chance_embed": (C, 64),
               "chance_film_scale": (64, L), "chance_film_shift": (64, L), "chance_dense1": (L, L),
               "chance_dense2": (L, L), "chance_proj": (L, L)}
    s = {}
    for name, (i, o) in dense_l.items():
        s[f"{name}/kernel"], s[f"{name}/bias"] = (i, o), (o,)
    for name, n in {"act_input_ln": L, "act_ln1": L, "act_ln2": L, "discount_ln": 32, "chance_input_ln": L,
                    "chance_ln1": L, "chance_ln2": L}.items():
        s[f"{name}/scale"], s[f"{name}/bias"] = (n,), (n,)
    for r in range(4):
        _resblock_shapes(s, f"ResBlock_{r}")
    out = {k: v for k, v in det.items() if k.startswith("representation/")}
    out.update({f"dynamics/{k}": v for k, v in s.items()})
    out.update({k: v for k, v in det.items() if k.startswith("prediction/")})
    return out


def init_classic_params(obs_channels: int, seed: int = 0) -> dict:
    """Flax-default initialisation (lecun_normal kernels truncated at 2 std, zero biases, unit LayerNorm
    scales) from seeded NumPy draws, in classic_param_shapes order."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, shp in classic_param_shapes(obs_channels).items():
        if k.endswith("kernel"):
            std = np.sqrt(1.0 / int(np.prod(shp[:-1]))) / 0.87962566103423978
            out[k] = (np.clip(rng.standard_normal(shp), -2.0, 2.0) * std).astype(np.float32)
        else:
            out[k] = (np.ones(shp) if k.endswith("scale") else np.zeros(shp)).astype(np.float32)
    return out


def _f32(t):
    return t.to(dtype=torch.float32).contiguous()


def root_inference_fn(net: DeviceClassicNet, observation: torch.Tensor, scratch: torch.Tensor | None = None):
    """root_inference_fn (453-462): obs [B, 2P+3, 56] -> (prior_logits [B, 4], value [B], embedding [B, 256])."""
    lib = _L.load()
    obs = _f32(observation)
    B, dev = obs.shape[0], obs.device
    if obs.shape[1] != net.C or obs.shape[2] != 56:
        raise ValueError(f"observation shape {tuple(obs.shape)} != (B, {net.C}, 56)")
    need = lib.muz_nets_root_scratch_bytes(B)
    if scratch is None or _L.nbytes(scratch) < need:
        scratch = torch.empty(need // 4, dtype=torch.float32, device=dev)
    logits = torch.empty((B, A_CLASSIC), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    emb = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    _L.check(lib.muz_classic_nets_root(net.w, _L.ptr(obs), B, _L.ptr(scratch), _L.nbytes(scratch), _L.ptr(logits),
                                       _L.ptr(value), _L.ptr(emb), _L.stream_ptr()), "muz_classic_nets_root")
    return logits, value, emb


def decision_recurrent_fn(net: DeviceClassicNet, action: torch.Tensor, embedding: torch.Tensor):
    """decision_recurrent_fn (414-432) -> (chance_logits [B,6], afterstate_value [B], afterstate [B,256],
    reward [B], discount [B]) -- the reference appends reward / discount to the afterstate."""
    emb = _f32(embedding)
    B, dev = emb.shape[0], emb.device
    act = action.to(device=dev, dtype=torch.int32).contiguous()
    after = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    reward = torch.empty((B,), dtype=torch.float32, device=dev)
    discount = torch.empty((B,), dtype=torch.float32, device=dev)
    cl = torch.empty((B, CHANCE), dtype=torch.float32, device=dev)
    av = torch.empty((B,), dtype=torch.float32, device=dev)
    _L.check(_L.load().muz_classic_nets_decision(net.w, _L.ptr(act), _L.ptr(emb), B, _L.ptr(after), _L.ptr(reward),
                                                 _L.ptr(discount), _L.ptr(cl), _L.ptr(av), _L.stream_ptr()),
             "muz_classic_nets_decision")
    return cl, av, after, reward, discount


def chance_recurrent_fn(net: DeviceClassicNet, chance: torch.Tensor, afterstate: torch.Tensor):
    """chance_recurrent_fn (434-451) -> (action_logits [B,4], value [B], next_embedding [B,256])."""
    after = _f32(afterstate)
    B, dev = after.shape[0], after.device
    ch = chance.to(device=dev, dtype=torch.int32).contiguous()
    nxt = torch.empty((B, LATENT), dtype=torch.float32, device=dev)
    logits = torch.empty((B, A_CLASSIC), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    _L.check(_L.load().muz_classic_nets_chance(net.w, _L.ptr(ch), _L.ptr(after), B, _L.ptr(nxt), _L.ptr(logits),
                                               _L.ptr(value), _L.stream_ptr()), "muz_classic_nets_chance")
    return logits, value, nxt


def make_cfg(num_simulations, max_depth, temperature=1.0, seed=0, turn=0, dirichlet_fraction=0.25,
             dirichlet_alpha=0.3, pb_c_init=1.25, pb_c_base=19652.0) -> _L.MuzStochCfg:
    c = _L.MuzStochCfg()
    c.num_simulations, c.max_depth = int(num_simulations), int(max_depth)
    c.dirichlet_fraction, c.dirichlet_alpha = float(dirichlet_fraction), float(dirichlet_alpha)
    c.pb_c_init, c.pb_c_base, c.temperature = float(pb_c_init), float(pb_c_base), float(temperature)
    c.seed, c.turn = int(seed) & ((1 << 64) - 1), int(turn)
    return c


def stochastic_muzero_policy(net: DeviceClassicNet, root_logits, root_value, root_emb, legal_bits, num_simulations,
                             max_depth, temperature=1.0, seed=0, turn=0, dirichlet=None, gumbel=None, game_id=None,
                             workspace: torch.Tensor | None = None):
    """mctx.stochastic_muzero_policy as called by run_stochastic_muzero_mcts (464-517).
    Returns (action [B], action_weights [B, 4], root_value [B] clipped to [-1, 1])."""
    lib = _L.load()
    B, dev = root_logits.shape[0], root_logits.device
    need = lib.muz_stochastic_workspace_bytes(B, num_simulations)
    if workspace is None or _L.nbytes(workspace) < need:
        workspace = torch.empty((need,), dtype=torch.uint8, device=dev)
    action = torch.empty((B,), dtype=torch.int32, device=dev)
    weights = torch.empty((B, A_CLASSIC), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    cfg = make_cfg(num_simulations, max_depth, temperature, seed, turn)
    lg, rv, re = _f32(root_logits), _f32(root_value), _f32(root_emb)
    lb = legal_bits.to(device=dev, dtype=torch.int32).contiguous()
    dn = None if dirichlet is None else _f32(dirichlet.to(dev))
    gm = None if gumbel is None else _f32(gumbel.to(dev))
    gi = None if game_id is None else game_id.to(device=dev, dtype=torch.int32).contiguous()
    _L.check(lib.muz_stochastic_search(net.w, ctypes.byref(cfg), _L.ptr(lg), _L.ptr(rv), _L.ptr(re), _L.ptr(lb),
                                       _L.ptr(dn), _L.ptr(gm), _L.ptr(gi), B, _L.ptr(workspace), _L.nbytes(workspace),
                                       _L.ptr(action), _L.ptr(weights), _L.ptr(value), _L.stream_ptr()),
             "muz_stochastic_search")
    return action, weights, value


def stochastic_muzero_mcts(net: DeviceClassicNet, observations, legal_bits, num_simulations, max_depth,
                           temperature, seed=0, turn=0, **kw):
    """Device-native form of run_stochastic_muzero_mcts: DeviceClassicNet, device observations, 4-bit legal
    mask per game; root inference + search.  Returns (action, action_weights, clipped root value)."""
    logits, value, emb = root_inference_fn(net, observations)
    return stochastic_muzero_policy(net, logits, value, emb, legal_bits, num_simulations, max_depth, temperature,
                                    seed=seed, turn=turn, **kw)


_NET_CACHE: dict = {}


def as_device_classic_net(params, obs_channels: int | None = None, device="cuda") -> DeviceClassicNet:
    """The reference's classic ``params`` (init_muzero_params' nested Flax tree, muzero_classic_madn.py, or a
    flat dict, or a DeviceClassicNet) -> DeviceClassicNet, packed once per params object."""
    if isinstance(params, DeviceClassicNet):
        return params
    from .nets import params_fingerprint
    fp = params_fingerprint(params)          # an in-place update of the same tree re-packs (nets.as_device_net)
    hit = _NET_CACHE.get(id(params))
    if hit is not None and hit[0] is params and hit[2] == fp and str(hit[1].buffer.device) == str(torch.device(device)):
        return hit[1]
    from . import checkpoint as CK
    flat = params if all(isinstance(k, str) and "/" in k for k in params) else CK.muzero_tree_to_flat_any(params)
    flat = {k: np.asarray(v.detach().cpu() if isinstance(v, torch.Tensor) else v, np.float32) for k, v in flat.items()}
    C = int(flat["representation/Dense_1/kernel"].shape[0]) + 6 if obs_channels is None else int(obs_channels)
    net = DeviceClassicNet(flat, C, device=device)
    prev = next(iter(_NET_CACHE.values()), None)
    if prev is not None and prev[1].C == C and prev[1].buffer.shape == net.buffer.shape \
            and prev[1].buffer.device == net.buffer.device:
        # same shapes: new weights into the live net, so the cached self-play engine keeps its buffers
        prev[1].buffer.copy_(net.buffer)
        prev[1].prepare()
        net = prev[1]
    _NET_CACHE.clear()
    _NET_CACHE[id(params)] = (params, net, fp)
    return net


def run_stochastic_muzero_mcts(params, rng_key, observations, invalid_actions, num_simulations, max_depth,
                               temperature):
    """run_stochastic_muzero_mcts (MuZero_Classic_MADN/muzero_classic_madn.py:464-517), reference signature:
    Flax params dict, int / uint32[2] key (the engine's Dirichlet / Gumbel streams, nets.rng_key_to_seed),
    observations [B, 2P + 3, 56], invalid_actions bool [B, 4].  Returns (PolicyOutput(action,
    action_weights), root_value = node_values[0] clipped to [-1, 1]) as cuda tensors."""
    from .mcts import PolicyOutput, invalid_to_bits
    from .nets import rng_key_to_seed
    dev = torch.device("cuda")
    net = as_device_classic_net(params, device=dev)
    obs = observations if isinstance(observations, torch.Tensor) else torch.from_numpy(np.asarray(observations))
    bits = invalid_to_bits(invalid_actions).to(dev)
    a, w, v = stochastic_muzero_mcts(net, obs.to(device=dev, dtype=torch.float32), bits, num_simulations, max_depth,
                                     temperature, seed=rng_key_to_seed(rng_key))
    return PolicyOutput(a, w), v
