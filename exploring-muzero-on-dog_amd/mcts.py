"""Gumbel MuZero search on the GPU: run_muzero_mcts (MuZero_det_MADN/muzero_deterministic_madn.py:663-704).

The whole ``mctx.gumbel_muzero_policy`` call (S simulations of select / expand / backup) is one
persistent HIP kernel (csrc/search.hip); the root inference runs first (csrc/nets.hip).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lib as _L
from . import nets as _N


@dataclass
class PolicyOutput:
    """mctx.PolicyOutput without the tree object (the tree stays in the device workspace)."""
    action: torch.Tensor          # int32 [B]
    action_weights: torch.Tensor  # fp32 [B, A]


class SearchWorkspace:
    """Device workspace for B searches: tree arrays + node embeddings (+ root-inference scratch)."""

    def __init__(self, batch: int, num_simulations: int, device="cuda"):
        lib = _L.load()
        cfg = make_cfg(num_simulations, 1)
        self.batch, self.S = batch, num_simulations
        nbytes = lib.muz_search_workspace_bytes(batch, cfg)
        self.tree = torch.empty((nbytes,), dtype=torch.uint8, device=device)
        self.scratch = torch.empty(lib.muz_nets_root_scratch_bytes(batch) // 4, dtype=torch.float32, device=device)

    def fits(self, batch, S):
        return batch <= self.batch and S <= self.S


def make_cfg(num_simulations, max_depth, temperature=1.0, max_num_considered=16, value_scale=0.5,
             maxvisit_init=50.0, seed=0, turn=0):
    c = _L.MuzSearchCfg()
    c.num_simulations = int(num_simulations)
    c.max_depth = int(max_depth)
    c.max_num_considered = int(max_num_considered)
    c.value_scale = float(value_scale)
    c.maxvisit_init = float(maxvisit_init)
    c.gumbel_scale = float(temperature)
    c.seed = int(seed) & ((1 << 64) - 1)
    c.turn = int(turn)
    return c


def gumbel_muzero_policy(net: _N.DeviceNet, root_logits, root_value, root_embedding, legal_bits,
                         num_simulations, max_depth, temperature=1.0, gumbel=None, seed=0, turn=0,
                         game_id=None, workspace: SearchWorkspace | None = None):
    """mctx.gumbel_muzero_policy with qtransform_completed_by_mix_value(value_scale=0.5),
    max_num_considered_actions=16, gumbel_scale=temperature.  ``gumbel`` = explicit (already scaled)
    noise [B, A] or None to draw it on device from (seed, game_id, turn).
    Returns (PolicyOutput, root_value = search_tree.summary().value)."""
    lib = _L.load()
    B = root_logits.shape[0]
    dev = root_logits.device
    if workspace is None or not workspace.fits(B, num_simulations):
        workspace = SearchWorkspace(B, num_simulations, dev)
    cfg = make_cfg(num_simulations, max_depth, temperature, seed=seed, turn=turn)
    action = torch.empty((B,), dtype=torch.int32, device=dev)
    weights = torch.empty((B, net.A), dtype=torch.float32, device=dev)
    value = torch.empty((B,), dtype=torch.float32, device=dev)
    g = None if gumbel is None else gumbel.to(device=dev, dtype=torch.float32).contiguous()
    gid = None if game_id is None else game_id.to(device=dev, dtype=torch.int32).contiguous()
    lb = legal_bits.to(device=dev, dtype=torch.int32).contiguous()
    _L.check(lib.muz_gumbel_search(net.w, cfg, _L.ptr(root_logits.contiguous()), _L.ptr(root_value.contiguous()),
                                   _L.ptr(root_embedding.contiguous()), _L.ptr(lb), _L.ptr(g), _L.ptr(gid), B,
                                   _L.ptr(workspace.tree), _L.nbytes(workspace.tree), _L.ptr(action), _L.ptr(weights),
                                   _L.ptr(value),
                                   _L.stream_ptr()), "muz_gumbel_search")
    return PolicyOutput(action, weights), value


def muzero_mcts(net: _N.DeviceNet, observations, legal_bits, num_simulations, max_depth, temperature,
                gumbel=None, seed=0, turn=0, workspace: SearchWorkspace | None = None):
    """Device-native form of run_muzero_mcts: a DeviceNet, device observations and the 24-bit legal mask
    per game (what the self-play / evaluation loops hold); root inference + Gumbel search."""
    scratch = workspace.scratch if workspace is not None else None
    logits, value, emb = _N.root_inference_fn(net, observations, scratch)
    return gumbel_muzero_policy(net, logits, value, emb, legal_bits, num_simulations, max_depth, temperature,
                                gumbel=gumbel, seed=seed, turn=turn, workspace=workspace)


def invalid_to_bits(invalid_actions) -> torch.Tensor:
    """bool [B, A] invalid mask (True = illegal, the reference's ``~valid_action``) -> int32 legal bits [B]."""
    inv = invalid_actions if isinstance(invalid_actions, torch.Tensor) else torch.from_numpy(
        np.asarray(invalid_actions, dtype=bool))
    inv = inv.reshape(inv.shape[0], -1).to(torch.bool)
    sh = torch.arange(inv.shape[1], device=inv.device, dtype=torch.int64)
    return ((~inv).to(torch.int64) << sh).sum(1).to(torch.int32)


def run_muzero_mcts(params, rng_key, observations, invalid_actions, num_simulations, max_depth, temperature):
    """run_muzero_mcts (MuZero_det_MADN/muzero_deterministic_madn.py:663-704), reference signature.

    ``params``: init_muzero_params' nested Flax dict (or a flat dict / DeviceNet, see nets.as_device_net);
    ``rng_key``: int or uint32[2] key (selects the engine's Gumbel stream, nets.rng_key_to_seed);
    ``observations``: [B, C, 56] (NumPy or torch, any device); ``invalid_actions``: bool [B, 24].
    Returns (PolicyOutput(action, action_weights), root_value = search_tree.summary().value) as device
    tensors on cuda.

    Kernel limits (k_gumbel_search; every reference call site is inside them: S = 50 / 100, D = 25 / 50):
    num_simulations 1..100, max_depth 1..64, 24 actions (det-MADN), max_num_considered_actions 16 (mctx's
    default); outside them muz_gumbel_search returns MUZ_E_UNSUPPORTED and this raises MuzError."""
    dev = torch.device("cuda")
    net = _N.as_device_net(params, device=dev)
    obs = observations if isinstance(observations, torch.Tensor) else torch.from_numpy(np.asarray(observations))
    obs = obs.to(device=dev, dtype=torch.float32)
    bits = invalid_to_bits(invalid_actions).to(dev)
    return muzero_mcts(net, obs, bits, num_simulations, max_depth, temperature, seed=_N.rng_key_to_seed(rng_key))
