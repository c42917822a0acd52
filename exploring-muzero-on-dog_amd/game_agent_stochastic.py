"""Batched Stochastic-MuZero self-play for classic MADN on the GPU (host mirror of
MuZero_Classic_MADN/game_agent_stochastic.py).

``StochasticSelfPlayEngine.play`` = ``play_n_games_v3`` (234-257) + ``play_batch_of_games_jitted``
(52-218): the whole loop runs natively (muz_classic_selfplay).  Buffers: the det keys with
``pol`` [n, T, 4], plus ``dice`` [n, T] and ``dice_dist`` [n, T, 6]; ``obs`` is int8.
"""
from __future__ import annotations

import ctypes

import torch

from . import classic as E
from . import lib as _L
from . import stochastic as ST

# MuZero_Classic_MADN/game_agent_stochastic.py:13-24
RULES = dict(E.SELFPLAY_RULES)


class StochasticSelfPlayEngine:
    def __init__(self, net: ST.DeviceClassicNet, num_envs: int, num_players: int = 4, max_steps: int = 550,
                 num_simulations: int = 50, max_depth: int = 25, rules: dict | None = None, starting_player=0,
                 device="cuda"):
        self.net = net
        self.n, self.P, self.T = int(num_envs), int(num_players), int(max_steps)
        self.S, self.D = int(num_simulations), int(max_depth)
        self.C = E.num_channels(self.P)
        if net.C != self.C:
            raise ValueError(f"network expects {net.C} observation channels, {self.P} players give {self.C}")
        self.rules = E.make_rules(self.P, starting_player=starting_player, **dict(RULES if rules is None else rules))
        self.state = E._alloc(self.n, self.P, self.rules, device)
        n, T = self.n, self.T
        z = dict(device=device)
        self.buffers = {
            "obs": torch.empty((n, T, self.C, E.CELLS), dtype=torch.int8, **z),
            "act": torch.empty((n, T), dtype=torch.int32, **z),
            "rew": torch.empty((n, T), dtype=torch.int32, **z),
            "val": torch.empty((n, T), dtype=torch.float32, **z),
            "pol": torch.empty((n, T, ST.A_CLASSIC), dtype=torch.float32, **z),
            "mask": torch.empty((n, T), dtype=torch.float32, **z),
            "dice": torch.empty((n, T), dtype=torch.int32, **z),
            "dice_dist": torch.empty((n, T, ST.CHANCE), dtype=torch.float32, **z),
            "player": torch.empty((n, T), dtype=torch.int32, **z),
            "team": torch.empty((n, T), dtype=torch.int32, **z),
            "discount": torch.empty((n, T), dtype=torch.int32, **z),
            "idx": torch.empty((n,), dtype=torch.int32, **z),
        }
        cfg = ST.make_cfg(self.S, self.D)
        self.workspace = torch.empty((_L.load().muz_classic_selfplay_workspace_bytes(n, self.C, cfg),),
                                     dtype=torch.uint8, **z)
        self.last_turns = 0
        self.last_stats = None

    def play(self, seed: int, temperature: float = 1.0, dirichlet_fraction: float = 0.25, stream=None,
             timing: bool = True) -> dict:
        lib = _L.load()
        cfg = ST.make_cfg(self.S, self.D, temperature=temperature, seed=seed, dirichlet_fraction=dirichlet_fraction)
        t = _L.MuzTraj()
        for k in ("obs", "act", "rew", "val", "pol", "mask", "player", "team", "discount", "idx"):
            setattr(t, k, self.buffers[k].data_ptr())
        t.max_steps = self.T
        ch = _L.MuzTrajChance()
        ch.dice, ch.dice_dist = self.buffers["dice"].data_ptr(), self.buffers["dice_dist"].data_ptr()
        st = _L.MuzSpStats()
        _L.check(lib.muz_classic_selfplay(self.rules, self.net.w, ctypes.byref(cfg), self.state.soa(), t, ch, self.n,
                                          _L.ptr(self.workspace), _L.nbytes(self.workspace),
                                          ctypes.byref(st) if timing else None, _L.stream_ptr(stream)),
                 "muz_classic_selfplay")
        self.last_stats = {"turns": st.turns, "searches": st.searches, "search_ms": st.search_ms,
                           "total_ms": st.total_ms} if timing else None
        self.last_turns = st.turns if timing else -1
        return self.buffers


    def play_stream(self, num_games: int, seed: int, temperature: float = 1.0, dirichlet_fraction: float = 0.25,
                    stream=None, timing: bool = True) -> dict:
        """``num_games`` games through this engine's lanes (muz_classic_selfplay_stream); game k's record
        equals game k of ``play`` on a batch of ``num_games``."""
        lib = _L.load()
        num_games = int(num_games)
        if getattr(self, "_sbuf_n", None) != num_games:
            z = dict(device=self.buffers["act"].device)
            self._sbuf = {k: torch.empty((num_games,) + tuple(v.shape[1:]), dtype=v.dtype, **z)
                          for k, v in self.buffers.items()}
            self._sbuf_n = num_games
        cfg = ST.make_cfg(self.S, self.D, temperature=temperature, seed=seed, dirichlet_fraction=dirichlet_fraction)
        t = _L.MuzTraj()
        for k in ("obs", "act", "rew", "val", "pol", "mask", "player", "team", "discount", "idx"):
            setattr(t, k, self._sbuf[k].data_ptr())
        t.max_steps = self.T
        ch = _L.MuzTrajChance()
        ch.dice, ch.dice_dist = self._sbuf["dice"].data_ptr(), self._sbuf["dice_dist"].data_ptr()
        st = _L.MuzSpStats()
        _L.check(lib.muz_classic_selfplay_stream(self.rules, self.net.w, ctypes.byref(cfg), self.state.soa(), t, ch,
                                                 num_games, self.n, _L.ptr(self.workspace), _L.nbytes(self.workspace),
                                                 ctypes.byref(st) if timing else None, _L.stream_ptr(stream)),
                 "muz_classic_selfplay_stream")
        self.last_stats = {"turns": st.turns, "searches": st.searches, "search_ms": st.search_ms,
                           "total_ms": st.total_ms} if timing else None
        self.last_turns = st.turns if timing else -1
        return self._sbuf


_ENGINE_CACHE = {}


def play_n_games_v3(params, rng_key, input_shape, num_envs, num_simulation, max_depth, max_steps, temp,
                    obs_dtype=torch.float32) -> dict:
    """play_n_games_v3 (MuZero_Classic_MADN/game_agent_stochastic.py:220-244), reference signature: Flax
    params dict (or flat dict / DeviceClassicNet), int / uint32[2] key (the engine's counter RNG), input_shape
    (2P + 3, 56).  Returns the reference's buffers (obs fp32 unless ``obs_dtype``; dice int32, dice_dist fp32)
    as device tensors.  The reference's reset seeds only feed jax's unused random start."""
    from .game_agent import REFERENCE_DTYPES, reference_buffers
    from .nets import rng_key_to_seed
    C = int(input_shape[0])
    if (C - 3) % 2 or int(input_shape[-1]) != E.CELLS:
        raise ValueError(f"input_shape {tuple(input_shape)} is not (2P + 3, 56)")
    net = ST.as_device_classic_net(params, C)
    key = (id(net), int(num_envs), (C - 3) // 2, int(max_steps), int(num_simulation), int(max_depth))
    hit = _ENGINE_CACHE.get(key)
    if hit is None or hit.net is not net:          # one live engine, reused by a test_training-style loop
        _ENGINE_CACHE.clear()
        hit = _ENGINE_CACHE[key] = StochasticSelfPlayEngine(net, num_envs, num_players=(C - 3) // 2,
                                                            max_steps=max_steps, num_simulations=num_simulation,
                                                            max_depth=max_depth)
    eng = hit
    buf = eng.play(rng_key_to_seed(rng_key), temp)
    dt = dict(REFERENCE_DTYPES, obs=obs_dtype, dice=torch.int32, dice_dist=torch.float32)
    return reference_buffers(buf, dt)
