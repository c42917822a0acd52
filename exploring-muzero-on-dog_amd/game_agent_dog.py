"""MuZero_DOG/game_agent.py on the GPU: DOG self-play with the MuZero policy of the DOG slice.

The reference's DOG self-play (``play_batch_of_games_jitted`` / ``play_n_games_v3``, MuZero_DOG/game_agent.py:52-65)
is ``pass``; its rules (``RULES``, game_agent.py:12-23) and the det-MADN loop it copies (MuZero_det_MADN/game_agent.py:
50-192: valid actions -> encode -> run_muzero_mcts -> env_step, or no_step without a legal move) define what it would
do.  ``DogSelfPlay`` runs that turn for a batch of games resident on the device -- muz_dog_legal, muz_dog_encode,
the root inference, the Gumbel search at A = 806 (k_dog_search) and muz_dog_step_restart, five launches per turn --
and restarts finished games in place so the batch stays full (config (d)'s actor).  Gumbel noise: the device stream
of (seed, game, turn); deals: the engine's counter keys.  Parity: followed turn by turn by oracle/dog.py +
oracle/mctx_gumbel.py driven by the same network kernels (tests/test_gpu_dog_muzero.py); unpinned beyond the env.
"""
from __future__ import annotations

import torch

from . import dog as DOG
from . import lib as _L
from . import muzero_dog as MD

RULES = dict(enable_teams=True, enable_initial_free_pin=False, enable_circular_board=True, enable_friendly_fire=True,
             enable_start_blocking=True, enable_jump_in_goal_area=False, must_traverse_start=True,
             disable_swapping=False, disable_hot_seven=False, disable_joker=False)


class DogSelfPlay:
    """A batch of 4-player DOG games played by the MuZero policy, state resident on the device."""

    def __init__(self, net: MD.DeviceDogNet, num_envs: int, num_simulations: int = 100, max_depth: int = 50,
                 temperature: float = 1.0, seed: int = 0, rules: dict | None = None, device="cuda"):
        self.net, self.B = net, int(num_envs)
        self.S, self.D, self.temp, self.seed = int(num_simulations), int(max_depth), float(temperature), int(seed)
        self.rules = dict(rules or RULES)
        self.env = DOG.env_reset(self.B, num_players=4, seed=self.seed, device=device, **self.rules)
        i32 = dict(dtype=torch.int32, device=device)
        self.words = torch.empty((self.B, DOG.MASK_WORDS), **i32)
        self.obs = torch.empty((self.B, MD.NUM_CHANNELS, 56), dtype=torch.float32, device=device)
        self.reward = torch.empty((self.B,), dtype=torch.int8, device=device)
        self.done = torch.empty((self.B,), dtype=torch.uint8, device=device)
        self.episodes = torch.zeros((self.B,), **i32)
        self.ws = MD.SearchWorkspace(self.B, self.S, device)
        self.turn_index = 0
        self.rec = None             # the trajectory buffers of the recording stream in progress (start_records)
        self._rec_cache = None

    def turn(self):
        """One turn of every game: (action [B] (-1 = no_step), action_weights [B, 806], root_value [B]).  While
        recording (``start_records``), the turn's records are written and the step is muz_dog_sp_record_step."""
        env, lib = self.env, _L.load()
        DOG.legal_mask(env, out=self.words)
        if self.rec is not None:
            self.words.masked_fill_(self.lane_game[:, None] < 0, 0)    # idle lanes: nothing legal, nothing searched
        MD.encode_board(env, out=self.obs)
        lg, v, e = MD.root_inference_fn(self.net, self.obs, self.ws.scratch)
        pol, rv = MD.gumbel_muzero_policy(self.net, lg, v, e, self.words, self.S, self.D, self.temp, seed=self.seed,
                                          turn=self.turn_index, workspace=self.ws)
        if self.rec is None:
            _L.check(lib.muz_dog_step_restart(env.rules, env.soa(), _L.ptr(pol.action), DOG.ctypes_u64(env.seed),
                                              _L.ptr(self.reward), _L.ptr(self.done), _L.ptr(self.episodes), self.B,
                                              _L.stream_ptr()), "muz_dog_step_restart")
        else:
            _L.check(lib.muz_dog_sp_record_step(env.rules, env.soa(), _L.ptr(self.obs), _L.ptr(pol.action),
                                                _L.ptr(pol.action_weights), _L.ptr(rv), DOG.ctypes_u64(env.seed),
                                                self._traj, _L.ptr(self.lane_game), _L.ptr(self.ended),
                                                _L.ptr(self.episodes), self.B, _L.stream_ptr()), "muz_dog_sp_record_step")
            _L.check(lib.muz_dog_sp_assign(_L.ptr(self.lane_game), _L.ptr(self.ended), _L.ptr(self.rec["idx"]),
                                           _L.ptr(self.counters), self.B, _L.stream_ptr()), "muz_dog_sp_assign")
        self.turn_index += 1
        return pol.action, pol.action_weights, rv

    # ---- play_n_games_v3 records (MuZero_DOG/game_agent.py:52-65 is `pass`; the det loop's bookkeeping,
    # MuZero_det_MADN/game_agent.py:64-192) ---------------------------------------------------------------------------
    def start_records(self, num_games: int, max_steps: int = 550, seed: int | None = None):
        """Reset every lane to a fresh game and record the next ``num_games`` games into [num_games, max_steps]
        buffers (the reference's buffer dict: obs int8 [34, 56], act, rew, val, pol [806], mask, player, team, discount,
        idx); lane l plays game l first, and a lane whose game ends (done, or max_steps records) takes the next game
        number in lane order until all are handed out.  ``seed`` (default: the engine's) keys the new deals and the
        Gumbel noise, as play_n_games_v3's rng_key does (MuZero_DOG/train.py:255: PRNGKey(seed + it ** 3))."""
        n, T, dev = int(num_games), int(max_steps), self.words.device
        if seed is not None:
            self.seed = int(seed)
        if self._rec_cache is None or self._rec_cache["act"].shape != (n, T):
            z = dict(device=dev)
            self._rec_cache = {
                "obs": torch.empty((n, T, MD.NUM_CHANNELS, 56), dtype=torch.int8, **z),
                "act": torch.empty((n, T), dtype=torch.int32, **z),
                "rew": torch.empty((n, T), dtype=torch.int32, **z),
                "val": torch.empty((n, T), dtype=torch.float32, **z),
                "pol": torch.empty((n, T, MD.NUM_ACTIONS), dtype=torch.float32, **z),
                "mask": torch.empty((n, T), dtype=torch.float32, **z),
                "player": torch.empty((n, T), dtype=torch.int32, **z),
                "team": torch.empty((n, T), dtype=torch.int32, **z),
                "discount": torch.empty((n, T), dtype=torch.int32, **z),
                "idx": torch.empty((n,), dtype=torch.int32, **z),
            }
            t = _L.MuzTraj()
            for k, v in self._rec_cache.items():
                setattr(t, k, v.data_ptr())
            t.max_steps = T
            self._traj = t
        self.rec = self._rec_cache
        self.rec["idx"].zero_()
        i32 = dict(dtype=torch.int32, device=dev)
        lanes = torch.arange(self.B, **i32)
        self.lane_game = torch.where(lanes < n, lanes, torch.full_like(lanes, -1))
        self.ended = torch.zeros((self.B,), **i32)
        self.counters = torch.tensor([min(n, self.B), n, min(n, self.B)], **i32)
        self.env = DOG.env_reset(self.B, num_players=4, seed=self.seed, device=dev, **self.rules)
        return self.rec

    def stop_records(self):
        self.rec = None

    def active_lanes(self) -> int:
        """Lanes still holding a game of the recording stream (a device sync)."""
        return int(self.counters[2].item())

    def play_stream(self, num_games: int, max_steps: int = 550, temperature: float | None = None,
                    seed: int | None = None, check_every: int = 8) -> dict:
        """``num_games`` complete games (each cut at ``max_steps`` records) through the B lanes; returns the buffer
        dict (device tensors, reused by the next call of the same shape)."""
        if temperature is not None:
            self.temp = float(temperature)
        self.start_records(num_games, max_steps, seed)
        while True:
            for _ in range(check_every):
                self.turn()
            if self.active_lanes() == 0:
                break
        rec = self.rec
        self.stop_records()
        return rec

    def play(self, nturns: int):
        for _ in range(int(nturns)):
            self.turn()
        return self.B * int(nturns)


REFERENCE_DTYPES = {"obs": torch.float32, "act": torch.int32, "rew": torch.int32, "val": torch.float32,
                    "pol": torch.float32, "mask": torch.float32, "player": torch.int32, "team": torch.int32,
                    "discount": torch.int32, "idx": torch.int32}
_ENGINE = {}


def play_n_games_v3(params, rng_key, input_shape, num_envs, num_simulation, max_depth, max_steps, temp,
                    obs_dtype=torch.float32) -> dict:
    """play_n_games_v3 (MuZero_DOG/game_agent.py:59-65; its play_batch_of_games_jitted, 52-57, is `pass`), reference
    signature: ``num_envs`` 4-player DOG games from fresh deals played to the end or ``max_steps`` turns with the
    MuZero policy, returned as the det loop's buffer dict (obs fp32 [num_envs, max_steps, 34, 56] -- ``obs_dtype=
    torch.int8`` keeps the engine's exact int8 copy --, act / rew / player / team / discount int32, val / mask fp32,
    pol fp32 [.., 806], idx).  ``params``: the slice's flat parameter dict or a DeviceDogNet; ``rng_key``: int or
    uint32[2] key (the engine's counter streams, not threefry)."""
    from . import nets as N
    if tuple(int(x) for x in input_shape) != (MD.NUM_CHANNELS, 56):
        raise ValueError(f"input_shape {tuple(input_shape)} != ({MD.NUM_CHANNELS}, 56)")
    net = MD.as_device_net(params)
    key = (id(net), int(num_envs), int(num_simulation), int(max_depth))
    sp = _ENGINE.get(key)
    if sp is None or sp.net is not net:
        _ENGINE.clear()
        sp = _ENGINE[key] = DogSelfPlay(net, num_envs, num_simulation, max_depth, temp)
    buf = sp.play_stream(num_envs, max_steps, temperature=temp, seed=N.rng_key_to_seed(rng_key))
    from .game_agent import reference_buffers
    return reference_buffers(buf, dict(REFERENCE_DTYPES, obs=obs_dtype))   # copies: the engine reuses its buffers

