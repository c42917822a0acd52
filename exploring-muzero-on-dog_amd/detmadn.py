"""Batched deterministic MADN environment on the GPU (host mirror of MADN/deterministic_madn.py).

The reference API is functional over one pytree state and is batched with ``jax.vmap``
(``game_agent.py:43-48``).  Here one ``DetMADNState`` holds B games as device-resident
struct-of-arrays (field-major int8 tensors, see include/muz.h) and every call is one HIP
launch over the whole batch.  ``env_step`` / ``no_step`` update the state in place and
return it, so ``env, reward, done = env_step(env, action)`` reads like the reference.

Reference entry points mirrored (file:line in the reference):
  env_reset            MADN/deterministic_madn.py:42-120  (+ game_agent.py:24-44)
  valid_action         MADN/deterministic_madn.py:299-393
  env_step             MADN/deterministic_madn.py:170-257
  no_step              MADN/deterministic_madn.py:283-297
  encode_board         MADN/deterministic_madn.py:395-438
  map_action           MADN/deterministic_madn.py:469-479
  random_round         game_agent.py:84-119's per-turn env work with a uniform random legal policy
  set_pins_on_board    MADN/deterministic_madn.py:259-271
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lib as _L

CELLS = 56
ACTIONS = 24

# MuZero_det_MADN/game_agent.py:12-22
SELFPLAY_RULES = dict(
    enable_teams=True,
    enable_initial_free_pin=True,
    enable_circular_board=False,
    enable_friendly_fire=False,
    enable_start_blocking=False,
    enable_jump_in_goal_area=True,
    enable_start_on_1=True,
    enable_bonus_turn_on_6=True,
    must_traverse_start=False,
)

# env_reset keyword defaults (deterministic_madn.py:42-58)
DEFAULT_RULES = dict(
    enable_teams=False,
    enable_initial_free_pin=False,
    enable_circular_board=True,
    enable_start_blocking=False,
    enable_jump_in_goal_area=True,
    enable_friendly_fire=False,
    enable_start_on_1=True,
    enable_bonus_turn_on_6=True,
    must_traverse_start=False,
)


def make_rules(num_players=4, layout=(True, True, True, True), distance=10, starting_player=0, **rules):
    r = dict(DEFAULT_RULES)
    unknown = set(rules) - set(r)
    if unknown:
        raise TypeError(f"unknown rule(s): {sorted(unknown)}")
    r.update(rules)
    c = _L.MuzRules()
    c.num_players = int(num_players)
    c.distance = int(distance)
    for i in range(4):
        c.layout[i] = int(bool(layout[i]))
    c.starting_player = int(starting_player)
    for k, v in r.items():
        setattr(c, k, int(bool(v)))
    return c


def num_channels(num_players: int) -> int:
    """encode_board channel count: P + 2 + P + 6P (deterministic_madn.py:437)."""
    return 8 * num_players + 2


@dataclass
class DetMADNState:
    """SoA batch state. Field c of game b is ``field[c, b]``."""

    board: torch.Tensor           # int8 [56, B]
    pins: torch.Tensor            # int8 [P*4, B]
    current_player: torch.Tensor  # int8 [B]
    reward: torch.Tensor          # int8 [B]
    done: torch.Tensor            # uint8 [B]
    action_set: torch.Tensor      # int8 [P*6, B]
    rules: _L.MuzRules
    num_players: int

    @property
    def batch(self) -> int:
        return self.current_player.shape[0]

    def soa(self) -> _L.MuzDetSoA:
        s = _L.MuzDetSoA()
        s.board = self.board.data_ptr()
        s.pins = self.pins.data_ptr()
        s.current_player = self.current_player.data_ptr()
        s.reward = self.reward.data_ptr()
        s.done = self.done.data_ptr()
        s.action_set = self.action_set.data_ptr()
        s.stride = self.batch
        return s

    def pins_bp(self) -> torch.Tensor:
        """pins as [B, P, 4] (the reference's per-game layout)."""
        return self.pins.T.reshape(self.batch, self.num_players, 4)

    def action_set_bp(self) -> torch.Tensor:
        return self.action_set.T.reshape(self.batch, self.num_players, 6)

    def clone(self) -> "DetMADNState":
        return DetMADNState(self.board.clone(), self.pins.clone(), self.current_player.clone(), self.reward.clone(),
                            self.done.clone(), self.action_set.clone(), self.rules, self.num_players)


def _alloc(batch: int, P: int, rules, device) -> DetMADNState:
    kw = dict(device=device)
    return DetMADNState(
        board=torch.empty((CELLS, batch), dtype=torch.int8, **kw),
        pins=torch.empty((P * 4, batch), dtype=torch.int8, **kw),
        current_player=torch.empty((batch,), dtype=torch.int8, **kw),
        reward=torch.empty((batch,), dtype=torch.int8, **kw),
        done=torch.empty((batch,), dtype=torch.uint8, **kw),
        action_set=torch.empty((P * 6, batch), dtype=torch.int8, **kw),
        rules=rules,
        num_players=P,
    )


def env_reset(batch: int, num_players=4, layout=(True, True, True, True), distance=10, starting_player=0,
              device="cuda", seeds=None, **rules) -> DetMADNState:
    """Batched env_reset (deterministic_madn.py:42-120, game_agent.py:24-44).  ``seeds`` (one int per game, the
    reference's ``seed`` argument) are needed only by a random starting player (starting_player < 0 or >= P,
    line 62): each game's seat is drawn from its seed (muz_detmadn_reset_seeded)."""
    r = make_rules(num_players, layout, distance, starting_player, **rules)
    st = _alloc(batch, int(num_players), r, device)
    lib = _L.load()
    if seeds is None:
        _L.check(lib.muz_detmadn_reset(r, st.soa(), batch, _L.stream_ptr()), "muz_detmadn_reset")
    else:
        sd = torch.as_tensor(np.asarray(seeds, np.int64) & 0xFFFFFFFF).to(torch.int64)
        sd = (sd - ((sd >> 31) << 32)).to(device=device, dtype=torch.int32).contiguous()   # uint32 bits as int32
        if sd.numel() != batch:
            raise ValueError("one seed per game")
        _L.check(lib.muz_detmadn_reset_seeded(r, st.soa(), _L.ptr(sd), batch, _L.stream_ptr()),
                 "muz_detmadn_reset_seeded")
    return st


def set_pins_on_board_host(pins: np.ndarray) -> np.ndarray:
    """set_pins_on_board (deterministic_madn.py:259-271) for host-side state construction."""
    pins = np.asarray(pins)
    board = -np.ones(CELLS, dtype=np.int8)
    for p in range(pins.shape[0]):
        for k in range(pins.shape[1]):
            if 0 <= pins[p, k] < CELLS:
                board[pins[p, k]] = p
    return board


def state_from_host(pins, current_player, rules: _L.MuzRules, action_set=None, done=None, reward=None,
                    board=None, device="cuda") -> DetMADNState:
    """Build a batch from host arrays (pins [B,P,4]); the board defaults to set_pins_on_board(pins)
    as in the reference tests (MADN/test.py:944)."""
    pins = np.asarray(pins, dtype=np.int8)
    B, P, _ = pins.shape
    if board is None:
        board = np.stack([set_pins_on_board_host(pins[b]) for b in range(B)])
    if action_set is None:
        action_set = np.full((B, P, 6), 4, dtype=np.int8)
    st = _alloc(B, P, rules, device)
    st.board.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(board, np.int8).T)))
    st.pins.copy_(torch.from_numpy(np.ascontiguousarray(pins.reshape(B, P * 4).T)))
    st.current_player.copy_(torch.from_numpy(np.asarray(current_player, np.int8).reshape(B)))
    st.reward.copy_(torch.from_numpy(np.zeros(B, np.int8) if reward is None else np.asarray(reward, np.int8)))
    st.done.copy_(torch.from_numpy(np.zeros(B, np.uint8) if done is None else np.asarray(done, np.uint8)))
    st.action_set.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(action_set, np.int8).reshape(B, P * 6).T)))
    return st


def legal_bits(env: DetMADNState, out: torch.Tensor | None = None) -> torch.Tensor:
    """valid_action as a 24-bit mask per game (bit pin*6 + move-1), int32 [B]."""
    out = torch.empty((env.batch,), dtype=torch.int32, device=env.board.device) if out is None else out
    _L.check(_L.load().muz_detmadn_legal(env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr()),
             "muz_detmadn_legal")
    return out


def bits_to_mask(bits: torch.Tensor) -> torch.Tensor:
    sh = torch.arange(ACTIONS, device=bits.device, dtype=torch.int32)
    return ((bits[:, None] >> sh[None, :]) & 1).bool()


def valid_action(env: DetMADNState) -> torch.Tensor:
    """valid_action (deterministic_madn.py:299-393) -> bool [B, 4, 6]."""
    return bits_to_mask(legal_bits(env)).reshape(env.batch, 4, 6)


def env_step(env: DetMADNState, action: torch.Tensor, next_legal: torch.Tensor | None = None):
    """env_step with action INDICES (map_action applied on device).  In place; returns (env, reward, done)."""
    action = action.to(device=env.board.device, dtype=torch.int32).contiguous()
    reward = torch.empty((env.batch,), dtype=torch.int8, device=env.board.device)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=env.board.device)
    _L.check(_L.load().muz_detmadn_step(env.rules, env.soa(), _L.ptr(action), _L.ptr(reward), _L.ptr(done),
                                        _L.ptr(next_legal), env.batch, _L.stream_ptr()), "muz_detmadn_step")
    return env, reward, done.bool()


def env_step_pin_move(env: DetMADNState, pin: torch.Tensor, move: torch.Tensor):
    """env_step(env, [pin, move]) as called by MADN/test.py:945."""
    dev = env.board.device
    pin = pin.to(device=dev, dtype=torch.int32).contiguous()
    move = move.to(device=dev, dtype=torch.int32).contiguous()
    reward = torch.empty((env.batch,), dtype=torch.int8, device=dev)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    _L.check(_L.load().muz_detmadn_step_pin_move(env.rules, env.soa(), _L.ptr(pin), _L.ptr(move), _L.ptr(reward),
                                                 _L.ptr(done), env.batch, _L.stream_ptr()), "muz_detmadn_step_pin_move")
    return env, reward, done.bool()


def no_step(env: DetMADNState):
    """no_step (deterministic_madn.py:283-297).  In place; returns (env, 0, done)."""
    reward = torch.empty((env.batch,), dtype=torch.int8, device=env.board.device)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=env.board.device)
    _L.check(_L.load().muz_detmadn_nostep(env.rules, env.soa(), _L.ptr(reward), _L.ptr(done), env.batch,
                                          _L.stream_ptr()), "muz_detmadn_nostep")
    return env, reward, done.bool()


def encode_board(env: DetMADNState, dtype=torch.float32) -> torch.Tensor:
    """encode_board (deterministic_madn.py:395-438) -> [B, 8P+2, 56]."""
    C = num_channels(env.num_players)
    out = torch.empty((env.batch, C, CELLS), dtype=dtype, device=env.board.device)
    lib = _L.load()
    if dtype == torch.float32:
        rc = lib.muz_detmadn_encode_f32(env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr())
    elif dtype == torch.int8:
        rc = lib.muz_detmadn_encode_i8(env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr())
    else:
        raise TypeError(dtype)
    _L.check(rc, "muz_detmadn_encode")
    return out


def random_round(env: DetMADNState, legal: torch.Tensor, seed: int, turn: int, obs: torch.Tensor | None = None,
                 reward: torch.Tensor | None = None, done: torch.Tensor | None = None, variant: int = 0):
    """One env-step of uniform random legal play for every game (muz_detmadn_random_round): the k-th legal
    action of ``legal`` (int32 [B], updated in place to the next mask), env_step / no_step, in-place reset of
    finished games, and encode_board of the next state into ``obs`` (int8 [B, 8P+2, 56]) when given.
    ``variant``: 0 = the kernel chosen by batch size, 1 = one game per lane, 2 / 3 / 4 / 5 = one game per
    32 / 8 / 4 / 16 lanes (same results)."""
    lib = _L.load()
    if variant == 0:
        rc = lib.muz_detmadn_random_round(env.rules, env.soa(), _L.ptr(legal), int(seed) & ((1 << 64) - 1), int(turn),
                                          _L.ptr(obs), _L.ptr(reward), _L.ptr(done), env.batch, _L.stream_ptr())
    else:
        rc = lib.muz_detmadn_random_round_variant(env.rules, env.soa(), _L.ptr(legal), int(seed) & ((1 << 64) - 1),
                                                  int(turn), _L.ptr(obs), _L.ptr(reward), _L.ptr(done), env.batch,
                                                  int(variant), _L.stream_ptr())
    _L.check(rc, "muz_detmadn_random_round")
    return env


def map_action(idx):
    """map_action (deterministic_madn.py:469-479): index -> (pin, move)."""
    return idx // 6, idx % 6 + 1
