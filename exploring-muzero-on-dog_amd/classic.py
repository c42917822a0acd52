"""Batched classic MADN environment on the GPU (host mirror of MADN/classic_madn.py).

Same conventions as ``detmadn.py``: one ``ClassicMADNState`` holds B games as device-resident
field-major SoA tensors (include/muz.h ``muz_classic_soa``); every call is one HIP launch over the
batch and updates the state in place.

Reference entry points mirrored (file:line in the reference):
  env_reset            MADN/classic_madn.py:51-131  (+ MuZero_Classic_MADN/game_agent_stochastic.py:25-44)
  is_soft_locked       MADN/classic_madn.py:180-206
  dice_probabilities   MADN/classic_madn.py:208-228
  throw_die            MADN/classic_madn.py:230-242  (uniform draw passed in: the threefry source is not restated)
  set_die              MADN/classic_madn.py:244-255
  env_step             MADN/classic_madn.py:257-337
  no_step              MADN/classic_madn.py:353-365
  valid_action         MADN/classic_madn.py:367-461
  encode_board         MADN/classic_madn.py:463-497
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lib as _L
from .detmadn import set_pins_on_board_host

CELLS = 56
ACTIONS = 4

# MuZero_Classic_MADN/game_agent_stochastic.py:13-24
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
    enable_dice_rethrow=True,
)

# env_reset keyword defaults (classic_madn.py:51-67)
DEFAULT_RULES = dict(
    enable_teams=False,
    enable_initial_free_pin=False,
    enable_circular_board=True,
    enable_start_blocking=False,
    enable_jump_in_goal_area=True,
    enable_friendly_fire=False,
    enable_start_on_1=True,
    enable_bonus_turn_on_6=True,
    enable_dice_rethrow=False,
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
    """encode_board channel count: P + 2 + P + 1 (classic_madn.py:494)."""
    return 2 * num_players + 3


@dataclass
class ClassicMADNState:
    """SoA batch state. Field c of game b is ``field[c, b]``."""

    board: torch.Tensor           # int8 [56, B]
    pins: torch.Tensor            # int8 [P*4, B]
    current_player: torch.Tensor  # int8 [B]
    reward: torch.Tensor          # int8 [B]
    done: torch.Tensor            # uint8 [B]
    die: torch.Tensor             # int8 [B]
    rules: _L.MuzRules
    num_players: int

    @property
    def batch(self) -> int:
        return self.current_player.shape[0]

    def soa(self) -> _L.MuzClassicSoA:
        s = _L.MuzClassicSoA()
        s.board = self.board.data_ptr()
        s.pins = self.pins.data_ptr()
        s.current_player = self.current_player.data_ptr()
        s.reward = self.reward.data_ptr()
        s.done = self.done.data_ptr()
        s.die = self.die.data_ptr()
        s.stride = self.batch
        return s

    def pins_bp(self) -> torch.Tensor:
        return self.pins.T.reshape(self.batch, self.num_players, 4)


def _alloc(batch: int, P: int, rules, device) -> ClassicMADNState:
    kw = dict(device=device)
    return ClassicMADNState(
        board=torch.empty((CELLS, batch), dtype=torch.int8, **kw),
        pins=torch.empty((P * 4, batch), dtype=torch.int8, **kw),
        current_player=torch.empty((batch,), dtype=torch.int8, **kw),
        reward=torch.empty((batch,), dtype=torch.int8, **kw),
        done=torch.empty((batch,), dtype=torch.uint8, **kw),
        die=torch.empty((batch,), dtype=torch.int8, **kw),
        rules=rules,
        num_players=P,
    )


def _call(name, *args):
    _L.check(getattr(_L.load(), name)(*args), name)


def env_reset(batch: int, num_players=4, layout=(True, True, True, True), distance=10, starting_player=0,
              device="cuda", seeds=None, **rules) -> ClassicMADNState:
    """Batched env_reset (classic_madn.py:51-131); ``seeds`` as detmadn.env_reset (a random starting player)."""
    r = make_rules(num_players, layout, distance, starting_player, **rules)
    st = _alloc(batch, int(num_players), r, device)
    if seeds is None:
        _call("muz_classic_reset", r, st.soa(), batch, _L.stream_ptr())
    else:
        sd = torch.as_tensor(np.asarray(seeds, np.int64) & 0xFFFFFFFF).to(torch.int64)
        sd = (sd - ((sd >> 31) << 32)).to(device=device, dtype=torch.int32).contiguous()
        if sd.numel() != batch:
            raise ValueError("one seed per game")
        _call("muz_classic_reset_seeded", r, st.soa(), _L.ptr(sd), batch, _L.stream_ptr())
    return st


def state_from_host(pins, current_player, rules: _L.MuzRules, die=None, done=None, reward=None, board=None,
                    device="cuda") -> ClassicMADNState:
    """Build a batch from host arrays (pins [B,P,4]); the board defaults to set_pins_on_board(pins)."""
    pins = np.asarray(pins, dtype=np.int8)
    B, P, _ = pins.shape
    if board is None:
        board = np.stack([set_pins_on_board_host(pins[b]) for b in range(B)])
    st = _alloc(B, P, rules, device)
    st.board.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(board, np.int8).T)))
    st.pins.copy_(torch.from_numpy(np.ascontiguousarray(pins.reshape(B, P * 4).T)))
    st.current_player.copy_(torch.from_numpy(np.asarray(current_player, np.int8).reshape(B)))
    st.reward.copy_(torch.from_numpy(np.zeros(B, np.int8) if reward is None else np.asarray(reward, np.int8)))
    st.done.copy_(torch.from_numpy(np.zeros(B, np.uint8) if done is None else np.asarray(done, np.uint8)))
    st.die.copy_(torch.from_numpy(np.zeros(B, np.int8) if die is None else np.asarray(die, np.int8)))
    return st


def set_die(env: ClassicMADNState, die) -> ClassicMADNState:
    """set_die (classic_madn.py:244-255), in place."""
    die = torch.as_tensor(die, dtype=torch.int32, device=env.board.device).reshape(env.batch).contiguous()
    _call("muz_classic_set_die", env.rules, env.soa(), _L.ptr(die), env.batch, _L.stream_ptr())
    return env


def dice_probabilities(env: ClassicMADNState, with_soft_lock=False):
    """dice_probabilities (classic_madn.py:208-228) -> float32 [B, 6] (+ is_soft_locked uint8 [B])."""
    dev = env.board.device
    probs = torch.empty((env.batch, 6), dtype=torch.float32, device=dev)
    soft = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    _call("muz_classic_dice_probs", env.rules, env.soa(), _L.ptr(probs), _L.ptr(soft), env.batch, _L.stream_ptr())
    return (probs, soft.bool()) if with_soft_lock else probs


def throw_die(env: ClassicMADNState, uniform: torch.Tensor) -> ClassicMADNState:
    """throw_die (classic_madn.py:230-242) with the uniform draw given: in place."""
    u = uniform.to(device=env.board.device, dtype=torch.float32).reshape(env.batch).contiguous()
    _call("muz_classic_throw_die", env.rules, env.soa(), _L.ptr(u), None, env.batch, _L.stream_ptr())
    return env


def legal_bits(env: ClassicMADNState, out: torch.Tensor | None = None) -> torch.Tensor:
    out = torch.empty((env.batch,), dtype=torch.int32, device=env.board.device) if out is None else out
    _call("muz_classic_legal", env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr())
    return out


def valid_action(env: ClassicMADNState) -> torch.Tensor:
    """valid_action (classic_madn.py:367-461) -> bool [B, 4]."""
    bits = legal_bits(env)
    sh = torch.arange(ACTIONS, device=bits.device, dtype=torch.int32)
    return ((bits[:, None] >> sh[None, :]) & 1).bool()


def env_step(env: ClassicMADNState, pin: torch.Tensor):
    """env_step (classic_madn.py:257-337) with one pin index per game.  In place; returns (env, reward, done)."""
    dev = env.board.device
    pin = pin.to(device=dev, dtype=torch.int32).reshape(env.batch).contiguous()
    reward = torch.empty((env.batch,), dtype=torch.int8, device=dev)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    _call("muz_classic_step", env.rules, env.soa(), _L.ptr(pin), _L.ptr(reward), _L.ptr(done), env.batch,
          _L.stream_ptr())
    return env, reward, done.bool()


def no_step(env: ClassicMADNState):
    """no_step (classic_madn.py:353-365).  In place; returns (env, 0, done)."""
    dev = env.board.device
    reward = torch.empty((env.batch,), dtype=torch.int8, device=dev)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    _call("muz_classic_nostep", env.rules, env.soa(), _L.ptr(reward), _L.ptr(done), env.batch, _L.stream_ptr())
    return env, reward, done.bool()


def encode_board(env: ClassicMADNState, dtype=torch.float32) -> torch.Tensor:
    """encode_board (classic_madn.py:463-497) -> [B, 2P+3, 56]."""
    C = num_channels(env.num_players)
    out = torch.empty((env.batch, C, CELLS), dtype=dtype, device=env.board.device)
    if dtype == torch.float32:
        _call("muz_classic_encode_f32", env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr())
    elif dtype == torch.int8:
        _call("muz_classic_encode_i8", env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr())
    else:
        raise TypeError(dtype)
    return out
