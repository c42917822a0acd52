"""Batched DOG environment on the GPU (host mirror of DOG/dog.py).

Same conventions as ``detmadn.py`` / ``classic.py``: one ``DOGState`` holds B games as device-resident
field-major SoA tensors (include/muz.h ``muz_dog_soa``); every call is one HIP launch over the batch and
updates the state in place.  One wavefront owns a game (csrc/env_dog.hip).

Reference entry points mirrored (file:line in the reference):
  env_reset / distribute_cards / reset_deck   DOG/dog.py:83-186, 201-298, 188-191
  valid_actions (-> valid_step_actions)       DOG/dog.py:693-711 (617-691)
  env_step (play / swap phase)                DOG/dog.py:1117-1131 (986-1062, 1077-1114)
  no_step                                     DOG/dog.py:713-752
  map_action_to_move / map_move_to_action     DOG/dog.py:1133-1239 (host helpers below)

The shuffle keys of a deal come from the engine's counter RNG (include/muz.h, DOG section) instead of
jax threefry; ``oracle/dog.py:engine_shuffle_keys`` restates them for the parity tests.  The
reference's ``encode_board`` is a stub (dog.py:1264-1272), so there is no DOG observation here.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lib as _L

CELLS = 56
CARDS = 14
ACTIONS = 806
PLAY_ACTIONS = 792
BASE = 396
MASK_WORDS = 26
NORMAL_MOVES = (1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13)

# env_reset keyword defaults (dog.py:83-100)
DEFAULT_RULES = dict(
    enable_teams=False,
    enable_initial_free_pin=False,
    enable_circular_board=True,
    enable_start_blocking=False,
    enable_jump_in_goal_area=True,
    enable_friendly_fire=False,
    must_traverse_start=True,
    disable_swapping=False,
    disable_hot_seven=False,
    disable_joker=False,
)

# MuZero_DOG/game_agent.py:12-23 (config (d))
SELFPLAY_RULES = dict(
    enable_teams=True,
    enable_initial_free_pin=False,
    enable_circular_board=True,
    enable_friendly_fire=True,
    enable_start_blocking=True,
    enable_jump_in_goal_area=False,
    must_traverse_start=True,
    disable_swapping=False,
    disable_hot_seven=False,
    disable_joker=False,
)


def all_pin_distributions(total=7):
    """utils/utility_funcs.py:4-21: lex order over (a0, a1, a2), a3 = total - a0 - a1 - a2 >= 0."""
    return np.array([(a, b, c, total - a - b - c) for a in range(total + 1) for b in range(total + 1)
                     for c in range(total + 1) if total - a - b - c >= 0], np.int32)


DISTS_7_4 = all_pin_distributions(7)


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


@dataclass
class DOGState:
    """SoA batch state. Field c of game b is ``field[c, b]``."""

    board: torch.Tensor           # int8 [56, B]
    pins: torch.Tensor            # int8 [P*4, B]
    deck: torch.Tensor            # int8 [14, B]
    hands: torch.Tensor           # int8 [P*14, B]
    swap_choices: torch.Tensor    # int8 [4, B]
    current_player: torch.Tensor  # int8 [B]
    round_starter: torch.Tensor   # int8 [B]
    phase: torch.Tensor           # int8 [B]
    hand_size: torch.Tensor       # int8 [B]
    reward: torch.Tensor          # int8 [B]
    done: torch.Tensor            # uint8 [B]
    deal: torch.Tensor            # int32 [B] (uint32 counter)
    rules: _L.MuzRules
    num_players: int
    seed: int = 0

    @property
    def batch(self) -> int:
        return self.current_player.shape[0]

    def soa(self) -> _L.MuzDogSoA:
        s = _L.MuzDogSoA()
        for k in ("board", "pins", "deck", "hands", "swap_choices", "current_player", "round_starter", "phase",
                  "hand_size", "reward", "done", "deal"):
            setattr(s, k, getattr(self, k).data_ptr())
        s.stride = self.batch
        return s

    def pins_bp(self) -> torch.Tensor:
        return self.pins.T.reshape(self.batch, self.num_players, 4)

    def hands_bp(self) -> torch.Tensor:
        return self.hands.T.reshape(self.batch, self.num_players, CARDS)


def _alloc(batch: int, P: int, rules, device, seed) -> DOGState:
    kw = dict(device=device)
    i8 = dict(dtype=torch.int8, **kw)
    return DOGState(board=torch.empty((CELLS, batch), **i8), pins=torch.empty((P * 4, batch), **i8),
                    deck=torch.empty((CARDS, batch), **i8), hands=torch.empty((P * CARDS, batch), **i8),
                    swap_choices=torch.empty((4, batch), **i8), current_player=torch.empty((batch,), **i8),
                    round_starter=torch.empty((batch,), **i8), phase=torch.empty((batch,), **i8),
                    hand_size=torch.empty((batch,), **i8), reward=torch.empty((batch,), **i8),
                    done=torch.empty((batch,), dtype=torch.uint8, **kw),
                    deal=torch.empty((batch,), dtype=torch.int32, **kw), rules=rules, num_players=P,
                    seed=int(seed))


def _call(name, *args):
    _L.check(getattr(_L.load(), name)(*args), name)


def env_reset(batch: int, num_players=4, layout=(True, True, True, True), distance=10, starting_player=0,
              seed=0, device="cuda", **rules) -> DOGState:
    """Batched env_reset (dog.py:83-186): empty board, deck (joker 6, others 8), first deal."""
    r = make_rules(num_players, layout, distance, starting_player, **rules)
    st = _alloc(batch, int(num_players), r, device, seed)
    _call("muz_dog_reset", r, st.soa(), ctypes_u64(seed), batch, _L.stream_ptr())
    return st


def ctypes_u64(x: int) -> int:
    return int(x) & 0xFFFFFFFFFFFFFFFF


def state_from_host(fields: dict, rules: _L.MuzRules, seed=0, device="cuda") -> DOGState:
    """Build a batch from host arrays: pins [B,P,4], board [B,56], deck [B,14], hands [B,P,14],
    swap_choices [B,4], and per-game scalars current_player / round_starter / phase / hand_size / reward /
    done / deal."""
    pins = np.asarray(fields["pins"], np.int8)
    B, P, _ = pins.shape
    st = _alloc(B, P, rules, device, seed)

    def put(dst, a):
        dst.copy_(torch.from_numpy(np.ascontiguousarray(a)))

    put(st.board, np.asarray(fields["board"], np.int8).T)
    put(st.pins, pins.reshape(B, P * 4).T)
    put(st.deck, np.asarray(fields["deck"], np.int8).T)
    put(st.hands, np.asarray(fields["hands"], np.int8).reshape(B, P * CARDS).T)
    put(st.swap_choices, np.asarray(fields["swap_choices"], np.int8).T)
    for k in ("current_player", "round_starter", "phase", "hand_size", "reward"):
        put(getattr(st, k), np.asarray(fields[k], np.int8).reshape(B))
    put(st.done, np.asarray(fields["done"], np.uint8).reshape(B))
    put(st.deal, np.asarray(fields["deal"], np.int64).astype(np.uint32).view(np.int32).reshape(B))
    return st


def to_host(st: DOGState) -> dict:
    """Per-game host view of the batch (inverse of state_from_host)."""
    B, P = st.batch, st.num_players
    return dict(board=st.board.T.cpu().numpy(), pins=st.pins.T.cpu().numpy().reshape(B, P, 4),
                deck=st.deck.T.cpu().numpy(), hands=st.hands.T.cpu().numpy().reshape(B, P, CARDS),
                swap_choices=st.swap_choices.T.cpu().numpy(), current_player=st.current_player.cpu().numpy(),
                round_starter=st.round_starter.cpu().numpy(), phase=st.phase.cpu().numpy(),
                hand_size=st.hand_size.cpu().numpy(), reward=st.reward.cpu().numpy(),
                done=st.done.cpu().numpy(), deal=st.deal.cpu().numpy().view(np.uint32))


def legal_mask(env: DOGState, out: torch.Tensor | None = None) -> torch.Tensor:
    """valid_actions as bitsets int32 [B, 26]."""
    out = torch.empty((env.batch, MASK_WORDS), dtype=torch.int32, device=env.board.device) if out is None else out
    _call("muz_dog_legal", env.rules, env.soa(), _L.ptr(out), env.batch, _L.stream_ptr())
    return out


def unpack_mask(bits: torch.Tensor) -> torch.Tensor:
    sh = torch.arange(32, device=bits.device, dtype=torch.int32)
    return ((bits[:, :, None] >> sh) & 1).reshape(bits.shape[0], MASK_WORDS * 32)[:, :ACTIONS].bool()


def valid_actions(env: DOGState) -> torch.Tensor:
    """valid_actions (dog.py:693-711) -> bool [B, 806]."""
    return unpack_mask(legal_mask(env))


def env_step(env: DOGState, action: torch.Tensor, seed: int | None = None):
    """env_step (dog.py:1117-1131), in place; a negative action applies no_step.  Returns (env, reward, done)."""
    dev = env.board.device
    action = action.to(device=dev, dtype=torch.int32).reshape(env.batch).contiguous()
    reward = torch.empty((env.batch,), dtype=torch.int8, device=dev)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    s = env.seed if seed is None else seed
    _call("muz_dog_step", env.rules, env.soa(), _L.ptr(action), ctypes_u64(s), _L.ptr(reward), _L.ptr(done),
          env.batch, _L.stream_ptr())
    return env, reward, done.bool()


def no_step(env: DOGState, seed: int | None = None):
    """no_step (dog.py:713-752), in place.  Returns (env, reward, done)."""
    dev = env.board.device
    reward = torch.empty((env.batch,), dtype=torch.int8, device=dev)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    s = env.seed if seed is None else seed
    _call("muz_dog_nostep", env.rules, env.soa(), ctypes_u64(s), _L.ptr(reward), _L.ptr(done), env.batch,
          _L.stream_ptr())
    return env, reward, done.bool()


STEP_KINDS = {"swap": 0, "normal": 1, "neg": 2, "hot7": 3}


def step_move(env: DOGState, kind, args):
    """step_swap / step_normal_move / step_neg_move / step_hot_7 (dog.py:754-984) on their own, one per game:
    kind[b] in STEP_KINDS, args[b] = (pin, pos|move, 0, 0) or the 4-pin distribution.  Board and pins change
    in place; returns (env, reward, done) like the reference functions."""
    dev = env.board.device
    k = torch.as_tensor(np.asarray([STEP_KINDS.get(x, x) for x in kind], np.int32), device=dev)
    a = torch.as_tensor(np.asarray(args, np.int32).reshape(env.batch, 4), device=dev).contiguous()
    reward = torch.empty((env.batch,), dtype=torch.int8, device=dev)
    done = torch.empty((env.batch,), dtype=torch.uint8, device=dev)
    _call("muz_dog_step_move", env.rules, env.soa(), _L.ptr(k), _L.ptr(a), _L.ptr(reward), _L.ptr(done), env.batch,
          _L.stream_ptr())
    return env, reward, done.bool()


def random_action(mask: torch.Tensor, uniform: torch.Tensor | None = None, seed=0, turn=0,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Uniform random legal action per game from the bitset mask (-1 if none)."""
    B = mask.shape[0]
    out = torch.empty((B,), dtype=torch.int32, device=mask.device) if out is None else out
    u = None if uniform is None else uniform.to(device=mask.device, dtype=torch.float32).contiguous()
    _call("muz_dog_random_action", _L.ptr(mask), _L.ptr(u), ctypes_u64(seed), int(turn), _L.ptr(out), B,
          _L.stream_ptr())
    return out


# ---- action <-> move helpers (dog.py:1133-1262), host side ---------------------------------------------
def map_action_to_move(action: int):
    """-> (kind, pin, value, joker): kind in {"swap", "hot7", "normal", "neg", "swap_card"}; value = swap
    position / distribution row / move / card."""
    a = int(action)
    if a >= PLAY_ACTIONS:
        return "swap_card", -1, a - PLAY_ACTIONS, False
    joker, i = a < BASE, a % BASE
    if i < 224:
        return "swap", i // CELLS, i % CELLS, joker
    if i < 344:
        return "hot7", -1, i - 224, joker
    if i < 392:
        return "normal", (i - 344) // 12, NORMAL_MOVES[(i - 344) % 12], joker
    return "neg", i - 392, -4, joker


def map_move_to_action(kind: str, pin: int, value: int, joker: bool) -> int:
    off = 0 if joker else BASE
    if kind == "swap_card":
        return PLAY_ACTIONS + int(value)
    if kind == "swap":
        return off + int(pin) * CELLS + int(value)
    if kind == "hot7":
        return off + 224 + int(value)
    if kind == "normal":
        return off + 344 + int(pin) * 12 + NORMAL_MOVES.index(int(value))
    return off + 392 + int(pin)


class RandomPlay:
    """Config (d)'s actor: B DOG games advanced by a uniform random legal action per turn, all on device
    (legal mask -> random action -> step; no_step when nothing is legal, as the step kernel does for -1).
    ``turn()`` is one batched env-step.  ``fused=True`` runs the whole turn as one kernel
    (muz_dog_random_turn: the mask stays in registers, finished games are skipped); otherwise three
    launches (legal mask -> random action -> step) that also step finished games, as env_step would."""

    def __init__(self, batch: int, seed=0, num_players=4, fused=True, **rules):
        r = dict(SELFPLAY_RULES)
        r.update(rules)
        self.env = env_reset(batch, num_players=num_players, seed=seed, **r)
        self.seed = int(seed)
        self.fused = bool(fused)
        self.t = 0
        dev = self.env.board.device
        self.mask = torch.empty((batch, MASK_WORDS), dtype=torch.int32, device=dev)
        self.action = torch.empty((batch,), dtype=torch.int32, device=dev)
        self.reward = torch.empty((batch,), dtype=torch.int8, device=dev)
        self.done = torch.empty((batch,), dtype=torch.uint8, device=dev)
        self._soa = self.env.soa()
        self._lib = _L.load()

    def turn(self):
        e, lib, s = self.env, self._lib, _L.stream_ptr()
        if self.fused:
            _L.check(lib.muz_dog_random_turn(e.rules, self._soa, ctypes_u64(self.seed), self.t, _L.ptr(self.action),
                                             _L.ptr(self.reward), _L.ptr(self.done), e.batch, s),
                     "muz_dog_random_turn")
            self.t += 1
            return
        _L.check(lib.muz_dog_legal(e.rules, self._soa, _L.ptr(self.mask), e.batch, s), "muz_dog_legal")
        _L.check(lib.muz_dog_random_action(_L.ptr(self.mask), None, ctypes_u64(self.seed), self.t,
                                           _L.ptr(self.action), e.batch, s), "muz_dog_random_action")
        _L.check(lib.muz_dog_step(e.rules, self._soa, _L.ptr(self.action), ctypes_u64(self.seed),
                                  _L.ptr(self.reward), _L.ptr(self.done), e.batch, s), "muz_dog_step")
        self.t += 1

    def play(self, nturns: int, env_steps: torch.Tensor | None = None, auto_reset: bool = False,
             episodes: torch.Tensor | None = None, record: "DogTrajectory | None" = None):
        """``nturns`` fused turns in ONE launch (muz_dog_random_play: every game stays in LDS for all of
        them).  ``env_steps`` / ``episodes`` (int32 [B]) accumulate turns played / games finished; with
        ``auto_reset`` a finished game restarts in place and keeps playing.  ``record`` (a DogTrajectory)
        receives one row per turn and game (muz_dog_random_play_record)."""
        e = self.env
        if record is None:
            _L.check(self._lib.muz_dog_random_play(e.rules, self._soa, ctypes_u64(self.seed), self.t, int(nturns),
                                                   int(bool(auto_reset)), _L.ptr(env_steps), _L.ptr(episodes),
                                                   e.batch, _L.stream_ptr()), "muz_dog_random_play")
        else:
            if record.batch != e.batch:
                raise ValueError("record batch differs from the actor's")
            _L.check(self._lib.muz_dog_random_play_record(e.rules, self._soa, ctypes_u64(self.seed), self.t,
                                                          int(nturns), int(bool(auto_reset)), _L.ptr(env_steps),
                                                          _L.ptr(episodes), record.struct(), e.batch,
                                                          _L.stream_ptr()), "muz_dog_random_play_record")
        self.t += int(nturns)


# ---- DOG actor trajectories (config (d): actors -> learner over RCCL) -----------------------------------
DOG_TRAJ_FIELDS = (("act", torch.int32), ("player", torch.int32), ("reward", torch.int32), ("legal", torch.int32),
                   ("done", torch.uint8))


class DogTrajectory:
    """Per-turn records of the DOG actor (muz_dog_traj in include/muz.h): [B, T] action (-1 = no_step),
    player who moved, reward, number of legal actions, game-finished flag, and idx [B] rows recorded.  The
    reference's DOG agent is a stub (MuZero_DOG/game_agent.py:52-57), so this record is the engine's own
    (parity-unpinned); transfer.gather_packed moves packed records to a learner rank like det games."""

    def __init__(self, batch: int, max_steps: int, device="cuda"):
        self.batch, self.T = int(batch), int(max_steps)
        self.buf = {k: torch.zeros((self.batch, self.T), dtype=dt, device=device) for k, dt in DOG_TRAJ_FIELDS}
        self.buf["idx"] = torch.zeros((self.batch,), dtype=torch.int32, device=device)

    def struct(self) -> _L.MuzDogTraj:
        t = _L.MuzDogTraj()
        for k, _ in DOG_TRAJ_FIELDS:
            setattr(t, k, self.buf[k].data_ptr())
        t.idx = self.buf["idx"].data_ptr()
        t.max_steps = self.T
        return t

    def reset(self):
        self.buf["idx"].zero_()

    def pack(self) -> dict:
        """Rows [0, idx) of every lane, contiguous per lane in lane order (the packed layout of
        transfer.pack): every field [R] with R = sum(idx), plus idx [B] and row_offset [B] (int64)."""
        idx = self.buf["idx"]
        full = int(idx.sum().item()) == self.batch * self.T      # one host sync
        if full:        # every lane recorded T rows (e.g. auto-reset play): the [B, T] buffers are the packed rows
            out = {k: self.buf[k].reshape(-1).clone() for k, _ in DOG_TRAJ_FIELDS}
            out["row_offset"] = torch.arange(self.batch, dtype=torch.int64, device=idx.device) * self.T
        else:
            keep = torch.arange(self.T, device=idx.device)[None, :] < idx[:, None]
            flat = keep.reshape(-1).nonzero().squeeze(1)
            out = {k: self.buf[k].reshape(-1).index_select(0, flat) for k, _ in DOG_TRAJ_FIELDS}
            out["row_offset"] = torch.cumsum(idx.to(torch.int64), 0) - idx.to(torch.int64)
        out["idx"] = idx.clone()
        return out
