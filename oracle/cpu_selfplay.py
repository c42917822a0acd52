"""ctypes binding of the C++ CPU restatement (oracle/cpu_selfplay.cpp -> oracle/libmuzcpu.so).

TEST INFRASTRUCTURE / CPU BASELINE ONLY: used by tests/test_cpu_baseline.py (checked against the NumPy
oracle) and by bench.py's cpu_baseline leg (the reference algorithm timed on the host cores,
at 1 core and at all cores).  The product path never loads it."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmuzcpu.so")

R_TEAMS, R_FREE_PIN, R_CIRCULAR, R_START_BLOCK, R_JUMP_GOAL, R_FRIENDLY, R_START_ON_1, R_BONUS_6, \
    R_MUST_TRAVERSE = (1 << i for i in range(9))
_FLAGS = dict(enable_teams=R_TEAMS, enable_initial_free_pin=R_FREE_PIN, enable_circular_board=R_CIRCULAR,
              enable_start_blocking=R_START_BLOCK, enable_jump_in_goal_area=R_JUMP_GOAL,
              enable_friendly_fire=R_FRIENDLY, enable_start_on_1=R_START_ON_1, enable_bonus_turn_on_6=R_BONUS_6,
              must_traverse_start=R_MUST_TRAVERSE)


class Det(ctypes.Structure):
    _fields_ = [("board", ctypes.c_int8 * 56), ("pins", ctypes.c_int8 * 16), ("action_set", ctypes.c_int8 * 24),
                ("start", ctypes.c_int8 * 4), ("target", ctypes.c_int8 * 4), ("goal", ctypes.c_int8 * 16),
                ("current_player", ctypes.c_int32), ("reward", ctypes.c_int32), ("done", ctypes.c_int32),
                ("num_players", ctypes.c_int32), ("board_size", ctypes.c_int32), ("total", ctypes.c_int32),
                ("rules", ctypes.c_int32)]


class Traj(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("val", ctypes.c_void_p), ("pol", ctypes.c_void_p),
                ("mask", ctypes.c_void_p), ("idx", ctypes.c_void_p)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: make -C oracle")
        L = ctypes.CDLL(LIB_PATH)
        vp, ip, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.muzcpu_net_create.restype = vp
        L.muzcpu_net_create.argtypes = [vp, vp, vp, ip, ip]
        L.muzcpu_net_destroy.argtypes = [vp]
        L.muzcpu_env_reset.argtypes = [vp, ip, vp, ip, ip, ip]
        L.muzcpu_valid_action.argtypes = [vp, vp]
        L.muzcpu_env_step.argtypes = [vp, ip, ip, vp, vp]
        L.muzcpu_no_step.argtypes = [vp]
        L.muzcpu_encode.argtypes = [vp, vp]
        L.muzcpu_root.argtypes = [vp, vp, ip, vp, vp, vp]
        L.muzcpu_recurrent.argtypes = [vp, vp, vp, ip, vp, vp, vp, vp, vp]
        L.muzcpu_selfplay.restype = ip
        L.muzcpu_selfplay.argtypes = [vp, ip, ip, ip, ip, ip, ip, fp, ctypes.c_uint64, vp]
        L.muzcpu_bench.restype = ctypes.c_int64
        L.muzcpu_bench.argtypes = [vp, ip, ip, ip, ip, ip, ip, fp, ctypes.c_uint64, ip, ctypes.c_double, vp, vp, vp]
        L.muzcpu_env_bench.restype = ctypes.c_int64
        L.muzcpu_env_bench.argtypes = [ip, ip, ip, ctypes.c_uint64, ip, ctypes.c_double, vp]
        _lib = L
    return _lib


def rule_bits(**rules) -> int:
    from oracle import detmadn as dm
    r = dict(dm.DEFAULT_RULES)
    r.update(rules)
    return sum(bit for k, bit in _FLAGS.items() if r[k])


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class CpuNet:
    """Flat Flax-path parameter dict -> the C++ network (copied once)."""

    def __init__(self, params: dict, obs_channels: int):
        L = load()
        self._keep = {k: np.ascontiguousarray(v, np.float32) for k, v in params.items()}
        names = [k.encode() for k in self._keep]
        n = len(names)
        cn = (ctypes.c_char_p * n)(*names)
        ptrs = (ctypes.c_void_p * n)(*[v.ctypes.data for v in self._keep.values()])
        sizes = (ctypes.c_int64 * n)(*[v.size for v in self._keep.values()])
        self.h = L.muzcpu_net_create(cn, ptrs, sizes, n, obs_channels)
        self.C = obs_channels
        self.A = int(self._keep["prediction/Dense_2/bias"].size) if "prediction/Dense_2/bias" in self._keep else 24

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.muzcpu_net_destroy(self.h)
            self.h = None

    def root(self, obs):
        obs = np.ascontiguousarray(obs, np.float32)
        B = obs.shape[0]
        lg, v, e = np.empty((B, self.A), np.float32), np.empty(B, np.float32), np.empty((B, 256), np.float32)
        load().muzcpu_root(self.h, _p(obs), B, _p(lg), _p(v), _p(e))
        return lg, v, e

    def recurrent(self, action, emb):
        a = np.ascontiguousarray(action, np.int32)
        emb = np.ascontiguousarray(emb, np.float32)
        B = emb.shape[0]
        r, d, v = (np.empty(B, np.float32) for _ in range(3))
        lg, nx = np.empty((B, self.A), np.float32), np.empty((B, 256), np.float32)
        fn = load().muzcpu_recurrent if self.A == 24 else _dog_lib().muzcpu_dog_recurrent
        fn(self.h, _p(a), _p(emb), B, _p(r), _p(d), _p(lg), _p(v), _p(nx))
        return r, d, lg, v, nx

    # ---- the DOG MuZero slice (A = 806; oracle/cpu_dog.cpp) ----
    def dog_search(self, logits, value, emb, invalid, gumbel, S, D):
        """One batched gumbel_muzero_policy at A = 806: (action [B], action_weights [B, 806], root_value [B])."""
        lg = np.ascontiguousarray(logits, np.float32)
        B = lg.shape[0]
        v, e = np.ascontiguousarray(value, np.float32), np.ascontiguousarray(emb, np.float32)
        inv = np.ascontiguousarray(invalid, np.uint8)
        g = np.ascontiguousarray(gumbel, np.float32)
        act, w, rv = np.empty(B, np.int32), np.empty((B, 806), np.float32), np.empty(B, np.float32)
        _dog_lib().muzcpu_dog_search(self.h, B, S, D, _p(lg), _p(v), _p(e), _p(inv), _p(g), _p(act), _p(w), _p(rv))
        return act, w, rv

    def dog_play(self, rules, n, turns, S, D, temp, seed):
        """n lanes of DOG MuZero self-play on one thread: (actions [turns, n], searches)."""
        acts = np.zeros((turns, n), np.int32)
        k = _dog_lib().muzcpu_dog_mz_play(self.h, dog_rule_bits(**rules), n, turns, S, D, temp, seed, _p(acts))
        return acts, int(k)

    def dog_bench(self, rules, lanes, S, D, temp, seed, threads, seconds):
        """DOG MuZero self-play on `threads` cores for `seconds`: dict(env_steps, searches, games, elapsed)."""
        s, g, t = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        steps = _dog_lib().muzcpu_dog_mz_bench(self.h, dog_rule_bits(**rules), lanes, S, D, temp, seed, threads, seconds,
                                               ctypes.byref(s), ctypes.byref(g), ctypes.byref(t))
        return dict(env_steps=int(steps), searches=int(s.value), games=int(g.value), elapsed=float(t.value))

    def selfplay(self, P, rules, n, S, D, T, temp, seed):
        """play_batch_of_games of n games (one thread): (buffers act / val / pol / mask / idx, turns)."""
        buf = {"act": np.zeros((n, T), np.int32), "val": np.zeros((n, T), np.float32),
               "pol": np.zeros((n, T, 24), np.float32), "mask": np.zeros((n, T), np.float32),
               "idx": np.zeros(n, np.int32)}
        tr = Traj(*[buf[k].ctypes.data for k in ("act", "val", "pol", "mask", "idx")])
        turns = load().muzcpu_selfplay(self.h, P, rule_bits(**rules), n, S, D, T, temp, seed, ctypes.byref(tr))
        return buf, turns

    def bench(self, P, rules, lanes, S, D, T, temp, seed, threads, seconds):
        """Streamed self-play on `threads` cores for `seconds`: dict(env_steps, searches, games, elapsed)."""
        s, g, t = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        steps = load().muzcpu_bench(self.h, P, rule_bits(**rules), lanes, S, D, T, temp, seed, threads, seconds,
                                    ctypes.byref(s), ctypes.byref(g), ctypes.byref(t))
        return dict(env_steps=int(steps), searches=int(s.value), games=int(g.value), elapsed=float(t.value))


def env_bench(P, rules, lanes, seed, threads, seconds):
    """Random-play env rounds on `threads` host cores for `seconds`: (env_steps, elapsed)."""
    t = ctypes.c_double()
    steps = load().muzcpu_env_bench(P, rule_bits(**rules), lanes, seed, threads, seconds, ctypes.byref(t))
    return int(steps), float(t.value)


def env_from_oracle(e) -> Det:
    """oracle/detmadn.State -> the C++ state struct."""
    d = Det()
    P = e.num_players
    d.board[:] = [int(x) for x in e.board]
    pins = -np.ones(16, np.int8)
    pins[:P * 4] = np.asarray(e.pins, np.int8).ravel()
    d.pins[:] = [int(x) for x in pins]
    aset = np.zeros(24, np.int8)
    aset[:P * 6] = np.asarray(e.action_set, np.int8).ravel()
    d.action_set[:] = [int(x) for x in aset]
    st, tg, gl = np.zeros(4, np.int8), np.zeros(4, np.int8), np.zeros(16, np.int8)
    st[:P], tg[:P], gl[:P * 4] = e.start, e.target, np.asarray(e.goal).ravel()
    d.start[:], d.target[:], d.goal[:] = [int(x) for x in st], [int(x) for x in tg], [int(x) for x in gl]
    d.current_player, d.reward, d.done = int(e.current_player), int(e.reward), int(e.done)
    d.num_players, d.board_size, d.total = P, e.board_size, e.total_board_size
    d.rules = rule_bits(**e.rules)
    return d


def valid_action(d: Det) -> np.ndarray:
    out = np.zeros(24, np.uint8)
    load().muzcpu_valid_action(ctypes.byref(d), _p(out))
    return out.astype(bool).reshape(4, 6)


def env_step(d: Det, pin, move):
    r, dn = ctypes.c_int(), ctypes.c_int()
    load().muzcpu_env_step(ctypes.byref(d), int(pin), int(move), ctypes.byref(r), ctypes.byref(dn))
    return r.value, bool(dn.value)


def no_step(d: Det):
    load().muzcpu_no_step(ctypes.byref(d))


def encode(d: Det) -> np.ndarray:
    C = 8 * d.num_players + 2
    out = np.zeros((C, 56), np.float32)
    load().muzcpu_encode(ctypes.byref(d), _p(out))
    return out


def pins(d: Det) -> np.ndarray:
    return np.array(d.pins[:d.num_players * 4], np.int8).reshape(d.num_players, 4)


# ---- classic MADN: Stochastic MuZero (oracle/cpu_classic.cpp) ---------------------------------------------
R_DICE_RETHROW = 1 << 9


class Classic(ctypes.Structure):
    _fields_ = [("board", ctypes.c_int8 * 56), ("pins", ctypes.c_int8 * 16), ("start", ctypes.c_int8 * 4),
                ("target", ctypes.c_int8 * 4), ("goal", ctypes.c_int8 * 16), ("current_player", ctypes.c_int32),
                ("reward", ctypes.c_int32), ("done", ctypes.c_int32), ("num_players", ctypes.c_int32),
                ("board_size", ctypes.c_int32), ("total", ctypes.c_int32), ("rules", ctypes.c_int32),
                ("die", ctypes.c_int32)]


class CTraj(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("val", ctypes.c_void_p), ("pol", ctypes.c_void_p),
                ("mask", ctypes.c_void_p), ("dice", ctypes.c_void_p), ("idx", ctypes.c_void_p)]


_classic_bound = False


def _classic_lib():
    global _classic_bound
    L = load()
    if not _classic_bound:
        vp, ip, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.muzcpu_classic_net_create.restype = vp
        L.muzcpu_classic_net_create.argtypes = [vp, vp, vp, ip, ip]
        L.muzcpu_classic_net_destroy.argtypes = [vp]
        L.muzcpu_classic_reset.argtypes = [vp, ip, vp, ip, ip, ip]
        L.muzcpu_classic_valid_action.argtypes = [vp, vp]
        L.muzcpu_classic_step.argtypes = [vp, ip, vp, vp]
        L.muzcpu_classic_no_step.argtypes = [vp]
        L.muzcpu_classic_encode.argtypes = [vp, vp]
        L.muzcpu_classic_soft_locked.argtypes = [vp]
        L.muzcpu_classic_soft_locked.restype = ip
        L.muzcpu_classic_dice_probs.argtypes = [vp, vp]
        L.muzcpu_classic_throw_die.argtypes = [vp, fp]
        L.muzcpu_classic_root.argtypes = [vp, vp, ip, vp, vp, vp]
        L.muzcpu_classic_decision.argtypes = [vp, vp, vp, ip, vp, vp, vp, vp, vp]
        L.muzcpu_classic_chance.argtypes = [vp, vp, vp, ip, vp, vp, vp]
        L.muzcpu_classic_selfplay.restype = ip
        L.muzcpu_classic_selfplay.argtypes = [vp, ip, ip, ip, ip, ip, ip, fp, ctypes.c_uint64, fp, vp]
        L.muzcpu_classic_bench.restype = ctypes.c_int64
        L.muzcpu_classic_bench.argtypes = [vp, ip, ip, ip, ip, ip, ip, fp, ctypes.c_uint64, fp, ip, ctypes.c_double,
                                           vp, vp, vp]
        _classic_bound = True
    return L


def classic_rule_bits(**rules) -> int:
    from oracle import classic_madn as cm
    r = dict(cm.DEFAULT_RULES)
    r.update(rules)
    bits = sum(bit for k, bit in _FLAGS.items() if r[k])
    return bits | (R_DICE_RETHROW if r["enable_dice_rethrow"] else 0)


def classic_from_oracle(e) -> Classic:
    """oracle/classic_madn.State -> the C++ state struct."""
    d = Classic()
    P = e.num_players
    d.board[:] = [int(x) for x in e.board]
    pins = -np.ones(16, np.int8)
    pins[:P * 4] = np.asarray(e.pins, np.int8).ravel()
    d.pins[:] = [int(x) for x in pins]
    st, tg, gl = np.zeros(4, np.int8), np.zeros(4, np.int8), np.zeros(16, np.int8)
    st[:P], tg[:P], gl[:P * 4] = e.start, e.target, np.asarray(e.goal).ravel()
    d.start[:], d.target[:], d.goal[:] = [int(x) for x in st], [int(x) for x in tg], [int(x) for x in gl]
    d.current_player, d.reward, d.done, d.die = int(e.current_player), int(e.reward), int(e.done), int(e.die)
    d.num_players, d.board_size, d.total = P, e.board_size, e.total_board_size
    d.rules = classic_rule_bits(**e.rules)
    return d


def classic_valid_action(d: Classic) -> np.ndarray:
    out = np.zeros(4, np.uint8)
    _classic_lib().muzcpu_classic_valid_action(ctypes.byref(d), _p(out))
    return out.astype(bool)


def classic_step(d: Classic, pin):
    r, dn = ctypes.c_int(), ctypes.c_int()
    _classic_lib().muzcpu_classic_step(ctypes.byref(d), int(pin), ctypes.byref(r), ctypes.byref(dn))
    return r.value, bool(dn.value)


def classic_no_step(d: Classic):
    _classic_lib().muzcpu_classic_no_step(ctypes.byref(d))


def classic_encode(d: Classic) -> np.ndarray:
    out = np.zeros((2 * d.num_players + 3, 56), np.float32)
    _classic_lib().muzcpu_classic_encode(ctypes.byref(d), _p(out))
    return out


def classic_dice(d: Classic):
    p = np.zeros(6, np.float32)
    L = _classic_lib()
    L.muzcpu_classic_dice_probs(ctypes.byref(d), _p(p))
    return bool(L.muzcpu_classic_soft_locked(ctypes.byref(d))), p


def classic_throw_die(d: Classic, u: float):
    _classic_lib().muzcpu_classic_throw_die(ctypes.byref(d), float(u))


class CpuClassicNet:
    """Flat Flax-path classic parameter dict (Repr2 / StochasticDynamicsNetwork4 / Pred4, A = 4) -> C++ network."""

    def __init__(self, params: dict, obs_channels: int):
        L = _classic_lib()
        self._keep = {k: np.ascontiguousarray(v, np.float32) for k, v in params.items()}
        names = [k.encode() for k in self._keep]
        n = len(names)
        cn = (ctypes.c_char_p * n)(*names)
        ptrs = (ctypes.c_void_p * n)(*[v.ctypes.data for v in self._keep.values()])
        sizes = (ctypes.c_int64 * n)(*[v.size for v in self._keep.values()])
        self.h = L.muzcpu_classic_net_create(cn, ptrs, sizes, n, obs_channels)
        self.C = obs_channels

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.muzcpu_classic_net_destroy(self.h)
            self.h = None

    def root(self, obs):
        obs = np.ascontiguousarray(obs, np.float32)
        B = obs.shape[0]
        lg, v, e = np.empty((B, 4), np.float32), np.empty(B, np.float32), np.empty((B, 256), np.float32)
        _classic_lib().muzcpu_classic_root(self.h, _p(obs), B, _p(lg), _p(v), _p(e))
        return lg, v, e

    def decision(self, action, emb):
        """-> (chance_logits, afterstate_value, afterstate, reward, discount) (oracle/classic_nets.decision_recurrent)."""
        a = np.ascontiguousarray(action, np.int32)
        emb = np.ascontiguousarray(emb, np.float32)
        B = emb.shape[0]
        cl, av, af = np.empty((B, 6), np.float32), np.empty(B, np.float32), np.empty((B, 256), np.float32)
        r, d = np.empty(B, np.float32), np.empty(B, np.float32)
        _classic_lib().muzcpu_classic_decision(self.h, _p(a), _p(emb), B, _p(cl), _p(av), _p(af), _p(r), _p(d))
        return cl, av, af, r, d

    def chance(self, outcome, after):
        """-> (action_logits, value, next_state) (oracle/classic_nets.chance_recurrent)."""
        c = np.ascontiguousarray(outcome, np.int32)
        after = np.ascontiguousarray(after, np.float32)
        B = after.shape[0]
        lg, v, nx = np.empty((B, 4), np.float32), np.empty(B, np.float32), np.empty((B, 256), np.float32)
        _classic_lib().muzcpu_classic_chance(self.h, _p(c), _p(after), B, _p(lg), _p(v), _p(nx))
        return lg, v, nx

    def selfplay(self, P, rules, n, S, D, T, temp, seed, dirichlet_fraction=0.0):
        buf = {"act": np.zeros((n, T), np.int32), "val": np.zeros((n, T), np.float32),
               "pol": np.zeros((n, T, 4), np.float32), "mask": np.zeros((n, T), np.float32),
               "dice": np.zeros((n, T), np.int32), "idx": np.zeros(n, np.int32)}
        tr = CTraj(*[buf[k].ctypes.data for k in ("act", "val", "pol", "mask", "dice", "idx")])
        turns = _classic_lib().muzcpu_classic_selfplay(self.h, P, classic_rule_bits(**rules), n, S, D, T, temp, seed,
                                                       dirichlet_fraction, ctypes.byref(tr))
        return buf, turns

    def bench(self, P, rules, lanes, S, D, T, temp, seed, threads, seconds, dirichlet_fraction=0.25):
        s, g, t = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        steps = _classic_lib().muzcpu_classic_bench(self.h, P, classic_rule_bits(**rules), lanes, S, D, T, temp, seed,
                                                    dirichlet_fraction, threads, seconds, ctypes.byref(s),
                                                    ctypes.byref(g), ctypes.byref(t))
        return dict(env_steps=int(steps), searches=int(s.value), games=int(g.value), elapsed=float(t.value))


# ---- DOG: random legal play (oracle/cpu_dog.cpp) -----------------------------------------------------------
class Dog(ctypes.Structure):
    _fields_ = [("board", ctypes.c_int8 * 56), ("deck", ctypes.c_int8 * 14), ("hands", ctypes.c_int8 * 56),
                ("swap_choices", ctypes.c_int8 * 4), ("pins", ctypes.c_int32 * 16), ("start", ctypes.c_int32 * 4),
                ("target", ctypes.c_int32 * 4), ("goal", ctypes.c_int32 * 16)] + \
               [(n, ctypes.c_int32) for n in ("current_player", "reward", "done", "num_players", "round_starter", "phase",
                                              "hand_size", "num_cards", "board_size", "total", "rules", "deal", "game")] + \
               [("seed", ctypes.c_uint64)]


_dog_bound = False


def _dog_lib():
    global _dog_bound
    L = load()
    if not _dog_bound:
        vp, ip, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
        L.muzcpu_dog_reset.argtypes = [vp, ip, ip, u64, ip]
        L.muzcpu_dog_valid_actions.argtypes = [vp, vp]
        L.muzcpu_dog_step.argtypes = [vp, ip, vp, vp]
        L.muzcpu_dog_no_step.argtypes = [vp]
        L.muzcpu_dog_step_kind.argtypes = [vp, ip, ip, ip, vp, vp, vp]
        L.muzcpu_dog_play.restype = ctypes.c_int64
        L.muzcpu_dog_play.argtypes = [ip, ip, ip, ip, u64, vp]
        L.muzcpu_dog_bench.restype = ctypes.c_int64
        L.muzcpu_dog_bench.argtypes = [ip, ip, ip, u64, ip, ctypes.c_double, vp, vp]
        fp = ctypes.c_float
        L.muzcpu_dog_encode.argtypes = [vp, vp]
        L.muzcpu_dog_recurrent.argtypes = [vp, vp, vp, ip, vp, vp, vp, vp, vp]
        L.muzcpu_dog_search.argtypes = [vp, ip, ip, ip, vp, vp, vp, vp, vp, vp, vp, vp]
        L.muzcpu_dog_mz_play.restype = ctypes.c_int64
        L.muzcpu_dog_mz_play.argtypes = [vp, ip, ip, ip, ip, ip, fp, u64, vp]
        L.muzcpu_dog_mz_bench.restype = ctypes.c_int64
        L.muzcpu_dog_mz_bench.argtypes = [vp, ip, ip, ip, ip, fp, u64, ip, ctypes.c_double, vp, vp, vp]
        _dog_bound = True
    return L


def dog_rule_bits(**rules) -> int:
    from oracle import dog as dg
    r = dict(dg.DEFAULT_RULES)
    r.update(rules)
    if r["disable_swapping"] or r["disable_hot_seven"] or r["disable_joker"]:
        raise ValueError("the C++ DOG restatement plays the full 14-card deck (the reference's DOG configs)")
    return sum(bit for k, bit in _FLAGS.items() if k in r and r[k])


def dog_from_oracle(e, seed=0, game=0) -> Dog:
    """oracle/dog.State -> the C++ state struct (seed / game select the engine's deal keys)."""
    d = Dog()
    P = e.num_players
    d.board[:] = [int(x) for x in e.board]
    d.deck[:] = [int(x) for x in e.deck]
    h = np.zeros((4, 14), np.int8)
    h[:P] = e.hands
    d.hands[:] = [int(x) for x in h.ravel()]
    d.swap_choices[:] = [int(x) for x in e.swap_choices]
    pins = -np.ones(16, np.int32)
    pins[:P * 4] = np.asarray(e.pins).ravel()
    d.pins[:] = [int(x) for x in pins]
    st, tg, gl = np.zeros(4, np.int32), np.zeros(4, np.int32), np.zeros(16, np.int32)
    st[:P], tg[:P], gl[:P * 4] = e.start, e.target, np.asarray(e.goal).ravel()
    d.start[:], d.target[:], d.goal[:] = [int(x) for x in st], [int(x) for x in tg], [int(x) for x in gl]
    for k in ("current_player", "reward", "round_starter", "phase", "hand_size", "num_cards", "deal"):
        setattr(d, k, int(getattr(e, k)))
    d.done, d.num_players, d.board_size, d.total = int(e.done), P, e.board_size, e.total_board_size
    d.rules, d.game, d.seed = dog_rule_bits(**e.rules), int(game), int(seed)
    return d


def dog_valid_actions(d: Dog) -> np.ndarray:
    out = np.zeros(806, np.uint8)
    _dog_lib().muzcpu_dog_valid_actions(ctypes.byref(d), _p(out))
    return out.astype(bool)


def dog_step(d: Dog, action):
    r, dn = ctypes.c_int(), ctypes.c_int()
    _dog_lib().muzcpu_dog_step(ctypes.byref(d), int(action), ctypes.byref(r), ctypes.byref(dn))
    return r.value, bool(dn.value)


def dog_no_step(d: Dog):
    _dog_lib().muzcpu_dog_no_step(ctypes.byref(d))


def dog_step_kind(d: Dog, kind: str, case: dict):
    """One DOG/test.py step_* call: kind normal_move / neg_move / swap_move / hot7_move -> (pins, reward, done)."""
    k = {"normal_move": 0, "neg_move": 1, "swap_move": 2, "hot7_move": 3}[kind]
    dist = np.ascontiguousarray(case.get("dist", [0, 0, 0, 0]), np.int32)
    a = case.get("pin", 0)
    b = case.get("pos", case.get("move", 0))
    r, dn = ctypes.c_int(), ctypes.c_int()
    _dog_lib().muzcpu_dog_step_kind(ctypes.byref(d), k, int(a), int(b), _p(dist), ctypes.byref(r), ctypes.byref(dn))
    return np.array(d.pins[:d.num_players * 4], np.int32).reshape(d.num_players, 4), r.value, bool(dn.value)


def dog_play(P, rules, n, turns, seed):
    """bench.py's DOG CPU loop on one thread: (actions [turns, n], env-steps)."""
    acts = np.zeros((turns, n), np.int32)
    steps = _dog_lib().muzcpu_dog_play(P, dog_rule_bits(**rules), n, turns, seed, _p(acts))
    return acts, int(steps)


def dog_encode(d: Dog) -> np.ndarray:
    """The DOG MuZero slice's observation [34, 56] (oracle/dog_muzero.encode_board)."""
    out = np.zeros((34, 56), np.float32)
    _dog_lib().muzcpu_dog_encode(ctypes.byref(d), _p(out))
    return out


def dog_bench(P, rules, lanes, seed, threads, seconds):
    g, t = ctypes.c_int64(), ctypes.c_double()
    steps = _dog_lib().muzcpu_dog_bench(P, dog_rule_bits(**rules), lanes, seed, threads, seconds, ctypes.byref(g),
                                        ctypes.byref(t))
    return dict(env_steps=int(steps), games=int(g.value), elapsed=float(t.value))
