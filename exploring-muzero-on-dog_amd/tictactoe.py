"""TicTacToe (config (a): CPU plumbing) -- host mirror of TicTacToe/TicTacToeV2.py, TicTacToe/mcts.py
and the TicTacToe/eval.py match protocol, over libmuz.so's host C ABI (csrc/tictactoe.cpp).

  env_reset / env_step / valid_action_mask / policy_function / value_function   TicTacToeV2.py:37-123
  run_mcts (mctx.muzero_policy, S = 25, max_depth 9, qtransform_by_min_max(-1, 1))  mcts.py:9-23
  get_mcts_action / get_random_action / match / evaluate                         eval.py:28-55, 97-125, 178-227
  SimplePolicy / LargerNN / ImprovedTicTacToeNet + get_trained_action            train.py:11-50, eval.py:44-49
  (loaded from the reference's flax .params checkpoints by checkpoint.load_flax_msgpack)

jax PRNG keys become integer seeds (counter streams, include/muz.h TicTacToe section).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import lib as _L


class TicTacToeV2:
    """The reference's pytree as a mutable host struct (muz_ttt_state)."""

    def __init__(self, raw: _L.MuzTttState | None = None):
        self.raw = raw if raw is not None else _L.MuzTttState()

    @property
    def board(self) -> np.ndarray:
        return np.array(list(self.raw.board), np.int8).reshape(3, 3)

    @property
    def current_player(self) -> int:
        return int(self.raw.current_player)

    @property
    def reward(self) -> int:
        return int(self.raw.reward)

    @property
    def done(self) -> bool:
        return bool(self.raw.done)

    @property
    def memory(self) -> np.ndarray:
        return np.array(list(self.raw.memory), np.int8).reshape(2, 3)

    def copy(self) -> "TicTacToeV2":
        r = _L.MuzTttState()
        ctypes.memmove(ctypes.byref(r), ctypes.byref(self.raw), ctypes.sizeof(r))
        return TicTacToeV2(r)


def _call(name, *args):
    _L.check(getattr(_L.load(), name)(*args), name)


def env_reset(_=None) -> TicTacToeV2:
    env = TicTacToeV2()
    _call("muz_ttt_reset", ctypes.byref(env.raw))
    return env


def env_step(env: TicTacToeV2, action: int):
    """-> (new env, reward, done); the input env is not modified (functional, like the reference)."""
    out = env.copy()
    r, d = ctypes.c_int8(), ctypes.c_uint8()
    _call("muz_ttt_step", ctypes.byref(out.raw), int(action), ctypes.byref(r), ctypes.byref(d))
    return out, int(r.value), bool(d.value)


def valid_action_mask(env: TicTacToeV2) -> np.ndarray:
    return np.zeros((3, 3), bool) if env.done else env.board == 0


def policy_function(env: TicTacToeV2) -> np.ndarray:
    out = (ctypes.c_double * 9)()
    _call("muz_ttt_policy_logits", ctypes.byref(env.raw), out)
    return np.array(list(out))


def value_function(env: TicTacToeV2, seed: int, eval_id: int = 0) -> float:
    v = ctypes.c_double()
    _call("muz_ttt_rollout", ctypes.byref(env.raw), int(seed) & 0xFFFFFFFFFFFFFFFF, int(eval_id) & 0xFFFFFFFF,
          ctypes.byref(v))
    return float(v.value)


def run_mcts(seed: int, env: TicTacToeV2, num_simulations: int = 25, max_depth: int = 9, temperature: float = 1.0,
             turn: int = 0) -> dict:
    """mcts.py:run_mcts -> {action, action_weights [9], value, visit_counts [9]}."""
    o = _L.MuzTttPolicyOut()
    _call("muz_ttt_muzero_policy", ctypes.byref(env.raw), int(num_simulations), int(max_depth), float(temperature),
          int(seed) & 0xFFFFFFFFFFFFFFFF, int(turn), ctypes.byref(o))
    return {"action": int(o.action), "action_weights": np.array(list(o.action_weights)), "value": float(o.value),
            "visit_counts": np.array(list(o.visits), np.int32)}


def match(mcts_player: int, num_simulations: int, seed: int, game: int, limit: int = 30) -> int:
    """One eval.py game: MCTS player vs uniform random player -> winner * mcts_player (0 at the limit)."""
    r = ctypes.c_int32()
    _call("muz_ttt_match", int(mcts_player), int(num_simulations), int(seed) & 0xFFFFFFFFFFFFFFFF, int(game),
          int(limit), ctypes.byref(r))
    return int(r.value)


def evaluate(num_matches: int = 1000, num_simulations: int = 5, seed: int = 1) -> dict:
    """eval.py:178-227: half the games as player 1, half as player -1 -> win / loss / draw rates."""
    res = [match(1 if g < num_matches // 2 else -1, num_simulations, seed, g) for g in range(num_matches)]
    n = float(len(res))
    return {"win": res.count(1) / n, "loss": res.count(-1) / n, "draw": res.count(0) / n}


class PolicyNet:
    """The Dense policy networks of TicTacToe/train.py (SimplePolicy, LargerNN, ImprovedTicTacToeNet):
    board.flatten() (float) -> [Dense -> relu]* -> Dense(9).  ``tree`` = the flax state dict."""

    def __init__(self, tree: dict):
        p = tree.get("params", tree)
        names = sorted((k for k in p if k.startswith("Dense_")), key=lambda k: int(k.split("_")[1]))
        if len(names) != len(p):
            raise NotImplementedError("only the Dense policy networks are supported (not ConvTicTacToeNet)")
        self.layers = [(np.asarray(p[k]["kernel"], np.float32), np.asarray(p[k]["bias"], np.float32))
                       for k in names]

    def logits(self, board) -> np.ndarray:
        x = np.asarray(board, np.float32).reshape(-1)
        for i, (w, b) in enumerate(self.layers):
            x = (x @ w + b).astype(np.float32)
            if i + 1 < len(self.layers):
                x = np.maximum(x, np.float32(0.0))
        return x


def trained_action(net: PolicyNet, env: TicTacToeV2) -> int:
    """eval.py:44-49 get_trained_action: argmax of the logits over empty cells."""
    lg = net.logits(env.board)
    return int(np.argmax(np.where(env.board.reshape(-1) == 0, lg, -np.inf)))


def trained_match(net: PolicyNet, trained_player: int, rng: np.random.Generator, limit: int = 30) -> int:
    """eval.py:97-125 play_match with num_simulations = 0: trained player vs uniform random player."""
    env = env_reset()
    ply = 0
    while not env.done and ply < limit:
        if env.current_player == trained_player:
            a = trained_action(net, env)
        else:
            a = int(rng.choice(np.flatnonzero(env.board.reshape(-1) == 0)))
        env, _, _ = env_step(env, a)
        ply += 1
    if ply == limit:
        return 0
    b = env.board
    lines = [b[0], b[1], b[2], b[:, 0], b[:, 1], b[:, 2], b.diagonal(), np.fliplr(b).diagonal()]
    sums = [int(l.sum()) for l in lines]
    w = -1 if -3 in sums else (1 if 3 in sums else 0)
    return w * trained_player


def evaluate_trained(net: PolicyNet, num_matches: int = 1000, seed: int = 1) -> dict:
    """eval.py:178-227 evaluate_agent (num_simulations = 0): half the games as player 1, half as -1."""
    rng = np.random.default_rng(seed)
    half = num_matches // 2
    first = [trained_match(net, 1, rng) for _ in range(half)]
    second = [trained_match(net, -1, rng) for _ in range(half)]
    res = first + second
    n = float(len(res))
    return {"win": res.count(1) / n, "loss": res.count(-1) / n, "draw": res.count(0) / n,
            "wins_as_first": first.count(1), "wins_as_second": second.count(1), "games_per_seat": half}
