"""CPU oracle: deterministic MADN environment (TEST INFRASTRUCTURE ONLY).

This module is a plain NumPy restatement of the reference environment
``MADN/deterministic_madn.py`` (+ the helpers it uses from
``utils/utility_funcs.py``).  It exists only so that ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg can check /
time the HIP implementation.  Nothing in the product path imports it.

Parity status: PINNED for transitions by the reference's own 64 golden step
vectors (``MADN/test.py:478-931`` -> ``tests/golden/detmadn_step_cases.json``).

JAX semantics reproduced on purpose:
  * gathers normalise a negative index ONCE (i<0 -> i+n) and then CLAMP into
    [0, n-1]  (``_g``);
  * ``//`` and ``%`` are floor division / Python modulo;
  * ``valid_action`` promotes int8 pins to int32 through ``jnp.arange(1, 7)``;
  * team substitution asymmetries (``board[start[cp_sub]] != current_player``,
    refill of the *unsubstituted* row from the *pre-step* action set).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

NUM_PINS = 4
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


def _g(arr, idx):
    """JAX gather semantics for one axis: normalise negatives once, then clamp."""
    n = arr.shape[0]
    idx = np.asarray(idx, dtype=np.int64)
    idx = np.where(idx < 0, idx + n, idx)
    idx = np.clip(idx, 0, n - 1)
    return arr[idx]


@dataclass
class State:
    """``deterministic_MADN`` pytree (deterministic_madn.py:24-40)."""

    board: np.ndarray            # int8[total_board_size], -1 empty else player id
    current_player: int          # int8 scalar
    pins: np.ndarray             # int8[P, 4]  (-1 home, 0..board_size-1 track, goal >= board_size)
    reward: int
    done: bool
    action_set: np.ndarray       # int8[P, 6]  remaining copies of moves 1..6
    num_players: int
    start: np.ndarray            # int8[P]
    target: np.ndarray           # int8[P]
    goal: np.ndarray             # int8[P, 4]
    board_size: int
    total_board_size: int
    rules: dict = field(default_factory=dict)

    def replace(self, **kw):
        s = copy.copy(self)
        for k, v in kw.items():
            setattr(s, k, v)
        return s


def set_pins_on_board(board, pins):
    """deterministic_madn.py:259-271 (scatter with mode='drop' for -1)."""
    out = np.full_like(board, -1, dtype=np.int8)
    P = pins.shape[0]
    for p in range(P):
        for k in range(pins.shape[1]):
            pos = int(pins[p, k])
            if 0 <= pos < out.shape[0]:
                out[pos] = p
    return out


_M64 = 0xFFFFFFFFFFFFFFFF
START_STREAM = 0x57A27C0DE5


def _mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def start_seat(key: int, P: int) -> int:
    """The engine's random starting player (csrc/rng.hpp start_seat): floor(U * P) in float32 of the counter RNG of
    ``key`` (det / classic: the game's reset seed as uint32; DOG: the deal key).  The reference draws the seat with
    jax.random.randint(split(PRNGKey(seed))[1], (), 0, P) (deterministic_madn.py:60-62); threefry is not restated,
    so parity of WHICH seat a seed gives is unpinned, only the uniform distribution over seats is shared."""
    u = np.float32((_mix64((key ^ START_STREAM) & _M64) >> 40) * (1.0 / 16777216.0))
    s = int(np.float32(u) * np.float32(P))
    return min(s, P - 1)


def env_reset(num_players=4, layout=(True, True, True, True), distance=10, starting_player=0, seed=None,
              **rules) -> State:
    """deterministic_madn.py:42-120.

    ``starting_player`` out of range: a random seat drawn from ``seed`` (line 62) with the engine's counter RNG
    (``start_seat``; jax threefry is not restated, parity of the seat unpinned)."""
    r = dict(DEFAULT_RULES)
    r.update(rules)
    P = int(num_players)
    if not (0 <= starting_player < P):
        if seed is None:
            raise ValueError("a random starting player needs the reset seed")
        starting_player = start_seat(int(seed) & 0xFFFFFFFF, P)
    board_size = 4 * int(distance)
    total = board_size + 16
    r["enable_teams"] = bool(r["enable_teams"] and P == 4)
    layout = np.asarray(layout, dtype=bool)
    if layout.sum() != P or (layout.all() and P < 4):
        layout = np.zeros(4, dtype=bool)
        layout[:P] = True
    start = (np.arange(4) * distance).astype(np.int8)[layout]
    target = ((start.astype(np.int64) - 1) % board_size).astype(np.int8)
    goal = np.arange(board_size, board_size + 16, dtype=np.int8).reshape(4, 4)[layout, :]
    pins = -np.ones((P, NUM_PINS), dtype=np.int8)
    if r["enable_initial_free_pin"]:
        pins[:, 0] = start
    board = -np.ones(total, dtype=np.int8)
    if r["enable_initial_free_pin"]:
        board = set_pins_on_board(board, pins)
    return State(board=board, current_player=int(starting_player), pins=pins, reward=0, done=False,
                 action_set=NUM_PINS * np.ones((P, 6), dtype=np.int8), num_players=P, start=start,
                 target=target, goal=goal, board_size=board_size, total_board_size=total, rules=r)


def is_player_done(num_players, board, goal, player) -> bool:
    """deterministic_madn.py:122-137."""
    if player >= num_players:
        return False
    return bool(np.all(board[goal[player].astype(np.int64)] >= 0))


def get_winner(env: State, board) -> np.ndarray:
    """deterministic_madn.py:139-168 -> bool[4]."""
    done = np.array([is_player_done(env.num_players, board, env.goal, p) for p in range(4)])
    if not env.rules["enable_teams"]:
        return done
    t0 = done[0] & done[2]
    t1 = done[1] & done[3]
    if (t0 & t1) or not (t0 | t1):
        return np.zeros(4, dtype=bool)
    return np.array([True, False, True, False]) if t0 else np.array([False, True, False, True])


def _sub_player(env: State) -> int:
    """Team substitution (deterministic_madn.py:184 / :310)."""
    p = env.current_player
    if env.rules["enable_teams"] and is_player_done(env.num_players, env.board, env.goal, p):
        return (p + 2) % 4
    return p


def check_goal_path_for_pin2(start, x_val, goal, board, cp):
    """utils/utility_funcs.py:142-163 (vectorised over leading dim)."""
    ga = np.arange(len(goal))[None, :]
    occ = (board[goal[ga].astype(np.int64)] != cp)
    sel = (np.asarray(start)[:, None] < ga) & (ga < np.asarray(x_val)[:, None])
    return np.all(np.where(sel, occ, True), axis=1)


def check_goal_path_for_pin(start, x_val, goal, board, cp) -> bool:
    """utils/utility_funcs.py:165-184."""
    ga = np.arange(len(goal))
    return bool(np.all(np.where((np.asarray(start) < ga) & (ga < x_val), board[goal.astype(np.int64)] != cp, True)))


def valid_action(env: State) -> np.ndarray:
    """deterministic_madn.py:299-393 -> bool[4, 6]."""
    R = env.rules
    cp0 = env.current_player
    cp = _sub_player(env)
    board = env.board
    cur_pins = env.pins[cp].astype(np.int64)          # (4,)
    target = int(env.target[cp])
    goal = env.goal[cp].astype(np.int64)
    aset = env.action_set[cp]
    avail = aset > 0
    start = env.start.astype(np.int64)
    P = start.shape[0]
    pins_on_start = board[start] == np.arange(P)
    cur = cur_pins[:, None]
    moved = cur + np.arange(1, 7)[None, :]            # int32 promotion
    fitted = moved % env.board_size
    x = moved - target - int(R["must_traverse_start"])
    res = (board[fitted] != cp) | R["enable_friendly_fire"]
    distance = env.board_size // 4
    nsb = ((cur // distance) + 1) % P
    nsa = fitted // distance
    trav = _g(start, nsb) == _g(start, nsa)
    res = np.where(R["enable_start_blocking"] & trav,
                   (~_g(pins_on_start, nsa) | (cur_pins == start[cp])[:, None]) & res, res)
    x = np.where(R["must_traverse_start"] & R["enable_start_blocking"] & trav & _g(pins_on_start, nsa), 0, x)
    if not R["enable_circular_board"]:
        res = np.where((cur <= target) & ((x > 4) | ((x == 0) & R["must_traverse_start"])), False, res)
    A = R["enable_circular_board"] & res
    B = board[_g(goal, x - 1)] != cp
    C = np.stack([R["enable_jump_in_goal_area"] | check_goal_path_for_pin2(-np.ones(6, np.int64), x[i], goal, board, cp)
                  for i in range(4)])
    res = np.where((4 >= x) & (x > 0) & (cur <= target), A | (B & C), res)
    D = np.stack([R["enable_jump_in_goal_area"] | check_goal_path_for_pin2(
        np.ones(6, np.int64) * (cur_pins[i] - goal[0]), moved[i] - goal[0] + 1, goal, board, cp) for i in range(4)])
    in_goal = np.isin(cur, goal)
    res = np.where(in_goal, (moved <= goal[-1]) & (_g(board, moved) != cp) & D, res)
    start_moves = np.array([1, 6]) if R["enable_start_on_1"] else np.array([-1, 6])
    from_home = np.isin(np.arange(1, 7), start_moves) & (board[start[cp]] != cp0)
    res = np.where((cur_pins == -1)[:, None], from_home[None, :], res)
    return res & avail[None, :]


def env_step(env: State, action):
    """deterministic_madn.py:170-257.  ``action`` = (pin, move) with move in 1..6."""
    R = env.rules
    pin = int(np.int8(action[0]))
    move = int(np.int8(action[1]))
    player_id = env.current_player
    cp = _sub_player(env)
    va = valid_action(env)
    invalid = not bool(va[pin, (move - 1) % 6 if move - 1 < 0 else move - 1])
    cur = int(env.pins[cp, pin])
    moved = cur + move
    fitted = moved % env.board_size
    x = moved - int(env.target[cp]) - int(R["must_traverse_start"])
    goal = env.goal[cp].astype(np.int64)
    board = env.board
    in_goal = cur in goal.tolist()
    if in_goal:
        a = check_goal_path_for_pin(cur - goal[0], moved - goal[0] + 1, goal, board, cp)
    else:
        a = check_goal_path_for_pin(-np.ones(4, np.int64), x, goal, board, cp)
    A = (int(board[int(_g(goal, x - 1))]) != cp) and (R["enable_jump_in_goal_area"] or a)
    if cur == -1:
        new_pos = int(env.start[cp])
    elif in_goal:
        new_pos = moved
    elif (4 >= x > 0) and A and (cur <= int(env.target[cp])):
        new_pos = int(_g(goal, x - 1))
    else:
        new_pos = fitted
    pin_at_pos = int(_g(board, new_pos))
    pins = env.pins.copy()
    if pin_at_pos != -1 and (pin_at_pos != cp or R["enable_friendly_fire"]) and not invalid:
        row = pins[pin_at_pos]
        pins[pin_at_pos] = np.where(row == new_pos, -1, row)
    pins[cp, pin] = env.pins[cp, pin] if invalid else new_pos
    new_board = board if invalid else set_pins_on_board(-np.ones_like(board), pins)
    mi = (move - 1) if (move - 1) >= 0 else (move - 1) + 6
    curr_state = int(env.action_set[cp, mi])
    action_set = env.action_set.copy()
    action_set[cp, mi] = curr_state if (invalid or curr_state == 0) else curr_state - 1
    if np.all(action_set[cp] == 0):
        action_set = env.action_set.copy()
        action_set[env.current_player] = NUM_PINS
    winner = get_winner(env, new_board)
    reward = 0 if env.done else (-1 if invalid else int(winner[cp]))
    done = bool(env.done or winner.any())
    if done or (R["enable_bonus_turn_on_6"] and move == 6):
        nxt = player_id
    else:
        nxt = (player_id + 1) % env.num_players
    env2 = env.replace(board=new_board, pins=pins, current_player=nxt, done=done, reward=reward,
                       action_set=action_set)
    return env2, reward, done


def no_step(env: State):
    """deterministic_madn.py:283-297."""
    aset = env.action_set.copy()
    aset[env.current_player] = NUM_PINS
    env2 = env.replace(action_set=aset, current_player=(env.current_player + 1) % env.num_players)
    return env2, 0, env2.done


def encode_board(env: State) -> np.ndarray:
    """deterministic_madn.py:395-438 -> int[8P+2, total_board_size]."""
    P = env.num_players
    distance = env.board_size // 4
    cp = env.current_player
    rolled = (np.arange(P) + cp) % P
    track = np.roll(env.board[:env.board_size], -distance * cp)
    goals = np.roll(env.board[env.board_size:env.total_board_size], -4 * cp)
    b = np.concatenate([track, goals])
    pc = (b[None, :] == rolled[:, None]).astype(np.int32)
    if env.rules["enable_teams"]:
        team = pc[::2].sum(0, keepdims=True)
        opp = pc[1::2].sum(0, keepdims=True)
    else:
        team = pc[0:1].sum(0, keepdims=True)
        opp = pc[1:].sum(0, keepdims=True)
    W = b.shape[0]
    home = np.count_nonzero(env.pins == -1, axis=1)[rolled][:, None] * np.ones((1, W), np.int32)
    act = np.repeat(env.action_set.astype(np.int32)[:, :, None], W, axis=2)[rolled].reshape(-1, W)
    return np.concatenate([pc, team, opp, home, act], axis=0)


def map_action(idx: int):
    """deterministic_madn.py:469-479."""
    return idx // 6, idx % 6 + 1


def num_channels(num_players: int) -> int:
    return 8 * num_players + 2
