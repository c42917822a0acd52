"""CPU oracle: classic MADN environment (TEST INFRASTRUCTURE ONLY).

Plain NumPy restatement of the reference environment ``MADN/classic_madn.py`` (+ the helpers it uses
from ``utils/utility_funcs.py``).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it; nothing in the product path imports it.

Parity status: PINNED for transitions by the reference's own 64 golden step vectors
(``MADN/test.py:7-460`` -> ``tests/golden/classic_madn_step_cases.json``).  The die draw
(``throw_die``: jax threefry + ``jax.random.choice``) is restated from an explicit uniform number, so
the random SOURCE is unpinned; the mapping uniform -> die follows ``jax.random.choice`` with ``p``
(cumsum, ``r = cum[-1] * (1 - u)``, ``searchsorted`` left).

Differences from the deterministic variant that matter ("Classic differences"):
  * the move is ``env.die``, the action is a pin index (4 actions), there is no action set;
  * home -> start needs die in {1, 6} (start_on_1) or {6}, and ``~pins_on_start[cp_sub]`` where
    ``pins_on_start[i] = board[start[i]] == i`` (the SUBSTITUTED player, classic_madn.py:455-459);
  * ``no_step`` only advances the player;
  * ``encode_board`` ends with a die channel: C = 2P + 3.
All arithmetic is int8 in the reference (pins + die); values stay in range, so Python ints are exact.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .detmadn import (NUM_PINS, State as _DetState, _g, check_goal_path_for_pin, get_winner, is_player_done,
                      set_pins_on_board)

# classic_madn.py:12-18
NORMAL_DICE_DISTRIBUTION = np.array([1 / 6] * 6, np.float32)
OUT_ON_SIX_DICE_DISTRIBUTION = np.array([25 / 216] * 5 + [91 / 216], np.float32)
OUT_ON_ONE_DICE_DISTRIBUTION = np.array([91 / 216] + [25 / 216] * 5, np.float32)
OUT_ON_ONE_AND_SIX_DICE_DISTRIBUTION = np.array([76 / 216] + [16 / 216] * 4 + [76 / 216], np.float32)

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
    enable_dice_rethrow=True,
    must_traverse_start=False,
)


@dataclass
class State(_DetState):
    """``classic_MADN`` pytree (classic_madn.py:33-49): the det fields plus ``die`` (``action_set`` unused)."""

    die: int = 0


def env_reset(num_players=4, layout=(True, True, True, True), distance=10, starting_player=0, seed=None,
              **rules) -> State:
    """classic_madn.py:51-131 (a random starting player from ``seed`` as oracle.detmadn.env_reset)."""
    from .detmadn import start_seat
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
    s = State(board=board, current_player=int(starting_player), pins=pins, reward=0, done=False,
              action_set=np.zeros((P, 6), np.int8), num_players=P, start=start, target=target, goal=goal,
              board_size=board_size, total_board_size=total, rules=r, die=0)
    return s


def _sub_player(env: State) -> int:
    """Team substitution (classic_madn.py:275 / 409)."""
    p = env.current_player
    if env.rules["enable_teams"] and is_player_done(env.num_players, env.board, env.goal, p):
        return (p + 2) % 4
    return p


def is_soft_locked(env: State) -> bool:
    """classic_madn.py:180-206 (uses the UNSUBSTITUTED current player)."""
    cp = env.current_player
    pins = env.pins[cp]
    goal_pos = env.goal[cp].astype(np.int64)
    not_home = len(pins) - int(np.count_nonzero(pins == -1))
    relevant = np.arange(4) >= (4 - not_home)
    occupied = env.board[goal_pos] == cp
    return bool(np.all(occupied | ~relevant)) if not_home > 0 else True


def dice_probabilities(env: State) -> np.ndarray:
    """classic_madn.py:208-228 -> float32[6]."""
    if is_soft_locked(env) and env.rules["enable_dice_rethrow"]:
        return OUT_ON_ONE_AND_SIX_DICE_DISTRIBUTION if env.rules["enable_start_on_1"] else OUT_ON_SIX_DICE_DISTRIBUTION
    return NORMAL_DICE_DISTRIBUTION


def choice_from_uniform(p: np.ndarray, u: float) -> int:
    """jax.random.choice(key, [1..6], p=p) with the uniform draw made explicit:
    cum = cumsum(p) (fp32, sequential); r = cum[-1] * (1 - u); index = searchsorted(cum, r, 'left')."""
    cum = np.cumsum(np.asarray(p, np.float32), dtype=np.float32)
    r = np.float32(cum[-1] * np.float32(np.float32(1.0) - np.float32(u)))
    return int(np.searchsorted(cum, r, side="left")) + 1


def throw_die(env: State, u: float) -> State:
    """classic_madn.py:230-242 with an explicit uniform number (the threefry source is unpinned)."""
    return set_die(env, choice_from_uniform(dice_probabilities(env), u))


def set_die(env: State, die: int) -> State:
    """classic_madn.py:244-255."""
    s = env.replace()
    s.die = int(np.int8(die))
    return s


def valid_action(env: State) -> np.ndarray:
    """classic_madn.py:367-461 -> bool[4]."""
    R = env.rules
    cp = _sub_player(env)
    board = env.board
    cur = env.pins[cp].astype(np.int64)
    target = int(env.target[cp])
    goal = env.goal[cp].astype(np.int64)
    start = env.start.astype(np.int64)
    die = int(env.die)
    P = start.shape[0]
    pins_on_start = board[start] == np.arange(P)
    moved = cur + die
    fitted = moved % env.board_size
    x = moved - target - int(R["must_traverse_start"])
    res = (board[fitted] != cp) | R["enable_friendly_fire"]
    distance = env.board_size // 4
    nsb = ((cur // distance) + 1) % P
    nsa = fitted // distance
    trav = _g(start, nsb) == _g(start, nsa)
    res = np.where(R["enable_start_blocking"] & trav, (~_g(pins_on_start, nsa) | (cur == start[cp])) & res, res)
    x = np.where(R["must_traverse_start"] & R["enable_start_blocking"] & trav & _g(pins_on_start, nsa), 0, x)
    if not R["enable_circular_board"]:
        res = np.where((cur <= target) & ((x > 4) | ((x == 0) & R["must_traverse_start"])), False, res)
    A = R["enable_circular_board"] & res
    B = board[_g(goal, x - 1)] != cp
    C = np.array([R["enable_jump_in_goal_area"] or check_goal_path_for_pin(-1, int(x[i]), goal, board, cp)
                  for i in range(4)])
    res = np.where((4 >= x) & (x > 0) & (cur <= target), A | (B & C), res)
    D = np.array([R["enable_jump_in_goal_area"] or check_goal_path_for_pin(int(cur[i] - goal[0]), int(moved[i] - goal[0] + 1),
                                                                         goal, board, cp) for i in range(4)])
    in_goal = np.isin(cur, goal)
    res = np.where(in_goal, (moved <= goal[-1]) & (_g(board, moved) != cp) & D, res)
    start_moves = (1, 6) if R["enable_start_on_1"] else (-1, 6)
    from_home = (die in start_moves) and not bool(pins_on_start[cp])
    res = np.where(cur == -1, from_home, res)
    return res.astype(bool)


def env_step(env: State, pin: int):
    """classic_madn.py:257-337: move pin ``pin`` of the (substituted) current player by ``env.die``."""
    R = env.rules
    pin = int(np.int8(pin))
    move = int(np.int8(env.die))
    player_id = env.current_player
    cp = _sub_player(env)
    invalid = not bool(_g(valid_action(env), pin))
    pi = int(np.clip(pin + 4 if pin < 0 else pin, 0, 3))
    cur = int(env.pins[cp, pi])
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
    pins[cp, pi] = env.pins[cp, pi] if invalid else new_pos
    new_board = board if invalid else set_pins_on_board(-np.ones_like(board), pins)
    winner = get_winner(env, new_board)
    reward = 0 if env.done else (-1 if invalid else int(winner[cp]))
    done = bool(env.done or winner.any())
    if done or (R["enable_bonus_turn_on_6"] and move == 6):
        nxt = player_id
    else:
        nxt = (player_id + 1) % env.num_players
    env2 = env.replace(board=new_board, pins=pins, current_player=nxt, done=done, reward=reward)
    return env2, reward, done


def no_step(env: State):
    """classic_madn.py:353-365: advance the player only."""
    env2 = env.replace(current_player=(env.current_player + 1) % env.num_players)
    return env2, 0, env2.done


def encode_board(env: State) -> np.ndarray:
    """classic_madn.py:463-497 -> int[2P+3, total_board_size]."""
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
    die = np.full((1, W), int(env.die), np.int32)
    return np.concatenate([pc, team, opp, home, die], axis=0)


def num_channels(num_players: int) -> int:
    return 2 * num_players + 3
