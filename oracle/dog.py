"""CPU oracle: the DOG environment (TEST INFRASTRUCTURE ONLY).

NumPy restatement of ``DOG/dog.py`` (+ ``utils/utility_funcs.py``: all_pin_distributions 4-21,
check_goal_path_for_pin 165-184, check_relative_order_preserved 186-234, get_path_matrix 237-303,
check_moving_pins_hit 310-319).  Only ``tests/`` may use it.

Parity status: PINNED for the four move kinds by the reference's own golden vectors
(``DOG/test.py``: test_normal_move 52 cases, test_neg_move 17, test_swap_move 14, test_7_move 29 ->
``tests/golden/dog_*_cases.json``).  The deck shuffle (``distribute_cards``: argsort of
``jax.random.uniform`` keys) is restated with the keys as an input; the key SOURCE is unpinned.

JAX semantics reproduced: gathers / scatters normalise a negative index once then clamp (``_g``,
``_s``), floor ``//`` and ``%``, team substitution through a finished player, the quirks of
valid_step_actions / env_step_play_phase using the substituted player's HAND, and no validity check in
the swap phase.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

NUM_PINS = 4
MAX_CARDS = 120
MAX_HAND = 6
NORMAL_MOVES = (1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13)


def all_pin_distributions(total=7):
    """utils/utility_funcs.py:4-21: (a0, a1, a2, a3 = total - a0 - a1 - a2 >= 0), lex order over (a0, a1, a2)."""
    out = []
    for a in range(total + 1):
        for b in range(total + 1):
            for c in range(total + 1):
                d = total - a - b - c
                if d >= 0:
                    out.append((a, b, c, d))
    return np.array(out, np.int32)


DISTS_7_4 = all_pin_distributions(7)          # (120, 4)

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

# MuZero_DOG/game_agent.py:12-23
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


def _g(arr, idx):
    """JAX gather along axis 0: normalise a negative index once, then clamp."""
    n = arr.shape[0]
    idx = np.asarray(idx, dtype=np.int64)
    idx = np.where(idx < 0, idx + n, idx)
    return arr[np.clip(idx, 0, n - 1)]


def _si(n, idx):
    """JAX scatter index (.at[i].set): normalise a negative index once; out of range is dropped (None)."""
    i = int(idx)
    i = i + n if i < 0 else i
    return i if 0 <= i < n else None


@dataclass
class State:
    """``DOG`` pytree (dog.py:31-56).  ``deal`` counts distribute_cards calls (it replaces jax's key)."""

    board: np.ndarray          # int8[56]
    current_player: int
    pins: np.ndarray           # int32[P, 4]
    reward: int
    done: bool
    deck: np.ndarray           # int8[num_cards]
    hands: np.ndarray          # int8[P, num_cards]
    num_players: int
    start: np.ndarray          # int32[P]
    target: np.ndarray         # int32[P]
    goal: np.ndarray           # int32[P, 4]
    swap_choices: np.ndarray   # int8[4]
    round_starter: int
    phase: int
    hand_size: int
    num_cards: int
    board_size: int
    total_board_size: int
    rules: dict = field(default_factory=dict)
    deal: int = 0

    def replace(self, **kw):
        s = copy.copy(self)
        for k, v in kw.items():
            setattr(s, k, v)
        return s


def play_action_size(env) -> int:
    """get_play_action_size (dog.py:58-59): 2 * (4 * (12 + 1 + 56) + 120) = 792."""
    return int(2 * (4 * (12 + 1 + env.total_board_size) + 120))


def set_pins_on_board(board, pins):
    out = np.full_like(board, -1, dtype=np.int8)
    for p in range(pins.shape[0]):
        for k in range(pins.shape[1]):
            pos = int(pins[p, k])
            if 0 <= pos < out.shape[0]:
                out[pos] = p
    return out


def env_reset(num_players=4, layout=(True, True, True, True), distance=10, starting_player=0, shuffle_keys=None,
              start_key=None, **rules) -> State:
    """dog.py:83-186.  ``shuffle_keys(env)`` -> float keys [120] for each distribute_cards call (default:
    the deal-count-seeded numpy generator of ``default_shuffle_keys``)."""
    r = dict(DEFAULT_RULES)
    r.update(rules)
    P = int(num_players)
    if not (0 <= starting_player < P):   # dog.py:102-104: a random seat, here from the engine's key (start_seat)
        if start_key is None:
            raise ValueError("a random starting player needs the reset's key (engine_start_key)")
        from .detmadn import start_seat
        starting_player = start_seat(int(start_key), P)
    board_size = 4 * int(distance)
    total = board_size + 16
    r["enable_teams"] = bool(r["enable_teams"] and P == 4)
    layout = np.asarray(layout, dtype=bool)
    if layout.sum() != P or (layout.all() and P < 4):
        layout = np.zeros(4, dtype=bool)
        layout[:P] = True
    start = (np.arange(4) * distance).astype(np.int32)[layout]
    target = (start - 1) % board_size
    goal = np.arange(board_size, board_size + 16, dtype=np.int32).reshape(4, 4)[layout, :]
    pins = -np.ones((P, NUM_PINS), np.int32)
    if r["enable_initial_free_pin"]:
        pins[:, 0] = start
    board = -np.ones(total, np.int8)
    if r["enable_initial_free_pin"]:
        board = set_pins_on_board(board, pins)
    num_cards = 14 - int(r["disable_joker"]) - int(r["disable_hot_seven"]) - int(r["disable_swapping"])
    deck = np.full(num_cards, 8, np.int8)
    deck[0] = 6 + 2 * int(r["disable_joker"])
    env = State(board=board, current_player=int(starting_player), pins=pins, reward=0, done=False, deck=deck,
                hands=np.zeros((P, num_cards), np.int8), num_players=P, start=start, target=target, goal=goal,
                swap_choices=np.full(4, -1, np.int8), round_starter=-1, phase=0, hand_size=6, num_cards=num_cards,
                board_size=board_size, total_board_size=total, rules=r, deal=0)
    return distribute_cards(env, shuffle_keys)


def reset_deck(env):
    """dog.py:188-191 (row 0 = 6 + 2 * (disable_joker ? 0 : 1): the reference's own formula)."""
    deck = np.full(env.num_cards, 8, np.int8)
    deck[0] = 6 + 2 * (0 if env.rules["disable_joker"] else 1)
    return deck


def distribute_cards(env: State, shuffle_keys=None) -> State:
    """dog.py:201-298.  The 120 shuffle keys come from ``shuffle_keys(env)`` (jax uniform in the reference)."""
    P = env.hands.shape[0]
    nct = len(env.deck)
    q = int(env.hand_size)
    dummy = nct
    deck = env.deck.astype(np.int8)
    if int(deck.astype(np.int64).sum()) < q * P:
        deck = reset_deck(env)
    size = int(deck.astype(np.int64).sum())
    counts = np.concatenate([deck.astype(np.int64), [MAX_CARDS - size]])
    pool = np.repeat(np.arange(nct + 1), counts)[:MAX_CARDS]
    keys = np.asarray((shuffle_keys or default_shuffle_keys)(env), np.float32)
    prio = np.where(pool == dummy, np.float32(2.0), keys)
    order = np.argsort(prio, kind="stable")
    shuffled = pool[order]
    cards = np.full((P, MAX_HAND), dummy, np.int64)
    for p in range(P):
        for s in range(MAX_HAND):
            if s < q:
                cards[p, s] = shuffled[p * q + s]
    add = np.zeros((P, nct), np.int8)
    for p in range(P):
        for s in range(MAX_HAND):
            if cards[p, s] < nct:
                add[p, cards[p, s]] += 1
    hands = (env.hands + add).astype(np.int8)
    deck = (deck - add.sum(0)).astype(np.int8)
    swap_phase = env.rules["enable_teams"] and P == 4
    rs = env.current_player if env.round_starter == -1 else (env.round_starter + 1) % P
    return env.replace(current_player=rs, deck=deck, hands=hands, swap_choices=np.full(4, -1, np.int8),
                       round_starter=rs, phase=1 if swap_phase else 0, hand_size=6 if q == 2 else q - 1,
                       deal=env.deal + 1)


def default_shuffle_keys(env):
    return np.random.default_rng(1000 + env.deal).random(MAX_CARDS, dtype=np.float32)


M64 = 0xFFFFFFFFFFFFFFFF
DEAL_STREAM = 0xDEA1C0DE5EED
RANDOM_ACTION_STREAM = 0x52A4D0DA11


def _mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def _u24(h):
    return np.float32((h >> 40) * (1.0 / 16777216.0))


def _game_key(seed, g, turn):
    return (seed & M64) ^ _mix64(((g & 0xFFFFFFFF) << 32) | (turn & 0xFFFFFFFF))


def engine_shuffle_keys(seed, game):
    """The device engine's deal keys (csrc/env_dog.hip:deal_key, include/muz.h DOG section) for game
    ``game`` of a batch reset with ``seed``: a ``shuffle_keys`` callback for env_reset / env_step."""
    def keys(env):
        base = _game_key(seed ^ DEAL_STREAM, game, env.deal)
        return np.array([_u24(_mix64(base ^ (((k + 1) * 0xA24BAED4963EE407) & M64))) for k in range(MAX_CARDS)],
                        np.float32)
    return keys


def engine_start_key(seed, game, deal=0):
    """The key of the device's random starting player for game ``game`` of a batch reset with ``seed`` (deal counter
    ``deal``: 0 for muz_dog_reset, the running count for an in-place restart): csrc/env_dog.hip dog_reset_lds."""
    return _game_key(seed, game, deal)


def engine_random_action(mask, seed, game, turn):
    """csrc/env_dog.hip:k_dog_random_action with the counter uniform: the k-th legal action."""
    legal = np.flatnonzero(np.asarray(mask, bool))
    if legal.size == 0:
        return -1
    u = _u24(_mix64(_game_key(seed ^ RANDOM_ACTION_STREAM, game, turn)))
    k = min(int(np.float32(u) * np.float32(legal.size)), legal.size - 1)
    return int(legal[k])


def is_player_done(num_players, board, goal, player) -> bool:
    if player >= num_players:
        return False
    return bool(np.all(board[goal[player].astype(np.int64)] >= 0))


def get_winner(env, board):
    done = np.array([is_player_done(env.num_players, board, env.goal, p) for p in range(4)])
    if not env.rules["enable_teams"]:
        return done
    t0, t1 = done[0] & done[2], done[1] & done[3]
    if (t0 & t1) or not (t0 | t1):
        return np.zeros(4, bool)
    return np.array([True, False, True, False]) if t0 else np.array([False, True, False, True])


def sub_player(env) -> int:
    p = env.current_player
    if env.rules["enable_teams"] and is_player_done(env.num_players, env.board, env.goal, p):
        return (p + 2) % 4
    return p


def check_goal_path_for_pin(start, x_val, goal, board, cp) -> bool:
    ga = np.arange(len(goal))
    return bool(np.all(np.where((start < ga) & (ga < x_val), board[goal.astype(np.int64)] != cp, True)))


def check_relative_order_preserved(old, new, board_size):
    old = np.asarray(old, np.int64)
    new = np.asarray(new, np.int64)
    outside = old < board_size
    ing = old >= board_size
    so = np.sign(old[:, None] - old[None, :])
    sn = np.sign(new[:, None] - new[None, :])
    pairs = ing[:, None] & ing[None, :]
    return outside | np.all(np.where(pairs, so == sn, True), axis=1)


# ------------------------------------------------------------------------------------ legality
def val_swap(env):
    """dog.py:361-391 -> bool[4, 56]."""
    R = env.rules
    cp = sub_player(env)
    pins = env.pins[cp].astype(np.int64)
    board = env.board
    N = board.shape[0]
    start = env.start.astype(np.int64)
    P = start.shape[0]
    m = np.tile(~np.isin(board, [-1, cp]), (4, 1))
    m[:, start] = (~((board[start] == np.arange(P)) & R["enable_start_blocking"]) & (board[start] != -1))[None, :]
    for p in pins:
        i = _si(N, p)
        if i is not None:
            m[:, i] = False
    for g in env.goal.reshape(-1):
        m[:, g] = False
    dis = np.concatenate([[-1], [start[cp]] if R["enable_start_blocking"] else [-1], env.goal[cp]])
    return m & (~np.isin(pins, dis))[:, None]


def _common(env, move_vec):
    cp = sub_player(env)
    cur = env.pins[cp].astype(np.int64)
    start = env.start.astype(np.int64)
    P = start.shape[0]
    pos = env.board[start] == np.arange(P)
    moved = cur + np.asarray(move_vec, np.int64)
    fitted = moved % env.board_size
    return cp, cur, start, P, pos, moved, fitted


def val_action_7(env, dist) -> bool:
    """dog.py:393-481 -> scalar bool for one hot-7 distribution."""
    R = env.rules
    cp, cur, start, P, pos, moved, fitted = _common(env, dist)
    board = env.board
    target = int(env.target[cp])
    goal = env.goal[cp].astype(np.int64)
    mt = int(R["must_traverse_start"])
    x = moved - target - mt
    pos = pos.copy()
    pos[cp] = bool(np.any(np.where(cur == start[cp], moved == start[cp], False)))
    if R["enable_circular_board"]:
        res = np.ones(4, bool)
    else:
        res = ~((cur <= target) & ((moved > target + 4) | ((x == 0) & bool(mt))))
    dist10 = env.board_size // 4
    nsb = ((cur // dist10) + 1) % P
    nsa = fitted // dist10
    trav = _g(start, nsb) == _g(start, nsa)
    res = np.where(R["enable_start_blocking"] & trav, ~_g(pos, nsa) & res, res)
    x = np.where(bool(mt) & R["enable_start_blocking"] & trav & _g(pos, nsa), 0, x)
    A = R["enable_circular_board"] & res
    tmp = env.pins.copy()
    tmp[cp] = np.where(np.isin(cur, goal), moved, cur)
    tb = set_pins_on_board(board, tmp)
    C = np.array([R["enable_jump_in_goal_area"] or check_goal_path_for_pin(-1, int(x[i]), goal, tb, cp) for i in range(4)])
    res = np.where((4 >= x) & (x > 0) & (cur <= target), A | C, res)
    D = R["enable_jump_in_goal_area"] | check_relative_order_preserved(cur, moved, env.board_size)
    res = np.where(np.isin(cur, goal), (moved <= goal[-1]) & D, res)
    mover = np.where(cur == -1, moved == -1, True)
    return bool(np.all(res & mover))


def val_action_7_all(env, dists=DISTS_7_4):
    """val_action_7 for every row of ``dists`` at once -> bool[n] (the same expressions, broadcast over the
    distributions; tests/test_dog_oracle.py checks it against the scalar form)."""
    R = env.rules
    cp, cur, start, P, pos, _, _ = _common(env, np.zeros(4, np.int64))
    D = np.asarray(dists, np.int64)
    n = D.shape[0]
    moved = cur[None, :] + D
    fitted = moved % env.board_size
    target = int(env.target[cp])
    goal = env.goal[cp].astype(np.int64)
    mt = int(R["must_traverse_start"])
    x = moved - target - mt
    posd = np.tile(pos, (n, 1))
    posd[:, cp] = np.any((cur == start[cp])[None, :] & (moved == start[cp]), axis=1)
    if R["enable_circular_board"]:
        res = np.ones((n, 4), bool)
    else:
        res = ~((cur[None, :] <= target) & ((moved > target + 4) | ((x == 0) & bool(mt))))
    dist10 = env.board_size // 4
    nsb = ((cur // dist10) + 1) % P
    nsa = fitted // dist10
    trav = _g(start, nsb)[None, :] == _g(start, nsa)
    pa = np.take_along_axis(posd, np.clip(np.where(nsa < 0, nsa + P, nsa), 0, P - 1), axis=1)
    res = np.where(R["enable_start_blocking"] & trav, ~pa & res, res)
    x = np.where(bool(mt) & R["enable_start_blocking"] & trav & pa, 0, x)
    A = R["enable_circular_board"] & res
    ing = np.isin(cur, goal)
    tmp = np.where(ing[None, :], moved, cur[None, :])                       # cp's pins on tmp_board
    occ = np.any(tmp[:, :, None] == goal[None, None, :], axis=1)             # (n, 4 goal cells)
    ga = np.arange(4)
    blocked = ((-1 < ga)[None, None, :] & (ga[None, None, :] < x[:, :, None])) & occ[:, None, :]
    C = R["enable_jump_in_goal_area"] | ~np.any(blocked, axis=2)
    res = np.where((4 >= x) & (x > 0) & (cur[None, :] <= target), A | C, res)
    so = np.sign(cur[:, None] - cur[None, :])
    sn = np.sign(moved[:, :, None] - moved[:, None, :])
    gin = cur >= env.board_size
    pairs = gin[:, None] & gin[None, :]
    Dd = R["enable_jump_in_goal_area"] | ((cur < env.board_size)[None, :] |
                                          np.all(np.where(pairs[None], so[None] == sn, True), axis=2))
    res = np.where(ing[None, :], (moved <= goal[-1]) & Dd, res)
    mover = np.where(cur[None, :] == -1, moved == -1, True)
    return np.all(res & mover, axis=1)


def val_action_normal_move(env, move):
    """dog.py:483-566 -> bool[4]."""
    R = env.rules
    cp, cur, start, P, pos, moved, fitted = _common(env, np.full(4, move))
    board = env.board
    target = int(env.target[cp])
    goal = env.goal[cp].astype(np.int64)
    mt = int(R["must_traverse_start"])
    x = moved - target - mt
    res = (board[fitted] != cp) | R["enable_friendly_fire"]
    dist10 = env.board_size // 4
    nsb = ((cur // dist10) + 1) % P
    nsa = fitted // dist10
    trav = _g(start, nsb) == _g(start, nsa)
    res = np.where(R["enable_start_blocking"] & trav, (~_g(pos, nsa) | (cur == start[cp])) & res, res)
    x = np.where(bool(mt) & R["enable_start_blocking"] & trav & _g(pos, nsa), 0, x)
    if not R["enable_circular_board"]:
        res = np.where((cur <= target) & ((x > 4) | ((x == 0) & bool(mt))), False, res)
    A = R["enable_circular_board"] & res
    B = board[_g(goal, x - 1)] != cp
    C = np.array([R["enable_jump_in_goal_area"] or check_goal_path_for_pin(-1, int(x[i]), goal, board, cp) for i in range(4)])
    res = np.where((4 >= x) & (x > 0) & (cur <= target), A | (B & C), res)
    D = np.array([R["enable_jump_in_goal_area"] or check_goal_path_for_pin(int(cur[i] - goal[0]), int(moved[i] - goal[0] + 1),
                                                                         goal, board, cp) for i in range(4)])
    res = np.where(np.isin(cur, goal), (moved <= goal[-1]) & (_g(board, moved) != cp) & D, res)
    res = np.where(cur == -1, (move in (1, 11, 13)) and not bool(pos[cp]), res)
    return res & (move > 0)


def val_neg_move(env, move):
    """dog.py:568-615 -> bool[4]."""
    R = env.rules
    cp, cur, start, P, pos, moved, fitted = _common(env, np.full(4, move))
    board = env.board
    goal = env.goal[cp].astype(np.int64)
    res = (board[fitted] != cp) | R["enable_friendly_fire"]
    dist10 = env.board_size // 4
    nsb = cur // dist10
    nsa = ((fitted // dist10) + 1) % P
    cond = _g(start, nsb) == _g(start, nsa)
    res = np.where(R["enable_start_blocking"] & cond, (~_g(pos, nsa) | (cur == start[cp])) & res, res)
    res = res & (R["enable_circular_board"] | (moved >= start[cp]))
    res = np.where(np.isin(cur, np.concatenate([[-1], goal])), False, res)
    return res


def valid_step_actions(env):
    """dog.py:618-691 -> bool[792] = [joker copies (396), real cards (396)]."""
    cp = sub_player(env)
    hand = env.hands[cp]
    have = hand > 0
    N = env.total_board_size
    nsw = 4 * N
    swaps = val_swap(env).reshape(-1)
    hot = val_action_7_all(env)
    normal = np.stack([val_action_normal_move(env, m) for m in NORMAL_MOVES])      # (12, 4)
    mask = np.concatenate([[hand[11] > 0], hand[[2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13]] > 0])
    neg = val_neg_move(env, -4)
    real = np.concatenate([swaps if have[1] else np.zeros(nsw, bool), hot if have[7] else np.zeros(120, bool),
                           np.where(mask[:, None], normal, False).T.reshape(-1), neg if hand[4] > 0 else np.zeros(4, bool)])
    joker = np.concatenate([swaps, hot, normal.T.reshape(-1), neg]) & (hand[0] > 0)
    return np.concatenate([joker, real])


def valid_actions(env):
    """dog.py:693-711 -> bool[806]."""
    cards = env.hands[env.current_player] > 0
    if env.phase == 0:
        return np.concatenate([valid_step_actions(env), np.zeros_like(cards, bool)])
    return np.concatenate([np.zeros(play_action_size(env), bool), cards])


# ------------------------------------------------------------------------------------ transitions
def _finish(env, cp, board, pins, invalid):
    winner = get_winner(env, board)
    done = bool(env.done or winner.any())
    reward = 0 if env.done else (-1 if invalid else int(winner[cp]))
    return board, pins, reward, done


def step_swap(env, pin_idx, swap_pos):
    """dog.py:755-788 -> (board, pins, reward, done)."""
    cp = sub_player(env)
    N = env.total_board_size
    invalid = not bool(val_swap(env)[int(np.clip(pin_idx, 0, 3)), int(np.clip(swap_pos, 0, N - 1))])
    if invalid:
        return _finish(env, cp, env.board, env.pins, True)
    sp = int(_g(env.board, swap_pos))
    pp = int(env.pins[cp, pin_idx])
    board = env.board.copy()
    board[_si(N, swap_pos)] = cp
    board[_si(N, pp)] = sp
    pins = env.pins.copy()
    pins[cp, pin_idx] = swap_pos
    row = _si(pins.shape[0], sp)
    pins[row] = np.where(pins[row] == swap_pos, pp, pins[row])
    return _finish(env, cp, board, pins, False)


def step_normal_move(env, pin, move):
    """dog.py:790-859."""
    R = env.rules
    cp = sub_player(env)
    pin, move = int(pin), int(move)
    invalid = not bool(val_action_normal_move(env, move)[pin])
    cur = int(env.pins[cp, pin])
    moved = cur + move
    fitted = moved % env.board_size
    x = moved - int(env.target[cp]) - int(R["must_traverse_start"])
    goal = env.goal[cp].astype(np.int64)
    in_goal = cur in goal.tolist()
    if in_goal:
        a = check_goal_path_for_pin(cur - goal[0], moved - goal[0] + 1, goal, env.board, cp)
    else:
        a = check_goal_path_for_pin(-1, x, goal, env.board, cp)
    gx = int(_g(goal, x - 1))
    A = (int(env.board[gx]) != cp) and (R["enable_jump_in_goal_area"] or a)
    if cur == -1:
        new = int(env.start[cp])
    elif in_goal:
        new = moved
    elif (4 >= x > 0) and A and cur <= int(env.target[cp]):
        new = gx
    else:
        new = fitted
    return _capture_move(env, cp, pin, new, invalid)


def _capture_move(env, cp, pin, new, invalid):
    R = env.rules
    pins = env.pins.copy()
    at = int(_g(env.board, new))
    if at != -1 and (at != cp or R["enable_friendly_fire"]) and not invalid:
        row = pins[at]
        pins[at] = np.where(row == new, -1, row)
    if not invalid:
        pins[cp, pin] = new
    board = env.board if invalid else set_pins_on_board(-np.ones_like(env.board), pins)
    return _finish(env, cp, board, pins, invalid)


def step_neg_move(env, pin, move):
    """dog.py:861-911."""
    cp = sub_player(env)
    pin, move = int(pin), int(move)
    invalid = not bool(val_neg_move(env, move)[pin])
    new = (int(env.pins[cp, pin]) + move) % env.board_size
    return _capture_move(env, cp, pin, new, invalid)


def get_path_matrix(start, end, start_idx, goal, target, board_size, total_board_size, traversal_over_start=False):
    """utils/utility_funcs.py:237-303 -> bool[4, total_board_size]."""
    start = np.asarray(start, np.int64)
    end = np.asarray(end, np.int64)
    A = np.isin(start, goal)
    B = np.isin(end, goal)
    same = A == B

    def rng(si, ei, N, same_area):
        idx = np.arange(N)
        if si == -1 or ei == -1 or (same_area and si == ei):
            return np.zeros(N, bool)
        return (idx >= si) & (idx <= ei) if si <= ei else (idx >= si) | (idx <= ei)

    m = np.zeros((4, total_board_size), bool)
    for i in range(4):
        if same[i]:
            m[i, :board_size] = rng(start[i], end[i], board_size, True)
        else:
            m[i, :board_size] = rng(start[i], target, board_size, False)
            m[i] |= rng(goal[0], end[i], total_board_size, False)
    if traversal_over_start and np.any(A != B):
        m[:, start_idx] = True
    return m


def check_moving_pins_hit(i, start, end, matrix):
    """utils/utility_funcs.py:310-319."""
    other = matrix.copy()
    other[i] = False
    o = other.any(0)
    return bool(_g(o, start)) and bool(_g(o, end))


def step_hot_7(env, dist):
    """dog.py:913-985."""
    R = env.rules
    cp = sub_player(env)
    dist = np.asarray(dist, np.int64)
    invalid = not val_action_7(env, dist)
    cur = env.pins[cp].astype(np.int64)
    moved = cur + dist
    fitted = moved % env.board_size
    target = int(env.target[cp])
    x = moved - target - int(R["must_traverse_start"])
    goal = env.goal[cp].astype(np.int64)
    tmp = env.pins.copy()
    tmp[cp] = np.where(np.isin(cur, goal), moved, cur)
    tb = set_pins_on_board(env.board, tmp)
    a = np.array([True if cur[i] in goal.tolist() else check_goal_path_for_pin(-1, int(x[i]), goal, tb, cp)
                  for i in range(4)])
    A = R["enable_jump_in_goal_area"] | a
    new = np.where(cur == -1, -1, np.where(np.isin(cur, goal), moved,
                                            np.where((4 >= x) & (x > 0) & A & (cur <= target), _g(goal, x - 1), fitted)))
    pins = env.pins.copy()
    if not invalid:
        pins[cp] = new
    paths = get_path_matrix(cur, new, int(env.start[cp]), goal, target, env.board_size, env.total_board_size, True)
    anyp = paths.any(0)
    hit = _g(anyp, env.pins.reshape(-1)).reshape(env.pins.shape)
    hit[cp] = [check_moving_pins_hit(i, cur[i], new[i], paths) for i in range(4)]
    if not invalid:
        pins = np.where(hit, -1, pins)
    board = env.board if invalid else set_pins_on_board(-np.ones_like(env.board), pins)
    return _finish(env, cp, board, pins, invalid)


def map_action_to_move(env, action):
    """dog.py:1134-1197 -> [is_joker, is_swap, d0, d1, d2, d3]."""
    size = play_action_size(env)
    half = size // 2
    is_joker = (action - half) < 0
    act = action % half
    pxb = 4 * env.total_board_size
    d = np.zeros(4, np.int64)
    is_swap = act < pxb
    if is_swap:
        d[:] = -1
        d[act // env.total_board_size] = act % env.total_board_size
    elif act < pxb + 120:
        d = DISTS_7_4[act - pxb].astype(np.int64)
    elif act < half - 4:
        na = act - (pxb + 120)
        mv = na % 12 + 1
        mv += int(mv >= 7)
        d[na // 12] = mv
    else:
        d[act - (half - 4)] = -4
    return np.concatenate([[int(is_joker), int(is_swap)], d])


def map_action_to_card(mapped) -> int:
    """dog.py:1241-1262."""
    s = int(np.sum(mapped[2:]))
    if mapped[0] == 1:
        return 0
    if mapped[1] == 1:
        return 1
    if s == -4:
        return 4
    return 11 if s == 1 else s


def map_move_to_action(env, mapped) -> int:
    """dog.py:1199-1239."""
    size = play_action_size(env)
    half = size // 2
    pxb = 4 * env.total_board_size
    d = np.asarray(mapped[2:], np.int64)
    if mapped[1] == 1:
        p = int(np.argmax(d >= 0))
        idx = p * env.total_board_size + int(d[p])
    elif int(d.sum()) == 7:
        idx = pxb + int(np.argmax(np.all(DISTS_7_4 == d[None, :], axis=1)))
    elif np.any(d == -4):
        idx = (half - 4) + int(np.argmax(d == -4))
    else:
        p = int(np.argmax(d != 0))
        mv = int(d[p])
        idx = pxb + 120 + p * 12 + mv - 1 - int(mv > 7)
    return idx if mapped[0] == 1 else idx + half


def _next_with_cards(env, hands):
    tot = hands.astype(np.int64).sum(1)
    for i in range(env.num_players):
        cand = (env.current_player + i + 1) % env.num_players
        if tot[cand] > 0:
            return cand, tot
    return -1, tot


def env_step_play_phase(env, action, shuffle_keys=None):
    """dog.py:987-1063."""
    cp = sub_player(env)
    mapped = map_action_to_move(env, action)
    card = map_action_to_card(mapped)
    valid_card = env.hands[cp, card] > 0
    d = mapped[2:]
    if not valid_card:
        board, pins, reward, done = env.board, env.pins, -1, env.done
    elif mapped[1] == 1:
        p = int(np.argmax(d >= 0))
        board, pins, reward, done = step_swap(env, p, int(d[p]))
    elif int(d.sum()) == 7:
        board, pins, reward, done = step_hot_7(env, d)
    else:
        p = int(np.argmax(d != 0))
        mv = int(d[p])
        board, pins, reward, done = (step_neg_move if mv < 0 else step_normal_move)(env, p, mv)
    hands = env.hands.copy()
    hands[cp, card] += 0 if reward == -1 else -1
    nxt, tot = _next_with_cards(env, hands)
    env2 = env.replace(current_player=cp if done else nxt, board=board, pins=pins, hands=hands, reward=reward,
                       done=done)
    if (np.all(tot == 0) or nxt == -1) and not done:
        env2 = distribute_cards(env2, shuffle_keys)
    return env2, reward, done


def env_step_swap_phase(env, card):
    """dog.py:1078-1116 (no validity check in the reference)."""
    hands = env.hands.copy()
    ci = _si(env.num_cards, card)
    if ci is not None:                       # out-of-range scatter is dropped
        hands[env.current_player, ci] -= 1
    choices = env.swap_choices.copy()
    choices[env.current_player] = np.array(card, np.int64).astype(np.int8)   # jnp.int8(card_idx) wraps
    nxt = (env.current_player + 1) % env.num_players
    complete = nxt == env.round_starter
    if complete:
        partners = [2, 3, 0, 1]
        for p in range(env.num_players):
            rc = int(choices[partners[p]])
            if 0 <= rc < env.num_cards:
                hands[p, rc] += 1
        choices = np.full(4, -1, np.int8)
    env2 = env.replace(current_player=env.round_starter if complete else nxt, hands=hands, swap_choices=choices,
                       phase=0 if complete else env.phase, reward=0)
    return env2, 0, env.done


def env_step(env, action, shuffle_keys=None):
    """dog.py:1118-1132."""
    if env.phase == 1:
        return env_step_swap_phase(env, int(action) - play_action_size(env))
    return env_step_play_phase(env, int(action), shuffle_keys)


def no_step(env, shuffle_keys=None):
    """dog.py:714-753."""
    hands = env.hands.copy()
    hands[env.current_player] = 0
    nxt, tot = _next_with_cards(env, hands)
    if np.any(tot > 0) and nxt != -1:
        return env.replace(hands=hands, current_player=nxt), 0, env.done
    env2 = distribute_cards(env.replace(hands=hands), shuffle_keys)
    return env2, 0, env2.done
