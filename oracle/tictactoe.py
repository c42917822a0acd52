"""CPU oracle: TicTacToeV2 + mctx.muzero_policy with rollout values (TEST INFRASTRUCTURE ONLY).

Restates TicTacToe/TicTacToeV2.py:14-140 (env_step with its operator-precedence quirks: the oldest
move is removed whenever it exists, even on an invalid or post-terminal move, and
``done = (env.done | reward) != (0 | invalid | full)``), the rollout value of policy_function, and
TicTacToe/mcts.py:9-23 ``run_mcts`` = mctx 0.0.6 ``muzero_policy`` (dirichlet_fraction 0,
qtransform_by_min_max(-1, 1), pb_c 1.25 / 19652, max_depth 9, no invalid-action mask) plus the
eval.py:28-55 / 97-125 match protocol (MCTS player = argmax of action_weights over empty cells, random
player = uniform over empty cells, 30-ply limit).

Randomness: jax threefry keys are replaced by the engine's counter streams (csrc/tictactoe.cpp:
ttt_gumbel / ttt_tiebreak), restated here bit-exactly; tree arithmetic is evaluated in double with the
C library's exp / log / sqrt (Python's math module) on both sides, so the product and this oracle agree
exactly.  Parity with the JAX reference: UNPINNED (no reference test covers TicTacToe; mctx is not
vendored; the reference computes in float32).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

M64 = 0xFFFFFFFFFFFFFFFF
ROLLOUT_STREAM = 0x7A11D0E5
TIE_STREAM = 0x71EB4EA5
ACTION_STREAM = 0xAC710B
RANDOM_STREAM = 0x4A4D0B07
MAX_ROLLOUT = 1000
LINES = ((0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6))


def _mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def _key(seed, stream, a, b):
    return (seed ^ stream ^ _mix64(((a & 0xFFFFFFFF) << 32) | (b & 0xFFFFFFFF))) & M64


def _u_open(h):
    """U(0, 1) on a 24-bit grid, never 0 or 1."""
    return ((h >> 40) + 0.5) / 16777216.0


def ttt_gumbel(seed, stream, a, b, action):
    h = _mix64(_key(seed, stream, a, b) ^ (((action + 1) * 0xD6E8FEB86659FD93) & M64))
    return -math.log(-math.log(_u_open(h)))


def ttt_tiebreak(seed, turn, sim, depth, action):
    h = _mix64(_key(seed, TIE_STREAM, turn, (sim << 8) | depth) ^ (((action + 1) * 0x9E6C63D0676A9A99) & M64))
    return (h >> 40) / 16777216.0


@dataclass
class State:
    board: list = field(default_factory=lambda: [0] * 9)
    current_player: int = 1
    reward: int = 0
    done: bool = False
    memory: list = field(default_factory=lambda: [[-1, -1, -1], [-1, -1, -1]])

    def copy(self):
        return State(list(self.board), self.current_player, self.reward, self.done, [list(self.memory[0]),
                                                                                    list(self.memory[1])])


def env_reset():
    return State()


def get_winner(board):
    sums = [board[a] + board[b] + board[c] for a, b, c in LINES]
    w = 1 if 3 in sums else 0
    return -1 if -3 in sums else w


def env_step(env: State, action: int):
    """TicTacToeV2.env_step (46-76) -> (state, reward, done)."""
    a = int(action)
    row, col = a // 3, a % 3
    cell = 3 * (row if row >= 0 else row + 3) + (col if col >= 0 else col + 3)
    invalid = env.board[cell] != 0
    p = 1 if env.current_player < 0 else 0
    old = env.memory[p]
    rolled = [old[1], old[2], old[0]]
    removed = rolled[2]
    new_row = [rolled[0], rolled[1], a]
    memory = [list(env.memory[0]), list(env.memory[1])]
    if not (env.done or invalid):
        memory[p] = new_row
    board = list(env.board)
    if not (env.done or invalid):
        board[cell] = env.current_player
    # `env.done | invalid_move | removed_action == -1` is `(done | invalid | removed) == -1`: true only for
    # removed == -1, so an existing oldest move is cleared even on an invalid or post-terminal step
    if removed != -1:
        board[3 * (removed // 3) + removed % 3] = 0
    reward = 0 if env.done else (-1 if invalid else get_winner(board) * env.current_player)
    lhs = reward | (1 if env.done else 0)
    rhs = 1 if (invalid or all(v != 0 for v in board)) else 0
    done = lhs != rhs
    nxt = State(board, env.current_player if done else -env.current_player, reward, done, memory)
    return nxt, reward, done


def valid_action_mask(env: State):
    return [False] * 9 if env.done else [v == 0 for v in env.board]


def winning_action_mask(env: State, player: int):
    e = env.copy()
    e.current_player = player
    return [env_step(e, a)[1] == 1 for a in range(9)]


def policy_function(env: State):
    v = valid_action_mask(env)
    opp = winning_action_mask(env, -env.current_player)
    own = winning_action_mask(env, env.current_player)
    return [100.0 * v[a] + 200.0 * opp[a] + 300.0 * own[a] for a in range(9)]


def categorical(logits, seed, stream, a, b):
    """jax.random.categorical = argmax(logits + Gumbel) with the counter Gumbel (first index on ties)."""
    best, arg = -math.inf, 0
    for i, l in enumerate(logits):
        s = l + ttt_gumbel(seed, stream, a, b, i)
        if s > best:
            best, arg = s, i
    return arg


def rollout(env: State, seed, eval_id):
    """TicTacToeV2.rollout (108-119): policy_function-sampled play to the end (guard: MAX_ROLLOUT plies)."""
    leaf = env
    ply = 0
    while not leaf.done and ply < MAX_ROLLOUT:
        a = categorical(policy_function(leaf), seed, ROLLOUT_STREAM, eval_id, ply)
        leaf = env_step(leaf, a)[0]
        ply += 1
    return float(leaf.reward * leaf.current_player * env.current_player) if leaf.done else 0.0


def _softmax(x):
    m = max(x)
    e = [math.exp(v - m) for v in x]
    s = sum(e)
    return [v / s for v in e]


class _Tree:
    def __init__(self, n):
        self.visits = [0] * n
        self.raw = [0.0] * n
        self.value = [0.0] * n
        self.emb = [None] * n
        self.parent = [-1] * n
        self.afp = [-1] * n
        self.c_index = [[-1] * 9 for _ in range(n)]
        self.c_prior = [[0.0] * 9 for _ in range(n)]
        self.c_value = [[0.0] * 9 for _ in range(n)]
        self.c_visits = [[0] * 9 for _ in range(n)]
        self.c_reward = [[0.0] * 9 for _ in range(n)]
        self.c_disc = [[0.0] * 9 for _ in range(n)]


def muzero_policy(root: State, num_simulations=25, max_depth=9, temperature=1.0, seed=0, turn=0):
    """run_mcts (mcts.py:9-23) -> (action, action_weights[9], root value, visit counts[9])."""
    S = num_simulations
    t = _Tree(S + 1)
    pl = policy_function(root)
    tiny = 1.1754943508222875e-38
    # dirichlet_fraction 0: logits = log(max(softmax(prior), tiny)); no invalid-action mask
    t.c_prior[0] = [math.log(max(p, tiny)) for p in _softmax(pl)]
    v0 = rollout(root, seed, turn << 10)
    t.raw[0] = t.value[0] = v0
    t.visits[0] = 1
    t.emb[0] = root

    def select(n, sim, depth):
        vis = t.c_visits[n]
        nv = t.visits[n]
        pb_c = 1.25 + math.log((nv + 19652.0 + 1.0) / 19652.0)
        probs = _softmax(t.c_prior[n])
        best, arg = -math.inf, 0
        for a in range(9):
            q = t.c_reward[n][a] + t.c_disc[n][a] * t.c_value[n][a]
            vs = (q if vis[a] > 0 else -1.0) + 1.0    # qtransform_by_min_max(-1, 1): (q - min) / (max - min)
            vs = vs / 2.0
            ps = math.sqrt(nv) * pb_c * probs[a] / (vis[a] + 1)
            s = vs + ps + 1e-7 * ttt_tiebreak(seed, turn, sim, depth, a)
            if s > best:
                best, arg = s, a
        return arg

    for sim in range(S):
        node, depth = 0, 0
        while True:
            a = select(node, sim, depth)
            nxt = t.c_index[node][a]
            depth += 1
            if nxt == -1 or depth >= max_depth:
                break
            node = nxt
        parent, action = node, a
        child = t.c_index[parent][action]
        if child == -1:
            child = sim + 1
        env, r, d = env_step(t.emb[parent], action)
        t.c_prior[child] = policy_function(env)
        v = 0.0 if d else rollout(env, seed, (turn << 10) | (sim + 1))
        t.raw[child] = t.value[child] = v
        t.visits[child] += 1
        t.emb[child] = env
        t.c_index[parent][action] = child
        t.c_reward[parent][action] = float(r)
        t.c_disc[parent][action] = 0.0 if d else -1.0
        t.parent[child] = parent
        t.afp[child] = action
        # backward
        leaf_v = t.value[child]
        idx = child
        while idx != 0:
            p = t.parent[idx]
            a = t.afp[idx]
            leaf_v = t.c_reward[p][a] + t.c_disc[p][a] * leaf_v
            cnt = t.visits[p]
            t.value[p] = (t.value[p] * cnt + leaf_v) / (cnt + 1.0)
            t.visits[p] = cnt + 1
            t.c_value[p][a] = t.value[idx]
            t.c_visits[p][a] += 1
            idx = p
    visits = list(t.c_visits[0])
    tot = sum(visits)
    weights = [v / max(tot, 1) for v in visits]
    logits = [math.log(w) if w > 0 else -math.inf for w in weights]
    m = max(logits)
    logits = [l - m for l in logits]
    scaled = [l / max(tiny, temperature) for l in logits]
    action = categorical(scaled, seed, ACTION_STREAM, turn, 0)
    return action, weights, t.value[0], visits


def mcts_action(env: State, num_simulations, seed, turn):
    """eval.py:28-34 get_mcts_action: argmax of the search's action_weights over empty cells."""
    _, w, _, _ = muzero_policy(env, num_simulations, 9, 1.0, seed, turn)
    best, arg = -math.inf, 0
    for a in range(9):
        s = w[a] if env.board[a] == 0 else -math.inf
        if s > best:
            best, arg = s, a
    return arg


def random_action(env: State, seed, game, ply):
    """eval.py:51-55 get_random_action: uniform over empty cells."""
    return categorical([0.0 if v == 0 else -math.inf for v in env.board], seed, RANDOM_STREAM, game, ply)


def match(mcts_player, num_simulations, seed, game, limit=30):
    """eval.py:97-125 / 252-276: MCTS player vs random player -> winner * mcts_player (0 at the ply limit)."""
    env = env_reset()
    ply = 0
    gseed = _mix64(seed ^ ((game + 1) * 0x632BE59BD9B4E019 & M64))
    while not env.done and ply < limit:
        if env.current_player == mcts_player:
            a = mcts_action(env, num_simulations, gseed, ply)
        else:
            a = random_action(env, seed, game, ply)
        env = env_step(env, a)[0]
        ply += 1
    return 0 if ply == limit else get_winner(env.board) * mcts_player
