// TicTacToeV2 + mctx.muzero_policy with rollout values (config (a): CPU plumbing, one game, S = 25).
//
// Host C++ in libmuz.so: TicTacToe/TicTacToeV2.py:14-140 (env_step keeps its operator-precedence
// quirks), TicTacToe/mcts.py:9-23 run_mcts = mctx 0.0.6 muzero_policy (dirichlet_fraction 0,
// qtransform_by_min_max(-1, 1), pb_c 1.25 / 19652, max_depth 9, no invalid-action mask) and the
// eval.py match protocol.  jax threefry keys are replaced by counter streams (include/muz.h); tree
// arithmetic is double with strict evaluation order so oracle/tictactoe.py reproduces it exactly.
#pragma clang fp contract(off)

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/muz.h"

namespace {

constexpr uint64_t kRolloutStream = 0x7A11D0E5ull, kTieStream = 0x71EB4EA5ull, kActionStream = 0xAC710Bull,
                   kRandomStream = 0x4A4D0B07ull;
constexpr int kMaxRollout = 1000;
constexpr double kTiny = 1.1754943508222875e-38;
constexpr int kLines[8][3] = {{0, 1, 2}, {3, 4, 5}, {6, 7, 8}, {0, 3, 6}, {1, 4, 7}, {2, 5, 8}, {0, 4, 8}, {2, 4, 6}};

inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline uint64_t key(uint64_t seed, uint64_t stream, uint32_t a, uint32_t b) {
  return seed ^ stream ^ mix64(((uint64_t)a << 32) | b);
}
inline double gumbel(uint64_t seed, uint64_t stream, uint32_t a, uint32_t b, int action) {
  const uint64_t h = mix64(key(seed, stream, a, b) ^ (uint64_t)(action + 1) * 0xD6E8FEB86659FD93ull);
  const double u = ((double)(h >> 40) + 0.5) / 16777216.0;
  return -std::log(-std::log(u));
}
inline double tiebreak(uint64_t seed, int turn, int sim, int depth, int action) {
  const uint64_t h = mix64(key(seed, kTieStream, (uint32_t)turn, ((uint32_t)sim << 8) | (uint32_t)depth) ^
                           (uint64_t)(action + 1) * 0x9E6C63D0676A9A99ull);
  return (double)(h >> 40) / 16777216.0;
}

int winner(const int8_t* b) {
  bool p = false, n = false;
  for (const auto& l : kLines) {
    const int s = b[l[0]] + b[l[1]] + b[l[2]];
    p |= s == 3;
    n |= s == -3;
  }
  return n ? -1 : (p ? 1 : 0);
}

// TicTacToeV2.env_step (46-76).
muz_ttt_state step(const muz_ttt_state& e, int a, int* reward_out, bool* done_out) {
  int row = a / 3, col = a % 3;   // floor div / mod (a >= 0 on every path that reaches here)
  if (a < 0) {
    row = (a - 2) / 3;
    col = a - 3 * row;
  }
  const int cell = 3 * (row < 0 ? row + 3 : row) + (col < 0 ? col + 3 : col);
  const bool invalid = e.board[cell] != 0;
  const int p = e.current_player < 0 ? 1 : 0;
  const int8_t* old = e.memory + 3 * p;
  const int removed = old[0];   // jnp.roll(-1) then [-1]: the oldest move
  muz_ttt_state n = e;
  if (!(e.done || invalid)) {
    n.memory[3 * p + 0] = old[1];
    n.memory[3 * p + 1] = old[2];
    n.memory[3 * p + 2] = (int8_t)a;
    n.board[cell] = e.current_player;
  }
  // `done | invalid | removed == -1` parses as `(done | invalid | removed) == -1`: an existing oldest move
  // is cleared even on an invalid or post-terminal step
  if (removed != -1) n.board[3 * (removed / 3) + removed % 3] = 0;
  const int reward = e.done ? 0 : (invalid ? -1 : winner(n.board) * e.current_player);
  bool full = true;
  for (int i = 0; i < 9; ++i) full &= n.board[i] != 0;
  // `env.done | reward != 0 | invalid_move | all(board != 0)` = `(done | reward) != (0 | invalid | full)`
  const int lhs = reward | (e.done ? 1 : 0);
  const int rhs = (invalid || full) ? 1 : 0;
  const bool done = lhs != rhs;
  n.reward = (int8_t)reward;
  n.done = done ? 1 : 0;
  n.current_player = done ? e.current_player : (int8_t)-e.current_player;
  if (reward_out) *reward_out = reward;
  if (done_out) *done_out = done;
  return n;
}

// policy_function (TicTacToeV2.py:97-104): 100 legal + 200 opponent's winning move + 300 own winning move.
void policy(const muz_ttt_state& e, double* out) {
  muz_ttt_state opp = e, own = e;
  opp.current_player = (int8_t)-e.current_player;
  for (int a = 0; a < 9; ++a) {
    const bool legal = !e.done && e.board[a] == 0;
    int ro = 0, rw = 0;
    step(opp, a, &ro, nullptr);
    step(own, a, &rw, nullptr);
    out[a] = 100.0 * (legal ? 1 : 0) + 200.0 * (ro == 1 ? 1 : 0) + 300.0 * (rw == 1 ? 1 : 0);
  }
}

int categorical(const double* logits, uint64_t seed, uint64_t stream, uint32_t a, uint32_t b) {
  double best = -INFINITY;
  int arg = 0;
  for (int i = 0; i < 9; ++i) {
    const double s = logits[i] + gumbel(seed, stream, a, b, i);
    if (s > best) {
      best = s;
      arg = i;
    }
  }
  return arg;
}

// rollout (108-119) -> value from the perspective of e's player.
double rollout(const muz_ttt_state& e, uint64_t seed, uint32_t eval_id) {
  muz_ttt_state leaf = e;
  double lg[9];
  int ply = 0;
  while (!leaf.done && ply < kMaxRollout) {
    policy(leaf, lg);
    leaf = step(leaf, categorical(lg, seed, kRolloutStream, eval_id, (uint32_t)ply), nullptr, nullptr);
    ++ply;
  }
  return leaf.done ? (double)(leaf.reward * leaf.current_player * e.current_player) : 0.0;
}

void softmax9(const double* x, double* p) {
  double m = x[0];
  for (int i = 1; i < 9; ++i) m = x[i] > m ? x[i] : m;
  double s = 0.0;
  for (int i = 0; i < 9; ++i) {
    p[i] = std::exp(x[i] - m);
    s += p[i];
  }
  for (int i = 0; i < 9; ++i) p[i] = p[i] / s;
}

struct Tree {
  int n;
  std::vector<int> visits, parent, afp, c_index, c_visits;
  std::vector<double> value, c_prior, c_value, c_reward, c_disc;
  std::vector<muz_ttt_state> emb;
  explicit Tree(int N)
      : n(N), visits(N, 0), parent(N, -1), afp(N, -1), c_index(9 * N, -1), c_visits(9 * N, 0), value(N, 0.0),
        c_prior(9 * N, 0.0), c_value(9 * N, 0.0), c_reward(9 * N, 0.0), c_disc(9 * N, 0.0), emb(N) {}
};

// mctx muzero_action_selection with qtransform_by_min_max(-1, 1) and the 1e-7 tie-break uniform.
int select(const Tree& t, int node, uint64_t seed, int turn, int sim, int depth) {
  const int nv = t.visits[node];
  const double pb_c = 1.25 + std::log(((double)nv + 19652.0 + 1.0) / 19652.0);
  double probs[9];
  softmax9(&t.c_prior[9 * node], probs);
  double best = -INFINITY;
  int arg = 0;
  for (int a = 0; a < 9; ++a) {
    const int e = 9 * node + a;
    const double q = t.c_reward[e] + t.c_disc[e] * t.c_value[e];
    double vs = (t.c_visits[e] > 0 ? q : -1.0) + 1.0;
    vs = vs / 2.0;
    const double ps = std::sqrt((double)nv) * pb_c * probs[a] / (double)(t.c_visits[e] + 1);
    const double s = vs + ps + 1e-7 * tiebreak(seed, turn, sim, depth, a);
    if (s > best) {
      best = s;
      arg = a;
    }
  }
  return arg;
}

void muzero_policy(const muz_ttt_state& root, int S, int D, double temperature, uint64_t seed, int turn,
                   muz_ttt_policy_out* out) {
  Tree t(S + 1);
  double pl[9], pr[9];
  policy(root, pl);
  softmax9(pl, pr);
  for (int a = 0; a < 9; ++a) t.c_prior[a] = std::log(pr[a] > kTiny ? pr[a] : kTiny);
  t.value[0] = rollout(root, seed, (uint32_t)turn << 10);
  t.visits[0] = 1;
  t.emb[0] = root;
  for (int sim = 0; sim < S; ++sim) {
    int node = 0, depth = 0, a = 0;
    for (;;) {
      a = select(t, node, seed, turn, sim, depth);
      const int nxt = t.c_index[9 * node + a];
      ++depth;
      if (nxt == -1 || depth >= D) break;
      node = nxt;
    }
    const int parent = node, action = a;
    int child = t.c_index[9 * parent + action];
    if (child == -1) child = sim + 1;
    int r = 0;
    bool d = false;
    const muz_ttt_state env = step(t.emb[parent], action, &r, &d);
    double lg[9];
    policy(env, lg);
    for (int k = 0; k < 9; ++k) t.c_prior[9 * child + k] = lg[k];
    t.value[child] = d ? 0.0 : rollout(env, seed, ((uint32_t)turn << 10) | (uint32_t)(sim + 1));
    t.visits[child] += 1;
    t.emb[child] = env;
    t.c_index[9 * parent + action] = child;
    t.c_reward[9 * parent + action] = (double)r;
    t.c_disc[9 * parent + action] = d ? 0.0 : -1.0;
    t.parent[child] = parent;
    t.afp[child] = action;
    double leaf_v = t.value[child];
    for (int idx = child; idx != 0;) {
      const int p = t.parent[idx], pa = t.afp[idx], e = 9 * p + pa;
      leaf_v = t.c_reward[e] + t.c_disc[e] * leaf_v;
      const int cnt = t.visits[p];
      t.value[p] = (t.value[p] * (double)cnt + leaf_v) / ((double)cnt + 1.0);
      t.visits[p] = cnt + 1;
      t.c_value[e] = t.value[idx];
      t.c_visits[e] += 1;
      idx = p;
    }
  }
  int tot = 0;
  for (int a = 0; a < 9; ++a) tot += t.c_visits[a];
  double lw[9], m = -INFINITY;
  for (int a = 0; a < 9; ++a) {
    out->visits[a] = t.c_visits[a];
    out->action_weights[a] = (double)t.c_visits[a] / (double)(tot > 1 ? tot : 1);
    lw[a] = out->action_weights[a] > 0.0 ? std::log(out->action_weights[a]) : -INFINITY;
    m = lw[a] > m ? lw[a] : m;
  }
  const double tt = temperature > kTiny ? temperature : kTiny;
  for (int a = 0; a < 9; ++a) lw[a] = (lw[a] - m) / tt;
  out->action = categorical(lw, seed, kActionStream, (uint32_t)turn, 0u);
  out->value = t.value[0];
}

}  // namespace

extern "C" {

int muz_ttt_reset(muz_ttt_state* s) {
  if (!s) return MUZ_E_INVALID;
  std::memset(s, 0, sizeof(*s));
  s->current_player = 1;
  for (int i = 0; i < 6; ++i) s->memory[i] = -1;
  return MUZ_OK;
}

int muz_ttt_step(muz_ttt_state* s, int32_t action, int8_t* reward, uint8_t* done) {
  if (!s || action < 0 || action > 8) return MUZ_E_INVALID;
  int r = 0;
  bool d = false;
  *s = step(*s, action, &r, &d);
  if (reward) *reward = (int8_t)r;
  if (done) *done = d ? 1 : 0;
  return MUZ_OK;
}

int muz_ttt_policy_logits(const muz_ttt_state* s, double* logits) {
  if (!s || !logits) return MUZ_E_INVALID;
  policy(*s, logits);
  return MUZ_OK;
}

int muz_ttt_rollout(const muz_ttt_state* s, uint64_t seed, uint32_t eval_id, double* value) {
  if (!s || !value) return MUZ_E_INVALID;
  *value = rollout(*s, seed, eval_id);
  return MUZ_OK;
}

int muz_ttt_muzero_policy(const muz_ttt_state* root, int32_t num_simulations, int32_t max_depth, double temperature,
                          uint64_t seed, int32_t turn, muz_ttt_policy_out* out) {
  if (!root || !out || num_simulations < 1 || num_simulations > 4096 || max_depth < 1) return MUZ_E_INVALID;
  muzero_policy(*root, num_simulations, max_depth, temperature, seed, turn, out);
  return MUZ_OK;
}

int muz_ttt_match(int32_t mcts_player, int32_t num_simulations, uint64_t seed, int32_t game, int32_t limit,
                  int32_t* result) {
  if (!result || (mcts_player != 1 && mcts_player != -1) || num_simulations < 1 || limit < 1) return MUZ_E_INVALID;
  muz_ttt_state e;
  muz_ttt_reset(&e);
  const uint64_t gseed = mix64(seed ^ ((uint64_t)(game + 1) * 0x632BE59BD9B4E019ull));
  int ply = 0;
  while (!e.done && ply < limit) {
    int a = 0;
    if (e.current_player == mcts_player) {   // eval.py:28-34: argmax of action_weights over empty cells
      muz_ttt_policy_out o;
      muzero_policy(e, num_simulations, 9, 1.0, gseed, ply, &o);
      double best = -INFINITY;
      for (int k = 0; k < 9; ++k) {
        const double s = e.board[k] == 0 ? o.action_weights[k] : -INFINITY;
        if (s > best) {
          best = s;
          a = k;
        }
      }
    } else {                                 // eval.py:51-55: uniform over empty cells
      double lg[9];
      for (int k = 0; k < 9; ++k) lg[k] = e.board[k] == 0 ? 0.0 : -INFINITY;
      a = categorical(lg, seed, kRandomStream, (uint32_t)game, (uint32_t)ply);
    }
    e = step(e, a, nullptr, nullptr);
    ++ply;
  }
  *result = ply == limit ? 0 : winner(e.board) * mcts_player;
  return MUZ_OK;
}

}  // extern "C"
