// CPU restatement of classic-MADN Stochastic MuZero self-play in C++ with OpenMP over games.
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY: the "port" CPU baseline of SURVEY.md §8(d) for config (c) -- the
// reference algorithm (MADN/classic_madn.py env, MuZero_Classic_MADN/muzero_classic_madn.py networks incl.
// StochasticDynamicsNetwork4, mctx 0.0.6 stochastic_muzero_policy, MuZero_Classic_MADN/
// game_agent_stochastic.py:52-218 self-play loop) restated as plain fp32 C++ so bench.py can time it on the
// GPU box's host cores beside the HIP engine.  It follows the NumPy oracle line by line (oracle/classic_madn.py,
// oracle/classic_nets.py, oracle/mctx_stochastic.py, oracle/selfplay.py:play_batch_of_games_stochastic) and is
// checked against it by tests/test_cpu_baseline_classic.py.  Only tests/ and bench.py's cpu_baseline leg load
// it; the product path never does.
//
// Randomness: the die, the 1e-7 tie-break uniforms and the final categorical's Gumbel draws use the engine's
// counter RNG (as the oracle restates it), so a trace can be compared with the oracle's; the root Dirichlet
// noise (fraction 0.25, alpha 0.3 in the reference) is drawn here with Marsaglia-Tsang gamma samples from the
// same counter hash -- parity-checked runs use fraction 0, as the oracle does.
#include "cpu_nets.hpp"

namespace {

constexpr int kAc = 4, kCh = 6, kAp = kAc + kCh;   // pins, die outcomes, child slots of a node

}  // namespace

extern "C" {

// one classic_MADN state (classic_madn.py:33-49); pins / goal rows = players
typedef struct {
  int8_t board[kCells];
  int8_t pins[16];
  int8_t start[4], target[4], goal[16];
  int32_t current_player, reward, done, num_players, board_size, total, rules, die;
} muzcpu_classic;

}  // extern "C"

namespace {

inline bool has(const muzcpu_classic& e, uint32_t f) { return (e.rules & f) != 0; }

void set_pins_on_board(int8_t* board, const int8_t* pins, int P, int total) {   // deterministic_madn.py:259-271
  for (int i = 0; i < total; ++i) board[i] = -1;
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < 4; ++k) {
      const int pos = pins[p * 4 + k];
      if (pos >= 0 && pos < total) board[pos] = (int8_t)p;
    }
}

bool is_player_done(const muzcpu_classic& e, const int8_t* board, int p) {
  if (p >= e.num_players) return false;
  for (int k = 0; k < 4; ++k)
    if (board[e.goal[p * 4 + k]] < 0) return false;
  return true;
}

void get_winner(const muzcpu_classic& e, const int8_t* board, bool w[4]) {
  bool d[4];
  for (int p = 0; p < 4; ++p) d[p] = is_player_done(e, board, p);
  if (!has(e, R_TEAMS)) {
    for (int p = 0; p < 4; ++p) w[p] = d[p];
    return;
  }
  const bool t0 = d[0] && d[2], t1 = d[1] && d[3];
  for (int p = 0; p < 4; ++p) w[p] = false;
  if ((t0 && t1) || !(t0 || t1)) return;
  if (t0) w[0] = w[2] = true; else w[1] = w[3] = true;
}

int sub_player(const muzcpu_classic& e) {   // classic_madn.py:275 / 409
  const int p = e.current_player;
  return (has(e, R_TEAMS) && is_player_done(e, e.board, p)) ? (p + 2) % 4 : p;
}

bool goal_path_free(long long start, long long x, const int8_t* goal, const int8_t* board, int cp) {
  for (int ga = 0; ga < 4; ++ga)
    if (start < ga && ga < x && board[goal[ga]] == cp) return false;
  return true;
}

void valid_action(const muzcpu_classic& e, bool va[4]) {   // classic_madn.py:367-461
  const int cp = sub_player(e), P = e.num_players, bs = e.board_size;
  const int8_t* board = e.board;
  const int8_t* goal = e.goal + cp * 4;
  const long long target = e.target[cp], die = e.die;
  const long long mt = has(e, R_MUST_TRAVERSE) ? 1 : 0;
  bool pos_[4];
  for (int p = 0; p < P; ++p) pos_[p] = board[e.start[p]] == p;
  const long long dist = bs / 4;
  for (int i = 0; i < 4; ++i) {
    const long long cur = e.pins[cp * 4 + i];
    const long long moved = cur + die;
    const long long fitted = pymod(moved, bs);
    long long x = moved - target - mt;
    bool res = (board[fitted] != cp) || has(e, R_FRIENDLY);
    const long long nsb = pymod(floordiv(cur, dist) + 1, P);
    const long long nsa = floordiv(fitted, dist);
    const bool trav = e.start[gidx(nsb, P)] == e.start[gidx(nsa, P)];
    const bool pos_nsa = pos_[gidx(nsa, P)];
    if (has(e, R_START_BLOCK) && trav) res = (!pos_nsa || cur == e.start[cp]) && res;
    if (has(e, R_MUST_TRAVERSE) && has(e, R_START_BLOCK) && trav && pos_nsa) x = 0;
    if (!has(e, R_CIRCULAR) && cur <= target && (x > 4 || (x == 0 && has(e, R_MUST_TRAVERSE)))) res = false;
    const bool A = has(e, R_CIRCULAR) && res;
    const bool B = board[goal[gidx(x - 1, 4)]] != cp;
    const bool C = has(e, R_JUMP_GOAL) || goal_path_free(-1, x, goal, board, cp);
    if (4 >= x && x > 0 && cur <= target) res = A || (B && C);
    const bool D = has(e, R_JUMP_GOAL) || goal_path_free(cur - goal[0], moved - goal[0] + 1, goal, board, cp);
    bool in_goal = false;
    for (int k = 0; k < 4; ++k) in_goal = in_goal || cur == goal[k];
    if (in_goal) res = (moved <= goal[3]) && (board[gidx(moved, e.total)] != cp) && D;
    const bool start_move = die == 6 || (die == 1 && has(e, R_START_ON_1));
    if (cur == -1) res = start_move && !pos_[cp];       // ~pins_on_start[cp_sub] (455-459)
    va[i] = res;
  }
}

void env_reset(muzcpu_classic& e, int P, const int* layout, int distance, int starting_player, int rules) {   // 51-131
  std::memset(&e, 0, sizeof(e));
  e.rules = rules;
  if (P != 4) e.rules &= ~R_TEAMS;
  e.num_players = P;
  e.board_size = 4 * distance;
  e.total = e.board_size + 16;
  bool lay[4];
  int cnt = 0;
  for (int i = 0; i < 4; ++i) cnt += (lay[i] = layout[i] != 0);
  if (cnt != P || (cnt == 4 && P < 4))
    for (int i = 0; i < 4; ++i) lay[i] = i < P;
  int k = 0;
  for (int s = 0; s < 4; ++s) {
    if (!lay[s]) continue;
    e.start[k] = (int8_t)(s * distance);
    e.target[k] = (int8_t)pymod(s * distance - 1, e.board_size);
    for (int j = 0; j < 4; ++j) e.goal[k * 4 + j] = (int8_t)(e.board_size + 4 * s + j);
    ++k;
  }
  for (int i = 0; i < 16; ++i) e.pins[i] = -1;
  if (e.rules & R_FREE_PIN)
    for (int p = 0; p < P; ++p) e.pins[p * 4] = e.start[p];
  set_pins_on_board(e.board, e.pins, P, e.total);
  e.current_player = starting_player;
}

bool is_soft_locked(const muzcpu_classic& e) {   // 180-206 (the UNSUBSTITUTED current player)
  const int cp = e.current_player;
  int not_home = 0;
  for (int k = 0; k < 4; ++k) not_home += e.pins[cp * 4 + k] != -1;
  if (not_home == 0) return true;
  for (int j = 0; j < 4; ++j) {
    const bool relevant = j >= 4 - not_home;
    if (relevant && e.board[e.goal[cp * 4 + j]] != cp) return false;
  }
  return true;
}

void dice_probabilities(const muzcpu_classic& e, float p[6]) {   // 208-228 (classic_madn.py:12-18)
  if (is_soft_locked(e) && has(e, R_DICE_RETHROW)) {
    if (has(e, R_START_ON_1)) {
      for (int i = 0; i < 6; ++i) p[i] = (i == 0 || i == 5) ? (float)(76.0 / 216.0) : (float)(16.0 / 216.0);
    } else {
      for (int i = 0; i < 6; ++i) p[i] = i == 5 ? (float)(91.0 / 216.0) : (float)(25.0 / 216.0);
    }
  } else {
    for (int i = 0; i < 6; ++i) p[i] = (float)(1.0 / 6.0);
  }
}

// jax.random.choice(key, [1..6], p=p) with the uniform made explicit: cum = cumsum(p) (fp32, sequential),
// r = cum[-1] * (1 - u), searchsorted left (oracle/classic_madn.py:choice_from_uniform)
int choice_from_uniform(const float p[6], float u) {
  float cum[6], c = 0.f;
  for (int i = 0; i < 6; ++i) cum[i] = (c += p[i]);
  const float r = cum[5] * (1.0f - u);
  int k = 0;
  while (k < 6 && cum[k] < r) ++k;
  return k + 1;
}

void env_step(muzcpu_classic& e, int pin, int& reward_out, int& done_out) {   // 257-337
  const int player_id = e.current_player, cp = sub_player(e);
  const int move = e.die;
  bool va[4];
  valid_action(e, va);
  const int pi = (int)std::min(std::max(pin < 0 ? pin + 4 : pin, 0), 3);
  const bool invalid = !va[gidx(pin, 4)];
  const long long cur = e.pins[cp * 4 + pi];
  const long long moved = cur + move;
  const long long fitted = pymod(moved, e.board_size);
  const long long x = moved - e.target[cp] - (has(e, R_MUST_TRAVERSE) ? 1 : 0);
  const int8_t* goal = e.goal + cp * 4;
  const int8_t* board = e.board;
  bool in_goal = false;
  for (int k = 0; k < 4; ++k) in_goal = in_goal || cur == goal[k];
  const bool a = in_goal ? goal_path_free(cur - goal[0], moved - goal[0] + 1, goal, board, cp)
                         : goal_path_free(-1, x, goal, board, cp);
  const bool A = (board[goal[gidx(x - 1, 4)]] != cp) && (has(e, R_JUMP_GOAL) || a);
  long long new_pos;
  if (cur == -1) new_pos = e.start[cp];
  else if (in_goal) new_pos = moved;
  else if (4 >= x && x > 0 && A && cur <= e.target[cp]) new_pos = goal[gidx(x - 1, 4)];
  else new_pos = fitted;
  const int pin_at = board[gidx(new_pos, e.total)];
  int8_t pins[16];
  std::memcpy(pins, e.pins, 16);
  if (pin_at != -1 && (pin_at != cp || has(e, R_FRIENDLY)) && !invalid)
    for (int k = 0; k < 4; ++k)
      if (pins[pin_at * 4 + k] == new_pos) pins[pin_at * 4 + k] = -1;
  if (!invalid) pins[cp * 4 + pi] = (int8_t)new_pos;
  int8_t nb[kCells];
  if (invalid) std::memcpy(nb, e.board, kCells);
  else set_pins_on_board(nb, pins, e.num_players, e.total);
  bool w[4];
  get_winner(e, nb, w);
  const int reward = e.done ? 0 : (invalid ? -1 : (w[cp] ? 1 : 0));
  const bool done = e.done || w[0] || w[1] || w[2] || w[3];
  const int nxt = (done || (has(e, R_BONUS_6) && move == 6)) ? player_id : (player_id + 1) % e.num_players;
  std::memcpy(e.board, nb, kCells);
  std::memcpy(e.pins, pins, 16);
  e.current_player = nxt;
  e.done = done;
  e.reward = reward;
  reward_out = reward;
  done_out = done;
}

void no_step(muzcpu_classic& e) { e.current_player = (e.current_player + 1) % e.num_players; }   // 353-365

void encode_board(const muzcpu_classic& e, float* out) {   // 463-497 -> [2P+3][56]
  const int P = e.num_players, bs = e.board_size, dist = bs / 4, cp = e.current_player, W = e.total;
  int8_t b[kCells];
  for (int i = 0; i < bs; ++i) b[i] = e.board[(i + dist * cp) % bs];
  for (int i = 0; i < 16; ++i) b[bs + i] = e.board[bs + (i + 4 * cp) % 16];
  int rolled[4];
  for (int k = 0; k < P; ++k) rolled[k] = (k + cp) % P;
  const int C = 2 * P + 3;
  std::memset(out, 0, sizeof(float) * C * W);
  for (int k = 0; k < P; ++k)
    for (int w = 0; w < W; ++w) out[k * W + w] = b[w] == rolled[k] ? 1.f : 0.f;
  for (int w = 0; w < W; ++w) {
    float t = 0.f, o = 0.f;
    for (int k = 0; k < P; ++k) {
      const bool team = has(e, R_TEAMS) ? (k % 2 == 0) : (k == 0);
      (team ? t : o) += out[k * W + w];
    }
    out[P * W + w] = t;
    out[(P + 1) * W + w] = o;
  }
  for (int k = 0; k < P; ++k) {
    int home = 0;
    for (int j = 0; j < 4; ++j) home += e.pins[rolled[k] * 4 + j] == -1;
    for (int w = 0; w < W; ++w) out[(P + 2 + k) * W + w] = (float)home;
  }
  for (int w = 0; w < W; ++w) out[(2 * P + 2) * W + w] = (float)e.die;
}

// ----------------------------------------------------------------- StochasticDynamicsNetwork4 (314-408)
// LN(x) * (1 + scale(e)) + shift(e) -> dense1 / LN / relu -> dense2 / LN / relu -> 2 ResBlocks -> proj,
// + input skip, min-max (339-360 / 381-406).  out may alias nothing; x_in [B][256], emb [B][64].
void film_trunk(const Net& net, const std::string& pre, int rb0, const float* x_in, const float* emb, int B, float* out,
                Scratch& s) {
  const std::string d = "dynamics/";
  std::vector<float> x(x_in, x_in + (size_t)B * kLat), sc((size_t)B * kLat), sh((size_t)B * kLat), y((size_t)B * kLat);
  layer_norm(net, d + pre + "_input_ln", x.data(), B, kLat, false);
  dense(net, d + pre + "_film_scale", emb, B, 64, kLat, sc.data());
  dense(net, d + pre + "_film_shift", emb, B, 64, kLat, sh.data());
  for (size_t i = 0; i < x.size(); ++i) x[i] = x[i] * (1.0f + sc[i]) + sh[i];
  dense(net, d + pre + "_dense1", x.data(), B, kLat, kLat, y.data());
  layer_norm(net, d + pre + "_ln1", y.data(), B, kLat, true);
  dense(net, d + pre + "_dense2", y.data(), B, kLat, kLat, x.data());
  layer_norm(net, d + pre + "_ln2", x.data(), B, kLat, true);
  for (int r = rb0; r < rb0 + 2; ++r) resblock(net, d + "ResBlock_" + std::to_string(r), x.data(), B, s.t1, s.t2);
  dense(net, d + pre + "_proj", x.data(), B, kLat, kLat, y.data());
  for (size_t i = 0; i < y.size(); ++i) out[i] = x_in[i] + y[i];
  minmax(out, B, kLat);
}

// decision_recurrent_fn (414-432): action_dynamics (329-371) + prediction of the afterstate
void decision(const Net& net, const int* action, const float* emb, int B, float* chance_logits, float* after_value,
              float* after, float* reward, float* discount, Scratch& s) {
  const std::string d = "dynamics/";
  std::vector<float> oh((size_t)B * kAc, 0.f), e((size_t)B * 64);
  for (int b = 0; b < B; ++b)
    if (action[b] >= 0 && action[b] < kAc) oh[(size_t)b * kAc + action[b]] = 1.f;
  dense(net, d + "act_embed", oh.data(), B, kAc, 64, e.data());
  relu_(e.data(), e.size());
  film_trunk(net, "act", 0, emb, e.data(), B, after, s);
  std::vector<float> ri((size_t)B * (kLat + kAc)), h((size_t)B * 64), l3((size_t)B * 3), dd((size_t)B * 32);
  for (int b = 0; b < B; ++b) {
    std::memcpy(&ri[(size_t)b * (kLat + kAc)], after + (size_t)b * kLat, sizeof(float) * kLat);
    std::memcpy(&ri[(size_t)b * (kLat + kAc) + kLat], &oh[(size_t)b * kAc], sizeof(float) * kAc);
  }
  dense(net, d + "reward_dense", ri.data(), B, kLat + kAc, 64, h.data());
  relu_(h.data(), h.size());
  dense(net, d + "reward_head", h.data(), B, 64, 3, l3.data());
  for (int b = 0; b < B; ++b) reward[b] = support3(&l3[(size_t)b * 3]);
  dense(net, d + "discount_dense", emb, B, kLat, 32, dd.data());
  layer_norm(net, d + "discount_ln", dd.data(), B, 32, true);
  dense(net, d + "discount_head", dd.data(), B, 32, 3, l3.data());
  for (int b = 0; b < B; ++b) discount[b] = support3(&l3[(size_t)b * 3]);
  dense(net, d + "chance_head", after, B, kLat, kCh, chance_logits);
  std::vector<float> lg((size_t)B * kAc);
  prediction(net, after, B, lg.data(), after_value, s);
}

// chance_recurrent_fn (434-451): chance_dynamics (373-408) + prediction of the next state
void chance(const Net& net, const int* outcome, const float* after, int B, float* logits, float* value, float* nxt,
            Scratch& s) {
  std::vector<float> oh((size_t)B * kCh, 0.f), e((size_t)B * 64);
  for (int b = 0; b < B; ++b)
    if (outcome[b] >= 0 && outcome[b] < kCh) oh[(size_t)b * kCh + outcome[b]] = 1.f;
  dense(net, "dynamics/chance_embed", oh.data(), B, kCh, 64, e.data());
  relu_(e.data(), e.size());
  film_trunk(net, "chance", 2, after, e.data(), B, nxt, s);
  prediction(net, nxt, B, logits, value, s);
}

// ------------------------------------------------------------------ mctx stochastic_muzero_policy (App. B.3)
struct STree {
  int N;
  std::vector<int> visits, parent, afp, c_index, c_visits;
  std::vector<uint8_t> is_dec;
  std::vector<float> raw, value, c_prior, c_value, c_reward, c_disc, emb, info;
  void init(int n) {
    N = n;
    visits.assign(n, 0);
    parent.assign(n, -1);
    afp.assign(n, -1);
    is_dec.assign(n, 0);
    raw.assign(n, 0.f);
    value.assign(n, 0.f);
    info.assign((size_t)n * 2, 0.f);
    c_index.assign((size_t)n * kAp, -1);
    c_visits.assign((size_t)n * kAp, 0);
    c_prior.assign((size_t)n * kAp, 0.f);
    c_value.assign((size_t)n * kAp, 0.f);
    c_reward.assign((size_t)n * kAp, 0.f);
    c_disc.assign((size_t)n * kAp, 0.f);
    emb.assign((size_t)n * kLat, 0.f);
  }
  void update(int node, const float* prior, float v, bool dec, const float* e, float r, float d) {
    std::memcpy(&c_prior[(size_t)node * kAp], prior, sizeof(float) * kAp);
    raw[node] = v;
    value[node] = v;
    visits[node] += 1;
    is_dec[node] = dec;
    std::memcpy(&emb[(size_t)node * kLat], e, sizeof(float) * kLat);
    info[(size_t)node * 2] = r;
    info[(size_t)node * 2 + 1] = d;
  }
};

// csrc/stochastic.hip:tiebreak_uniform (oracle/mctx_stochastic.py)
inline float tiebreak_uniform(uint64_t seed, int gid, int turn, int sim, int depth, int a) {
  const uint64_t h = mix64(seed ^ mix64(((uint64_t)(uint32_t)gid << 32) | (uint32_t)turn) ^
                           mix64(((uint64_t)(sim & 0xFFFF) << 16) | (uint64_t)(depth & 0xFFFF)) ^
                           ((uint64_t)(a + 1) * 0x9E6C63D0676A9A99ull));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

// qtransform_by_parent_and_siblings (eps 1e-8)
void qtransform(const STree& t, int n, float* out) {
  const size_t o = (size_t)n * kAp;
  const float nv = t.value[n];
  float q[kAp], lo = nv, hi = nv;
  for (int a = 0; a < kAp; ++a) {
    q[a] = t.c_reward[o + a] + t.c_disc[o + a] * t.c_value[o + a];
    const float safe = t.c_visits[o + a] > 0 ? q[a] : nv;
    lo = std::min(lo, safe);
    hi = std::max(hi, safe);
  }
  const float den = std::max(hi - lo, 1e-8f);
  for (int a = 0; a < kAp; ++a) out[a] = ((t.c_visits[o + a] > 0 ? q[a] : lo) - lo) / den;
}

// muzero_action_selection (pb_c 1.25 / 19652, 1e-7 tie-break), the root mask at depth 0
int decision_select(const STree& t, int n, int depth, const bool* root_invalid, uint64_t seed, int gid, int turn,
                    int sim) {
  const size_t o = (size_t)n * kAp;
  const float nvis = (float)t.visits[n];
  const float pb_c = 1.25f + std::log((nvis + 19652.0f + 1.0f) / 19652.0f);
  float probs[kAp], cq[kAp], score[kAp];
  softmax(&t.c_prior[o], probs, kAp);
  qtransform(t, n, cq);
  const float sq = std::sqrt(nvis);
  for (int a = 0; a < kAp; ++a) {
    const float policy = sq * pb_c * probs[a] / (float)(t.c_visits[o + a] + 1);
    score[a] = cq[a] + policy + 1e-7f * tiebreak_uniform(seed, gid, turn, sim, depth, a);
    if (depth == 0 && root_invalid[a]) score[a] = -kInf;
  }
  return argmax(score, kAp);
}

int chance_select(const STree& t, int n) {
  const size_t o = (size_t)n * kAp;
  float p[kCh], x[kCh];
  softmax(&t.c_prior[o + kAc], p, kCh);
  for (int c = 0; c < kCh; ++c) x[c] = p[c] / (float)(t.c_visits[o + kAc + c] + 1);
  return argmax(x, kCh) + kAc;
}

struct SSearch {
  int S, D;
  float temperature, dirichlet_fraction;
};

// Dirichlet(alpha) noise over the kAc root actions from the counter hash (Marsaglia-Tsang gamma; alpha < 1 via
// the U^(1/alpha) boost): the CPU baseline's stand-in for the reference's jax.random.dirichlet
void dirichlet_noise(uint64_t seed, int gid, int turn, float alpha, float* out) {
  uint64_t ctr = mix64(seed ^ 0xD121C4E7ull ^ mix64(((uint64_t)(uint32_t)gid << 32) | (uint32_t)turn));
  auto uni = [&]() {
    ctr = mix64(ctr);
    return std::max((float)(ctr >> 40) * (1.0f / 16777216.0f), 1e-7f);
  };
  float sum = 0.f;
  for (int a = 0; a < kAc; ++a) {
    const float d = alpha + 1.0f - 1.0f / 3.0f, c = 1.0f / std::sqrt(9.0f * d);
    float g;
    while (true) {
      const float u1 = uni(), u2 = uni();
      const float z = std::sqrt(-2.0f * std::log(u1)) * std::cos(6.2831853f * u2);
      const float v = (1.0f + c * z) * (1.0f + c * z) * (1.0f + c * z);
      if (v <= 0.f) continue;
      if (std::log(uni()) < 0.5f * z * z + d - d * v + d * std::log(v)) {
        g = d * v;
        break;
      }
    }
    g *= std::pow(uni(), 1.0f / alpha);
    out[a] = g;
    sum += g;
  }
  for (int a = 0; a < kAc; ++a) out[a] = sum > 0.f ? out[a] / sum : 1.0f / kAc;
}

// One batched stochastic_muzero_policy over `B` games (root inference outputs given).  gids / turn / seed feed
// the tie-break and (with dirichlet_fraction > 0) the Dirichlet draws; gumbel [B][kAc] the final categorical.
void stochastic_search(const Net& net, const SSearch& sr, int B, const float* logits, const float* rvalue,
                       const float* remb, const bool* invalid, const float* gumbel, const int* gids, int turn,
                       uint64_t seed, std::vector<STree>& trees, int* action_out, float* weights_out, float* value_out,
                       Scratch& s) {
  const int S = sr.S;
  std::vector<uint8_t> root_invalid((size_t)B * kAp);
  for (int b = 0; b < B; ++b) {
    STree& t = trees[b];
    t.init(S + 1);
    float probs[kAc], noise[kAc] = {0.f, 0.f, 0.f, 0.f}, pr[kAp];
    softmax(logits + (size_t)b * kAc, probs, kAc);
    if (sr.dirichlet_fraction > 0.f) dirichlet_noise(seed, gids[b], turn, 0.3f, noise);
    float m = -kInf;
    for (int a = 0; a < kAc; ++a) {
      const float noisy = (1.0f - sr.dirichlet_fraction) * probs[a] + sr.dirichlet_fraction * noise[a];
      pr[a] = std::log(std::max(noisy, kTiny));
      m = std::max(m, pr[a]);
    }
    for (int a = 0; a < kAc; ++a) {
      pr[a] = invalid[(size_t)b * kAc + a] ? kFMin : pr[a] - m;
      root_invalid[(size_t)b * kAp + a] = invalid[(size_t)b * kAc + a];
    }
    for (int c = 0; c < kCh; ++c) {
      pr[kAc + c] = -kInf;
      root_invalid[(size_t)b * kAp + kAc + c] = 1;
    }
    t.update(0, pr, rvalue[b], true, remb + (size_t)b * kLat, 0.f, 0.f);
  }
  std::vector<int> parent(B), act(B), nxt(B), dec, cha, da, ca;
  std::vector<float> pe, cl, av, af, rw, ds, lg, vv, ns;
  for (int sim = 0; sim < S; ++sim) {
    dec.clear();
    cha.clear();
    for (int b = 0; b < B; ++b) {   // simulate
      const STree& t = trees[b];
      bool rinv[kAp];
      for (int a = 0; a < kAp; ++a) rinv[a] = root_invalid[(size_t)b * kAp + a];
      int node = 0, depth = 0, a = 0;
      while (true) {
        a = t.is_dec[node] ? decision_select(t, node, depth, rinv, seed, gids[b], turn, sim) : chance_select(t, node);
        const int child = t.c_index[(size_t)node * kAp + a];
        ++depth;
        if (child == -1 || depth >= sr.D) break;
        node = child;
      }
      parent[b] = node;
      act[b] = a;
      const int c = t.c_index[(size_t)node * kAp + a];
      nxt[b] = c == -1 ? sim + 1 : c;
      (t.is_dec[node] ? dec : cha).push_back(b);
    }
    if (!dec.empty()) {   // decision expansions: afterstates
      const int n = (int)dec.size();
      pe.resize((size_t)n * kLat);
      da.resize(n);
      for (int j = 0; j < n; ++j) {
        da[j] = act[dec[j]];
        std::memcpy(&pe[(size_t)j * kLat], &trees[dec[j]].emb[(size_t)parent[dec[j]] * kLat], sizeof(float) * kLat);
      }
      cl.resize((size_t)n * kCh);
      av.resize(n);
      af.resize((size_t)n * kLat);
      rw.resize(n);
      ds.resize(n);
      decision(net, da.data(), pe.data(), n, cl.data(), av.data(), af.data(), rw.data(), ds.data(), s);
      for (int j = 0; j < n; ++j) {
        const int b = dec[j];
        STree& t = trees[b];
        const int p = parent[b], a = act[b], nn = nxt[b];
        float prior[kAp];
        for (int q = 0; q < kAc; ++q) prior[q] = -kInf;
        for (int c = 0; c < kCh; ++c) prior[kAc + c] = cl[(size_t)j * kCh + c];
        t.update(nn, prior, av[j], false, &af[(size_t)j * kLat], rw[j], ds[j]);
        const size_t e = (size_t)p * kAp + a;
        t.c_reward[e] = 0.f;
        t.c_disc[e] = 1.f;
        t.c_index[e] = nn;
        t.parent[nn] = p;
        t.afp[nn] = a;
      }
    }
    if (!cha.empty()) {   // chance expansions: next states
      const int n = (int)cha.size();
      pe.resize((size_t)n * kLat);
      ca.resize(n);
      for (int j = 0; j < n; ++j) {
        ca[j] = act[cha[j]] - kAc;
        std::memcpy(&pe[(size_t)j * kLat], &trees[cha[j]].emb[(size_t)parent[cha[j]] * kLat], sizeof(float) * kLat);
      }
      lg.resize((size_t)n * kAc);
      vv.resize(n);
      ns.resize((size_t)n * kLat);
      chance(net, ca.data(), pe.data(), n, lg.data(), vv.data(), ns.data(), s);
      for (int j = 0; j < n; ++j) {
        const int b = cha[j];
        STree& t = trees[b];
        const int p = parent[b], a = act[b], nn = nxt[b];
        float prior[kAp];
        for (int q = 0; q < kAc; ++q) prior[q] = lg[(size_t)j * kAc + q];
        for (int c = 0; c < kCh; ++c) prior[kAc + c] = -kInf;
        t.update(nn, prior, vv[j], true, &ns[(size_t)j * kLat], 0.f, 0.f);
        const size_t e = (size_t)p * kAp + a;
        t.c_reward[e] = t.info[(size_t)p * 2];
        t.c_disc[e] = t.info[(size_t)p * 2 + 1];
        t.c_index[e] = nn;
        t.parent[nn] = p;
        t.afp[nn] = a;
      }
    }
    for (int b = 0; b < B; ++b) {   // search.py backward
      STree& t = trees[b];
      int idx = nxt[b];
      float leaf = t.value[idx];
      while (idx != 0) {
        const int pr = t.parent[idx], pa = t.afp[idx];
        const int cnt = t.visits[pr];
        const size_t e = (size_t)pr * kAp + pa;
        leaf = t.c_reward[e] + t.c_disc[e] * leaf;
        t.value[pr] = (t.value[pr] * (float)cnt + leaf) / ((float)cnt + 1.0f);
        t.visits[pr] = cnt + 1;
        t.c_value[e] = t.value[idx];
        t.c_visits[e] += 1;
        idx = pr;
      }
    }
  }
  for (int b = 0; b < B; ++b) {   // _mask_tree + summary + _apply_temperature + categorical
    const STree& t = trees[b];
    float w[kAc], lw[kAc], tot = 0.f;
    for (int a = 0; a < kAc; ++a) tot += (float)t.c_visits[a];
    for (int a = 0; a < kAc; ++a) w[a] = tot > 0.f ? (float)t.c_visits[a] / std::max(tot, 1.0f) : 1.0f / kAc;
    float m = -kInf;
    for (int a = 0; a < kAc; ++a) {
      lw[a] = std::log(w[a]);
      m = std::max(m, lw[a]);
    }
    const float temp = std::max(kTiny, sr.temperature);
    float sc[kAc];
    for (int a = 0; a < kAc; ++a) sc[a] = (lw[a] - m) / temp + gumbel[(size_t)b * kAc + a];
    action_out[b] = argmax(sc, kAc);
    std::memcpy(weights_out + (size_t)b * kAc, w, sizeof(w));
    value_out[b] = std::min(std::max(t.value[0], -1.0f), 1.0f);
  }
}

constexpr uint64_t kDieStream = 0xD1CE5EEDF00Dull, kGumbelStream = 0xC2B2AE3D27D4EB4Full;

inline float die_uniform(uint64_t seed, int g, int turn) {   // csrc/selfplay_classic.hip:die_uniform
  const uint64_t h = mix64((seed ^ kDieStream) ^ mix64(((uint64_t)(uint32_t)g << 32) | (uint32_t)turn));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

void gumbel4(uint64_t seed, int gid, int turn, float* out) {   // oracle/selfplay.py:gumbel_noise(A = 4)
  for (int a = 0; a < kAc; ++a) {
    const uint64_t h = mix64(seed ^ mix64(((uint64_t)(uint32_t)gid << 32) | (uint32_t)turn) ^
                             ((uint64_t)(a + 1) * 0xD6E8FEB86659FD93ull));
    float u = (float)(h >> 40) * (1.0f / 16777216.0f);
    u = std::max(u, kTiny);
    out[a] = -std::log(-std::log(u));
  }
}

void throw_die(muzcpu_classic& e, float u) {   // classic_madn.py:230-242 with an explicit uniform
  float p[6];
  dice_probabilities(e, p);
  e.die = choice_from_uniform(p, u);
}

struct CLane {
  muzcpu_classic env;
  int game = -1, t = 0;
};

}  // namespace

extern "C" {

typedef struct {   // optional records of muzcpu_classic_selfplay (game_agent_stochastic.py:180-200), [n][T]
  int32_t* act;
  float* val;
  float* pol;      // [n][T][4]
  float* mask;
  int32_t* dice;
  int32_t* idx;    // [n]
} muzcpu_ctraj;

void* muzcpu_classic_net_create(const char** names, const float** data, const int64_t* sizes, int count,
                                int obs_channels) {
  Net* n = new Net;
  n->C = obs_channels;
  n->A = kAc;
  for (int i = 0; i < count; ++i) n->p[names[i]] = std::vector<float>(data[i], data[i] + sizes[i]);
  return n;
}
void muzcpu_classic_net_destroy(void* n) { delete (Net*)n; }

void muzcpu_classic_reset(muzcpu_classic* e, int P, const int* layout, int distance, int starting_player, int rules) {
  env_reset(*e, P, layout, distance, starting_player, rules);
}
void muzcpu_classic_valid_action(const muzcpu_classic* e, uint8_t* out4) {
  bool va[4];
  valid_action(*e, va);
  for (int i = 0; i < 4; ++i) out4[i] = va[i];
}
void muzcpu_classic_step(muzcpu_classic* e, int pin, int* reward, int* done) { env_step(*e, pin, *reward, *done); }
void muzcpu_classic_no_step(muzcpu_classic* e) { no_step(*e); }
void muzcpu_classic_encode(const muzcpu_classic* e, float* out) { encode_board(*e, out); }
int muzcpu_classic_soft_locked(const muzcpu_classic* e) { return is_soft_locked(*e); }
void muzcpu_classic_dice_probs(const muzcpu_classic* e, float* out6) { dice_probabilities(*e, out6); }
void muzcpu_classic_throw_die(muzcpu_classic* e, float u) { throw_die(*e, u); }

void muzcpu_classic_root(void* net, const float* obs, int B, float* logits, float* value, float* emb) {
  Scratch s;
  representation(*(Net*)net, obs, B, emb, s);
  prediction(*(Net*)net, emb, B, logits, value, s);
}
void muzcpu_classic_decision(void* net, const int* action, const float* emb, int B, float* chance_logits,
                             float* after_value, float* after, float* reward, float* discount) {
  Scratch s;
  decision(*(Net*)net, action, emb, B, chance_logits, after_value, after, reward, discount, s);
}
void muzcpu_classic_chance(void* net, const int* outcome, const float* after, int B, float* logits, float* value,
                           float* nxt) {
  Scratch s;
  chance(*(Net*)net, outcome, after, B, logits, value, nxt, s);
}

// play_batch_of_games_stochastic (oracle/selfplay.py; game_agent_stochastic.py:52-218) of n games on one thread:
// returns the number of batched turns; records into tr (if non-null).
int muzcpu_classic_selfplay(void* netp, int P, int rules, int n, int S, int D, int T, float temp, uint64_t seed,
                            float dirichlet_fraction, const muzcpu_ctraj* tr) {
  const Net& net = *(Net*)netp;
  const int C = 2 * P + 3;
  const int layout[4] = {1, 1, 1, 1};
  std::vector<muzcpu_classic> envs(n);
  for (auto& e : envs) env_reset(e, P, layout, 10, 0, rules);
  SSearch sr{S, D, temp, dirichlet_fraction};
  Scratch s;
  std::vector<STree> trees(n);
  std::vector<int> idx(n, 0);
  int step = 0;
  while (step < T) {
    std::vector<int> search, nomove;
    std::vector<uint8_t> inv;
    bool any_active = false;
    for (int i = 0; i < n; ++i) {
      if (envs[i].done) continue;
      any_active = true;
      throw_die(envs[i], die_uniform(seed, i, step));
      bool va[4];
      valid_action(envs[i], va);
      if (va[0] || va[1] || va[2] || va[3]) {
        search.push_back(i);
        for (int k = 0; k < 4; ++k) inv.push_back(!va[k]);
      } else {
        nomove.push_back(i);
      }
    }
    if (!any_active) break;
    const int B = (int)search.size();
    if (B) {
      std::vector<float> obs((size_t)B * C * kCells), lg((size_t)B * kAc), v(B), e((size_t)B * kLat),
          gum((size_t)B * kAc), w((size_t)B * kAc), rv(B);
      std::vector<int> act(B);
      std::unique_ptr<bool[]> ib(new bool[inv.size()]);
      for (size_t q = 0; q < inv.size(); ++q) ib[q] = inv[q];
      for (int k = 0; k < B; ++k) {
        encode_board(envs[search[k]], &obs[(size_t)k * C * kCells]);
        gumbel4(seed ^ kGumbelStream, search[k], step, &gum[(size_t)k * kAc]);
      }
      representation(net, obs.data(), B, e.data(), s);
      prediction(net, e.data(), B, lg.data(), v.data(), s);
      stochastic_search(net, sr, B, lg.data(), v.data(), e.data(), ib.get(), gum.data(), search.data(), step, seed,
                        trees, act.data(), w.data(), rv.data(), s);
      for (int k = 0; k < B; ++k) {
        const int i = search[k], t = idx[i];
        if (tr) {
          tr->act[(size_t)i * T + t] = act[k];
          tr->val[(size_t)i * T + t] = rv[k];
          std::memcpy(&tr->pol[((size_t)i * T + t) * kAc], &w[(size_t)k * kAc], sizeof(float) * kAc);
          tr->mask[(size_t)i * T + t] = 1.f;
          tr->dice[(size_t)i * T + t] = envs[i].die;
        }
        int r, d;
        env_step(envs[i], act[k], r, d);
        idx[i] = t + 1;
      }
    }
    for (int i : nomove) {
      const int t = idx[i];
      if (tr) {
        tr->act[(size_t)i * T + t] = -1;
        tr->mask[(size_t)i * T + t] = 0.f;
        tr->dice[(size_t)i * T + t] = envs[i].die;
      }
      no_step(envs[i]);
      idx[i] = t + 1;
    }
    ++step;
  }
  if (tr)
    for (int i = 0; i < n; ++i) tr->idx[i] = idx[i];
  return step;
}

// The config (c) CPU baseline: `threads` OpenMP threads, each playing `lanes` concurrent classic games (die
// thrown per turn, Stochastic MuZero search with the reference's Dirichlet root noise, a lane refilled with the
// next game when its game ends or reaches max_steps) until `seconds` have passed.  Returns env-steps.
int64_t muzcpu_classic_bench(void* netp, int P, int rules, int lanes, int S, int D, int T, float temp, uint64_t seed,
                             float dirichlet_fraction, int threads, double seconds, int64_t* searches_out,
                             int64_t* games_out, double* elapsed_out) {
  const Net& net = *(Net*)netp;
  const int C = 2 * P + 3;
  const int layout[4] = {1, 1, 1, 1};
  std::atomic<int> next_game{0};
  std::atomic<int64_t> steps{0}, searches{0}, games{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
#pragma omp parallel num_threads(threads)
  {
    SSearch sr{S, D, temp, dirichlet_fraction};
    Scratch s;
    std::vector<STree> trees(lanes);
    std::vector<CLane> L(lanes);
    auto fresh = [&](CLane& l) {
      env_reset(l.env, P, layout, 10, 0, rules);
      l.game = next_game.fetch_add(1);
      l.t = 0;
    };
    for (auto& l : L) fresh(l);
    int64_t my_steps = 0, my_searches = 0, my_games = 0;
    std::vector<float> obs((size_t)lanes * C * kCells), lg((size_t)lanes * kAc), v(lanes), e((size_t)lanes * kLat),
        gum((size_t)lanes * kAc), w((size_t)lanes * kAc), rv(lanes);
    std::vector<int> act(lanes), search, gids(lanes);
    std::unique_ptr<bool[]> inv(new bool[(size_t)lanes * kAc]);
    int turn = 0;
    while (elapsed() < seconds) {
      search.clear();
      for (int i = 0; i < lanes; ++i) {
        CLane& l = L[i];
        throw_die(l.env, die_uniform(seed, l.game, l.t));
        bool va[4];
        valid_action(l.env, va);
        if (va[0] || va[1] || va[2] || va[3]) {
          const int k = (int)search.size();
          for (int q = 0; q < kAc; ++q) inv[(size_t)k * kAc + q] = !va[q];
          encode_board(l.env, &obs[(size_t)k * C * kCells]);
          gumbel4(seed ^ kGumbelStream, l.game, l.t, &gum[(size_t)k * kAc]);
          gids[k] = l.game;
          search.push_back(i);
        } else {
          no_step(l.env);
        }
      }
      const int B = (int)search.size();
      if (B) {
        representation(net, obs.data(), B, e.data(), s);
        prediction(net, e.data(), B, lg.data(), v.data(), s);
        stochastic_search(net, sr, B, lg.data(), v.data(), e.data(), inv.get(), gum.data(), gids.data(), turn, seed,
                          trees, act.data(), w.data(), rv.data(), s);
        for (int k = 0; k < B; ++k) {
          int r, d;
          env_step(L[search[k]].env, act[k], r, d);
        }
      }
      my_searches += B;
      my_steps += lanes;
      ++turn;
      for (auto& l : L) {
        l.t += 1;
        if (l.env.done || l.t >= T) {
          ++my_games;
          fresh(l);
        }
      }
    }
    steps += my_steps;
    searches += my_searches;
    games += my_games;
  }
  if (searches_out) *searches_out = searches.load();
  if (games_out) *games_out = games.load();
  if (elapsed_out) *elapsed_out = elapsed();
  return steps.load();
}

}  // extern "C"
