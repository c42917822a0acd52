// CPU restatement of det-MADN MuZero self-play in C++ with OpenMP over games.
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY: this is the "port" CPU baseline of SURVEY.md §8(d) -- the
// reference algorithm (MADN/deterministic_madn.py env, MuZero_det_MADN/muzero_deterministic_madn.py
// networks, mctx 0.0.6 gumbel_muzero_policy, MuZero_det_MADN/game_agent.py:50-183 self-play loop) restated
// as plain fp32 C++ so bench.py can time it on the GPU box's host cores beside the HIP engine.  It follows
// the NumPy oracle line by line (oracle/detmadn.py, oracle/nets.py, oracle/mctx_gumbel.py,
// oracle/selfplay.py) and is checked against it by tests/test_cpu_baseline.py (golden step vectors, network
// outputs, a short self-play trace).  Only tests/, smoke() and bench.py's cpu_baseline leg load it; the
// product path never does.
//
// Parallelism mirrors the reference's vmap over games: each OpenMP thread owns a batch of game lanes,
// searches them together (batched network calls, per-game trees) and refills a lane with the next game
// when its game ends.
#include "cpu_search.hpp"

extern "C" {

// one deterministic_MADN state (deterministic_madn.py:24-40); pins / action_set / goal rows = players
typedef struct {
  int8_t board[kCells];
  int8_t pins[16];
  int8_t action_set[24];
  int8_t start[4], target[4], goal[16];
  int32_t current_player, reward, done, num_players, board_size, total, rules;
} muzcpu_det;

}  // extern "C"

namespace {

inline bool has(const muzcpu_det& e, uint32_t f) { return (e.rules & f) != 0; }

void set_pins_on_board(int8_t* board, const int8_t* pins, int P, int total) {   // 259-271
  for (int i = 0; i < total; ++i) board[i] = -1;
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < 4; ++k) {
      const int pos = pins[p * 4 + k];
      if (pos >= 0 && pos < total) board[pos] = (int8_t)p;
    }
}

bool is_player_done(const muzcpu_det& e, const int8_t* board, int p) {   // 122-137
  if (p >= e.num_players) return false;
  for (int k = 0; k < 4; ++k)
    if (board[e.goal[p * 4 + k]] < 0) return false;
  return true;
}

void get_winner(const muzcpu_det& e, const int8_t* board, bool w[4]) {   // 139-168
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

int sub_player(const muzcpu_det& e) {   // 184 / 310
  const int p = e.current_player;
  return (has(e, R_TEAMS) && is_player_done(e, e.board, p)) ? (p + 2) % 4 : p;
}

// utils/utility_funcs.py:142-184: all(board[goal[ga]] != cp for start < ga < x)
bool goal_path_free(long long start, long long x, const int8_t* goal, const int8_t* board, int cp) {
  for (int ga = 0; ga < 4; ++ga)
    if (start < ga && ga < x && board[goal[ga]] == cp) return false;
  return true;
}

void valid_action(const muzcpu_det& e, bool va[4][6]) {   // 299-393
  const int cp0 = e.current_player, cp = sub_player(e), P = e.num_players, bs = e.board_size;
  const int8_t* board = e.board;
  const int8_t* goal = e.goal + cp * 4;
  const long long target = e.target[cp];
  const long long mt = has(e, R_MUST_TRAVERSE) ? 1 : 0;
  bool pos_[4];
  for (int p = 0; p < P; ++p) pos_[p] = board[e.start[p]] == p;
  const long long dist = bs / 4;
  for (int i = 0; i < 4; ++i) {
    const long long cur = e.pins[cp * 4 + i];
    for (int m = 1; m <= 6; ++m) {
      const long long moved = cur + m;
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
      const bool start_move = m == 6 || (m == 1 && has(e, R_START_ON_1));
      if (cur == -1) res = start_move && (board[e.start[cp]] != cp0);
      va[i][m - 1] = res && e.action_set[cp * 6 + m - 1] > 0;
    }
  }
}

void env_reset(muzcpu_det& e, int P, const int* layout, int distance, int starting_player, int rules) {   // 42-120
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
  for (int i = 0; i < 24; ++i) e.action_set[i] = i < 6 * P ? 4 : 0;
  e.current_player = starting_player;
}

void env_step(muzcpu_det& e, int pin, int move, int& reward_out, int& done_out) {   // 170-257
  const int player_id = e.current_player, cp = sub_player(e);
  bool va[4][6];
  valid_action(e, va);
  const int mi = (int)pymod(move - 1, 6);
  const bool invalid = !va[pin][mi];
  const long long cur = e.pins[cp * 4 + pin];
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
  if (!invalid) pins[cp * 4 + pin] = (int8_t)new_pos;
  int8_t nb[kCells];
  if (invalid) std::memcpy(nb, e.board, kCells);
  else set_pins_on_board(nb, pins, e.num_players, e.total);
  const int cs = e.action_set[cp * 6 + mi];
  int8_t aset[24];
  std::memcpy(aset, e.action_set, 24);
  aset[cp * 6 + mi] = (int8_t)((invalid || cs == 0) ? cs : cs - 1);
  bool empty = true;
  for (int j = 0; j < 6; ++j) empty = empty && aset[cp * 6 + j] == 0;
  if (empty) {   // refill restores the PRE-step set with the current player's row full (quirk, 235-240)
    std::memcpy(aset, e.action_set, 24);
    for (int j = 0; j < 6; ++j) aset[player_id * 6 + j] = 4;
  }
  bool w[4];
  get_winner(e, nb, w);
  const int reward = e.done ? 0 : (invalid ? -1 : (w[cp] ? 1 : 0));
  const bool done = e.done || w[0] || w[1] || w[2] || w[3];
  const int nxt = (done || (has(e, R_BONUS_6) && move == 6)) ? player_id : (player_id + 1) % e.num_players;
  std::memcpy(e.board, nb, kCells);
  std::memcpy(e.pins, pins, 16);
  std::memcpy(e.action_set, aset, 24);
  e.current_player = nxt;
  e.done = done;
  e.reward = reward;
  reward_out = reward;
  done_out = done;
}

void no_step(muzcpu_det& e) {   // 283-297
  for (int j = 0; j < 6; ++j) e.action_set[e.current_player * 6 + j] = 4;
  e.current_player = (e.current_player + 1) % e.num_players;
}

void encode_board(const muzcpu_det& e, float* out) {   // 395-438 -> [8P+2][56]
  const int P = e.num_players, bs = e.board_size, dist = bs / 4, cp = e.current_player, W = e.total;
  int8_t b[kCells];
  for (int i = 0; i < bs; ++i) b[i] = e.board[(i + dist * cp) % bs];
  for (int i = 0; i < 16; ++i) b[bs + i] = e.board[bs + (i + 4 * cp) % 16];
  int rolled[4];
  for (int k = 0; k < P; ++k) rolled[k] = (k + cp) % P;
  const int C = 8 * P + 2;
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
  for (int k = 0; k < P; ++k)
    for (int m = 0; m < 6; ++m)
      for (int w = 0; w < W; ++w) out[(2 * P + 2 + k * 6 + m) * W + w] = (float)e.action_set[rolled[k] * 6 + m];
}


// recurrent_inference_fn (632-661) with DynamicsNetwork4 (391-457)
void recurrent(const Net& net, const int* action, const float* emb, int B, float* reward, float* discount,
               float* logits, float* value, float* nxt, Scratch& s) {
  const std::string d = "dynamics/";
  std::vector<float> oh((size_t)B * kA, 0.f);
  for (int b = 0; b < B; ++b)
    if (action[b] >= 0 && action[b] < kA) oh[(size_t)b * kA + action[b]] = 1.f;
  std::vector<float> e((size_t)B * 64), sc((size_t)B * kLat), shf((size_t)B * kLat);
  dense(net, d + "Dense_0", oh.data(), B, kA, 64, e.data());
  relu_(e.data(), e.size());
  std::vector<float> x(emb, emb + (size_t)B * kLat);
  layer_norm(net, d + "LayerNorm_0", x.data(), B, kLat, false);
  dense(net, d + "Dense_1", e.data(), B, 64, kLat, sc.data());
  dense(net, d + "Dense_2", e.data(), B, 64, kLat, shf.data());
  for (size_t i = 0; i < x.size(); ++i) x[i] = x[i] * (1.0f + sc[i]) + shf[i];
  std::vector<float> y((size_t)B * kLat);
  dense(net, d + "Dense_3", x.data(), B, kLat, kLat, y.data());
  layer_norm(net, d + "LayerNorm_1", y.data(), B, kLat, true);
  dense(net, d + "Dense_4", y.data(), B, kLat, kLat, x.data());
  layer_norm(net, d + "LayerNorm_2", x.data(), B, kLat, true);
  for (int i = 0; i < 2; ++i) resblock(net, d + "ResBlock_" + std::to_string(i), x.data(), B, s.t1, s.t2);
  dense(net, d + "Dense_5", x.data(), B, kLat, kLat, y.data());
  for (size_t i = 0; i < y.size(); ++i) nxt[i] = emb[i] + y[i];
  minmax(nxt, B, kLat);
  std::vector<float> ri((size_t)B * (kLat + kA)), h((size_t)B * 64), l3((size_t)B * 3);
  for (int b = 0; b < B; ++b) {
    std::memcpy(&ri[(size_t)b * (kLat + kA)], nxt + (size_t)b * kLat, sizeof(float) * kLat);
    std::memcpy(&ri[(size_t)b * (kLat + kA) + kLat], &oh[(size_t)b * kA], sizeof(float) * kA);
  }
  dense(net, d + "Dense_6", ri.data(), B, kLat + kA, 64, h.data());
  relu_(h.data(), h.size());
  dense(net, d + "reward_head", h.data(), B, 64, 3, l3.data());
  for (int b = 0; b < B; ++b) reward[b] = support3(&l3[(size_t)b * 3]);
  dense(net, d + "Dense_7", ri.data(), B, kLat + kA, 64, h.data());
  relu_(h.data(), h.size());
  dense(net, d + "discount_head", h.data(), B, 64, 3, l3.data());
  for (int b = 0; b < B; ++b) discount[b] = support3(&l3[(size_t)b * 3]);
  prediction(net, nxt, B, logits, value, s);
}

// the search: oracle/cpu_search.hpp (gumbel_search<24>) driving this file's recurrent inference
struct DetRec {
  const Net& net;
  Scratch& s;
  void operator()(const int* action, const float* emb, int B, float* reward, float* discount, float* logits,
                  float* value, float* nxt) const {
    recurrent(net, action, emb, B, reward, discount, logits, value, nxt, s);
  }
};

struct Lane {
  muzcpu_det env;
  int game = -1, t = 0;
};

}  // namespace

extern "C" {

typedef struct {   // optional trajectory records of muzcpu_selfplay (game_agent.py:158-169), [n][T]
  int32_t* act;
  float* val;
  float* pol;      // [n][T][24]
  float* mask;
  int32_t* idx;    // [n]
} muzcpu_traj;

void* muzcpu_net_create(const char** names, const float** data, const int64_t* sizes, int count, int obs_channels) {
  Net* n = new Net;
  n->C = obs_channels;
  for (int i = 0; i < count; ++i) n->p[names[i]] = std::vector<float>(data[i], data[i] + sizes[i]);
  if (n->w("prediction/Dense_2/bias")) n->A = (int)n->n("prediction/Dense_2/bias");   // 24 det, 806 DOG
  return n;
}
void muzcpu_net_destroy(void* n) { delete (Net*)n; }

void muzcpu_env_reset(muzcpu_det* e, int P, const int* layout, int distance, int starting_player, int rules) {
  env_reset(*e, P, layout, distance, starting_player, rules);
}
void muzcpu_valid_action(const muzcpu_det* e, uint8_t* out24) {
  bool va[4][6];
  valid_action(*e, va);
  for (int i = 0; i < 24; ++i) out24[i] = va[i / 6][i % 6];
}
void muzcpu_env_step(muzcpu_det* e, int pin, int move, int* reward, int* done) { env_step(*e, pin, move, *reward, *done); }
void muzcpu_no_step(muzcpu_det* e) { no_step(*e); }
void muzcpu_encode(const muzcpu_det* e, float* out) { encode_board(*e, out); }

void muzcpu_root(void* net, const float* obs, int B, float* logits, float* value, float* emb) {
  Scratch s;
  representation(*(Net*)net, obs, B, emb, s);
  prediction(*(Net*)net, emb, B, logits, value, s);
}
void muzcpu_recurrent(void* net, const int* action, const float* emb, int B, float* reward, float* discount,
                      float* logits, float* value, float* nxt) {
  Scratch s;
  recurrent(*(Net*)net, action, emb, B, reward, discount, logits, value, nxt, s);
}

// play_batch_of_games (game_agent.py:50-183) of n games on one thread, the oracle's loop exactly: returns the
// number of batched turns; records into tr (if non-null).
int muzcpu_selfplay(void* netp, int P, int rules, int n, int S, int D, int T, float temp, uint64_t seed,
                    const muzcpu_traj* tr) {
  const Net& net = *(Net*)netp;
  const int C = 8 * P + 2;
  const int layout[4] = {1, 1, 1, 1};
  std::vector<muzcpu_det> envs(n);
  for (auto& e : envs) env_reset(e, P, layout, 10, 0, rules);
  Search sr;
  sr.init(S, D);
  Scratch s;
  std::vector<Tree<kA>> trees(n);
  std::vector<int> idx(n, 0);
  int step = 0;
  while (step < T) {
    std::vector<int> search, nomove;
    std::vector<uint8_t> inv;
    for (int i = 0; i < n; ++i) {
      if (envs[i].done) continue;
      bool va[4][6];
      valid_action(envs[i], va);
      bool any = false;
      for (int k = 0; k < 24; ++k) any = any || va[k / 6][k % 6];
      if (any) {
        search.push_back(i);
        for (int k = 0; k < 24; ++k) inv.push_back(!va[k / 6][k % 6]);
      } else {
        nomove.push_back(i);
      }
    }
    if (search.empty() && nomove.empty()) break;
    const int B = (int)search.size();
    if (B) {
      std::vector<float> obs((size_t)B * C * kCells), lg((size_t)B * kA), v(B), e((size_t)B * kLat),
          gum((size_t)B * kA), w((size_t)B * kA), rv(B);
      std::vector<int> act(B);
      for (int k = 0; k < B; ++k) {
        encode_board(envs[search[k]], &obs[(size_t)k * C * kCells]);
        gumbel_noise<kA>(seed, search[k], step, temp, &gum[(size_t)k * kA]);
      }
      representation(net, obs.data(), B, e.data(), s);
      prediction(net, e.data(), B, lg.data(), v.data(), s);
      std::vector<bool> invb(inv.begin(), inv.end());
      std::unique_ptr<bool[]> ib(new bool[invb.size()]);
      for (size_t q = 0; q < invb.size(); ++q) ib[q] = invb[q];
      gumbel_search<kA>(sr, B, lg.data(), v.data(), e.data(), ib.get(), gum.data(), trees, act.data(), w.data(),
                        rv.data(), DetRec{net, s});
      for (int k = 0; k < B; ++k) {
        const int i = search[k], t = idx[i];
        if (tr) {
          tr->act[(size_t)i * T + t] = act[k];
          tr->val[(size_t)i * T + t] = rv[k];
          std::memcpy(&tr->pol[((size_t)i * T + t) * kA], &w[(size_t)k * kA], sizeof(float) * kA);
          tr->mask[(size_t)i * T + t] = 1.f;
        }
        int r, d;
        env_step(envs[i], act[k] / 6, act[k] % 6 + 1, r, d);
        idx[i] = t + 1;
      }
    }
    for (int i : nomove) {
      const int t = idx[i];
      if (tr) {
        tr->act[(size_t)i * T + t] = -1;
        tr->mask[(size_t)i * T + t] = 0.f;
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

// The CPU baseline: `threads` OpenMP threads, each playing `lanes` concurrent games (refilled with the next
// game when one ends or reaches max_steps) until `seconds` have passed.  Returns env-steps (turns of
// unfinished games, game_agent.py:140), and the searches / finished games / elapsed seconds through the
// pointers.
int64_t muzcpu_bench(void* netp, int P, int rules, int lanes, int S, int D, int T, float temp, uint64_t seed,
                     int threads, double seconds, int64_t* searches_out, int64_t* games_out, double* elapsed_out) {
  const Net& net = *(Net*)netp;
  const int C = 8 * P + 2;
  const int layout[4] = {1, 1, 1, 1};
  std::atomic<int> next_game{0};
  std::atomic<int64_t> steps{0}, searches{0}, games{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
#pragma omp parallel num_threads(threads)
  {
    Search sr;
    sr.init(S, D);
    Scratch s;
    std::vector<Tree<kA>> trees(lanes);
    std::vector<Lane> L(lanes);
    auto fresh = [&](Lane& l) {
      env_reset(l.env, P, layout, 10, 0, rules);
      l.game = next_game.fetch_add(1);
      l.t = 0;
    };
    for (auto& l : L) fresh(l);
    int64_t my_steps = 0, my_searches = 0, my_games = 0;
    std::vector<float> obs((size_t)lanes * C * kCells), lg((size_t)lanes * kA), v(lanes), e((size_t)lanes * kLat),
        gum((size_t)lanes * kA), w((size_t)lanes * kA), rv(lanes);
    std::vector<int> act(lanes), search;
    std::unique_ptr<bool[]> inv(new bool[(size_t)lanes * kA]);
    while (elapsed() < seconds) {
      search.clear();
      for (int i = 0; i < lanes; ++i) {
        Lane& l = L[i];
        bool va[4][6];
        valid_action(l.env, va);
        bool any = false;
        for (int k = 0; k < 24; ++k) any = any || va[k / 6][k % 6];
        if (any) {
          const int k = (int)search.size();
          for (int q = 0; q < 24; ++q) inv[(size_t)k * kA + q] = !va[q / 6][q % 6];
          encode_board(l.env, &obs[(size_t)k * C * kCells]);
          gumbel_noise<kA>(seed, l.game, l.t, temp, &gum[(size_t)k * kA]);
          search.push_back(i);
        } else {
          no_step(l.env);
        }
      }
      const int B = (int)search.size();
      if (B) {
        representation(net, obs.data(), B, e.data(), s);
        prediction(net, e.data(), B, lg.data(), v.data(), s);
        gumbel_search<kA>(sr, B, lg.data(), v.data(), e.data(), inv.get(), gum.data(), trees, act.data(), w.data(),
                          rv.data(), DetRec{net, s});
        for (int k = 0; k < B; ++k) {
          int r, d;
          env_step(L[search[k]].env, act[k] / 6, act[k] % 6 + 1, r, d);
        }
      }
      my_searches += B;
      my_steps += lanes;
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

// The env-only CPU baseline (SURVEY §8(d)(b')): `threads` threads each advance `lanes` games by rounds of
// uniform random legal play (valid_action -> k-th legal action -> env_step / no_step -> reset of finished
// games -> encode_board) for `seconds`; returns env-steps.
int64_t muzcpu_env_bench(int P, int rules, int lanes, uint64_t seed, int threads, double seconds, double* elapsed_out) {
  const int layout[4] = {1, 1, 1, 1};
  const int C = 8 * P + 2;
  std::atomic<int64_t> steps{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
#pragma omp parallel num_threads(threads)
  {
    const int tid = omp_get_thread_num();
    std::vector<muzcpu_det> envs(lanes);
    for (auto& e : envs) env_reset(e, P, layout, 10, 0, rules);
    std::vector<float> obs((size_t)C * kCells);
    int64_t mine = 0;
    for (int turn = 0; elapsed() < seconds; ++turn) {
      for (int i = 0; i < lanes; ++i) {
        muzcpu_det& e = envs[i];
        bool va[4][6];
        valid_action(e, va);
        int legal[24], cnt = 0;
        for (int k = 0; k < 24; ++k)
          if (va[k / 6][k % 6]) legal[cnt++] = k;
        if (cnt == 0) {
          no_step(e);
        } else {
          const uint64_t h = mix64((seed ^ 0xD37A11D0ull) ^ mix64(((uint64_t)(uint32_t)(tid * lanes + i) << 32) | (uint32_t)turn));
          const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
          const int k = std::min((int)(u * (float)cnt), cnt - 1);
          int r, d;
          env_step(e, legal[k] / 6, legal[k] % 6 + 1, r, d);
        }
        if (e.done) env_reset(e, P, layout, 10, 0, rules);
        encode_board(e, obs.data());
      }
      mine += lanes;
    }
    steps += mine;
  }
  if (elapsed_out) *elapsed_out = elapsed();
  return steps.load();
}

}  // extern "C"
