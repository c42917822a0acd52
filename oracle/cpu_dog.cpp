// CPU restatement of the DOG environment and its random-legal-policy play in C++ with OpenMP over games.
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY: the "port" CPU baseline of SURVEY.md §8(d) for config (d) -- the
// reference environment (DOG/dog.py:83-1131 + utils/utility_funcs.py:4-319; the reference has no DOG network,
// so config (d) plays the uniform random legal policy) restated as plain C++ so bench.py can time
// it on the GPU box's host cores beside k_dog_play.  It follows the NumPy oracle (oracle/dog.py) function by
// function -- JAX's clamped gathers / dropped out-of-range scatters, floor division, team substitution and the
// swap-phase quirks included -- with the engine's counter-RNG deal keys and action choice
// (oracle/dog.py:engine_shuffle_keys / engine_random_action), and is checked against it by
// tests/test_cpu_baseline_dog.py (the reference's golden step vectors, lockstep random play through deals and
// restarts).  Only tests/ and bench.py's cpu_baseline leg load it; the product path never does.
#include "cpu_search.hpp"

namespace {

constexpr int kNC = 14;            // cards: joker, swap(1), 2..13
constexpr int kMaxCards = 120;
constexpr int kMaxHand = 6;
constexpr int kPlay = 792;         // get_play_action_size: 2 * (4 * (12 + 1 + 56) + 120)
constexpr int kHalf = kPlay / 2;   // 396
constexpr int kSwapA = 4 * kCells; // 224
constexpr int kActions = kPlay + kNC;
constexpr int kNormal[12] = {1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13};
constexpr uint64_t kDealStream = 0xDEA1C0DE5EEDull, kActionStream = 0x52A4D0DA11ull;

int g_dists[120][4];               // all_pin_distributions(7) (utils/utility_funcs.py:4-21), lex over (a0, a1, a2)
struct DistInit {
  DistInit() {
    int n = 0;
    for (int a = 0; a <= 7; ++a)
      for (int b = 0; b <= 7; ++b)
        for (int c = 0; c <= 7; ++c) {
          const int d = 7 - a - b - c;
          if (d >= 0) {
            g_dists[n][0] = a, g_dists[n][1] = b, g_dists[n][2] = c, g_dists[n][3] = d;
            ++n;
          }
        }
  }
} g_dist_init;

}  // namespace

extern "C" {

// one DOG state (dog.py:31-56); pins / goal / hands rows = players.  `deal` counts distribute_cards calls and,
// with (seed, game), selects the deal's shuffle keys (it replaces jax's key).
typedef struct {
  int8_t board[kCells];
  int8_t deck[kNC];
  int8_t hands[4 * kNC];
  int8_t swap_choices[4];
  int32_t pins[16];
  int32_t start[4], target[4], goal[16];
  int32_t current_player, reward, done, num_players, round_starter, phase, hand_size, num_cards, board_size, total,
      rules, deal, game;
  uint64_t seed;
} muzcpu_dog;

}  // extern "C"

namespace {

inline bool has(const muzcpu_dog& e, uint32_t f) { return (e.rules & f) != 0; }
inline int si(long long i, long long n) { if (i < 0) i += n; return (i >= 0 && i < n) ? (int)i : -1; }   // scatter
inline float u24(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }
inline uint64_t game_key(uint64_t seed, int g, int turn) {
  return seed ^ mix64(((uint64_t)(uint32_t)g << 32) | (uint32_t)turn);
}

void set_pins_on_board(int8_t* out, const int32_t* pins, int P, int total) {
  for (int i = 0; i < total; ++i) out[i] = -1;
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < 4; ++k) {
      const int pos = pins[p * 4 + k];
      if (pos >= 0 && pos < total) out[pos] = (int8_t)p;
    }
}

bool is_player_done(const muzcpu_dog& e, const int8_t* board, int p) {
  if (p >= e.num_players) return false;
  for (int k = 0; k < 4; ++k)
    if (board[e.goal[p * 4 + k]] < 0) return false;
  return true;
}

void get_winner(const muzcpu_dog& e, const int8_t* board, bool w[4]) {
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

int sub_player(const muzcpu_dog& e) {
  const int p = e.current_player;
  return (has(e, R_TEAMS) && is_player_done(e, e.board, p)) ? (p + 2) % 4 : p;
}

bool check_goal_path(long long start, long long x, const int32_t* goal, const int8_t* board, int cp) {
  for (int ga = 0; ga < 4; ++ga)
    if (start < ga && ga < x && board[goal[ga]] == cp) return false;
  return true;
}

bool in_goal(long long v, const int32_t* goal) { return v == goal[0] || v == goal[1] || v == goal[2] || v == goal[3]; }

inline int sgn(long long v) { return (v > 0) - (v < 0); }

// utils/utility_funcs.py:186-234
void relative_order_preserved(const long long* old, const long long* nw, long long bs, bool out[4]) {
  for (int i = 0; i < 4; ++i) {
    bool ok = true;
    for (int j = 0; j < 4; ++j)
      if (old[i] >= bs && old[j] >= bs && sgn(old[i] - old[j]) != sgn(nw[i] - nw[j])) ok = false;
    out[i] = old[i] < bs || ok;
  }
}

// ------------------------------------------------------------------------------------------- deals
// distribute_cards (dog.py:201-298) with the engine's counter-RNG keys (oracle/dog.py:engine_shuffle_keys)
void distribute_cards(muzcpu_dog& e) {
  const int P = e.num_players, nct = e.num_cards, q = e.hand_size, dummy = nct;
  int8_t deck[kNC];
  std::memcpy(deck, e.deck, kNC);
  long long sum = 0;
  for (int c = 0; c < nct; ++c) sum += deck[c];
  if (sum < (long long)q * P) {   // reset_deck (dog.py:188-191): row 0 = 6 + 2 * (joker enabled)
    for (int c = 0; c < nct; ++c) deck[c] = 8;
    deck[0] = 8;
    sum = 0;
    for (int c = 0; c < nct; ++c) sum += deck[c];
  }
  int pool[kMaxCards];
  int n = 0;
  for (int c = 0; c < nct; ++c)
    for (int k = 0; k < deck[c] && n < kMaxCards; ++k) pool[n++] = c;
  while (n < kMaxCards) pool[n++] = dummy;
  const uint64_t base = game_key(e.seed ^ kDealStream, e.game, e.deal);
  float prio[kMaxCards];
  int order[kMaxCards];
  for (int k = 0; k < kMaxCards; ++k) {
    prio[k] = pool[k] == dummy ? 2.0f : u24(mix64(base ^ ((uint64_t)(k + 1) * 0xA24BAED4963EE407ull)));
    order[k] = k;
  }
  std::stable_sort(order, order + kMaxCards, [&](int a, int b) { return prio[a] < prio[b]; });
  for (int p = 0; p < P; ++p)
    for (int s = 0; s < kMaxHand && s < q; ++s) {
      const int c = pool[order[p * q + s]];
      if (c < nct) {
        e.hands[p * kNC + c] += 1;
        deck[c] -= 1;
      }
    }
  std::memcpy(e.deck, deck, kNC);
  const bool swap_phase = has(e, R_TEAMS) && P == 4;
  const int rs = e.round_starter == -1 ? e.current_player : (e.round_starter + 1) % P;
  e.current_player = rs;
  for (int i = 0; i < 4; ++i) e.swap_choices[i] = -1;
  e.round_starter = rs;
  e.phase = swap_phase ? 1 : 0;
  e.hand_size = q == 2 ? 6 : q - 1;
  e.deal += 1;
}

void env_reset(muzcpu_dog& e, int P, int rules, uint64_t seed, int game) {   // dog.py:83-186
  std::memset(&e, 0, sizeof(e));
  e.rules = rules;
  if (P != 4) e.rules &= ~R_TEAMS;
  e.num_players = P;
  e.board_size = 40;
  e.total = 56;
  for (int p = 0; p < P; ++p) {
    e.start[p] = p * 10;
    e.target[p] = (int)pymod(p * 10 - 1, 40);
    for (int j = 0; j < 4; ++j) e.goal[p * 4 + j] = 40 + 4 * p + j;
  }
  for (int i = 0; i < 16; ++i) e.pins[i] = -1;
  if (e.rules & R_FREE_PIN)
    for (int p = 0; p < P; ++p) e.pins[p * 4] = e.start[p];
  for (int i = 0; i < kCells; ++i) e.board[i] = -1;
  if (e.rules & R_FREE_PIN) set_pins_on_board(e.board, e.pins, P, e.total);
  e.num_cards = kNC;
  for (int c = 0; c < kNC; ++c) e.deck[c] = 8;
  e.deck[0] = 6;
  for (int i = 0; i < 4; ++i) e.swap_choices[i] = -1;
  e.round_starter = -1;
  e.hand_size = 6;
  e.seed = seed;
  e.game = game;
  distribute_cards(e);
}

// ---------------------------------------------------------------------------------------- legality
void val_swap(const muzcpu_dog& e, bool m[4][kCells]) {   // dog.py:361-391
  const int cp = sub_player(e), P = e.num_players, N = e.total;
  const int8_t* board = e.board;
  for (int j = 0; j < N; ++j) {
    const bool v = board[j] != -1 && board[j] != cp;
    for (int i = 0; i < 4; ++i) m[i][j] = v;
  }
  for (int p = 0; p < P; ++p) {
    const int s = e.start[p];
    const bool v = !((board[s] == p) && has(e, R_START_BLOCK)) && (board[s] != -1);
    for (int i = 0; i < 4; ++i) m[i][s] = v;
  }
  for (int k = 0; k < 4; ++k) {
    const int c = si(e.pins[cp * 4 + k], N);
    if (c >= 0)
      for (int i = 0; i < 4; ++i) m[i][c] = false;
  }
  for (int g = 0; g < P * 4; ++g)
    for (int i = 0; i < 4; ++i) m[i][e.goal[g]] = false;
  const long long dis1 = has(e, R_START_BLOCK) ? e.start[cp] : -1;
  for (int i = 0; i < 4; ++i) {
    const long long pin = e.pins[cp * 4 + i];
    const bool bad = pin == -1 || pin == dis1 || in_goal(pin, e.goal + cp * 4);
    if (bad)
      for (int j = 0; j < N; ++j) m[i][j] = false;
  }
}

struct Common {
  int cp, P;
  long long cur[4], moved[4], fitted[4];
  bool pos[4];
};

Common common(const muzcpu_dog& e, const long long mv[4]) {
  Common c;
  c.cp = sub_player(e);
  c.P = e.num_players;
  for (int p = 0; p < c.P; ++p) c.pos[p] = e.board[e.start[p]] == p;
  for (int i = 0; i < 4; ++i) {
    c.cur[i] = e.pins[c.cp * 4 + i];
    c.moved[i] = c.cur[i] + mv[i];
    c.fitted[i] = pymod(c.moved[i], e.board_size);
  }
  return c;
}

bool val_action_7(const muzcpu_dog& e, const int* dist) {   // dog.py:393-481
  long long mv[4] = {dist[0], dist[1], dist[2], dist[3]};
  Common c = common(e, mv);
  const int cp = c.cp, P = c.P;
  const long long target = e.target[cp], mt = has(e, R_MUST_TRAVERSE) ? 1 : 0, bs = e.board_size;
  const int32_t* goal = e.goal + cp * 4;
  bool pos[4];
  std::memcpy(pos, c.pos, sizeof(pos));
  bool any = false;
  for (int i = 0; i < 4; ++i) any = any || (c.cur[i] == e.start[cp] && c.moved[i] == e.start[cp]);
  pos[cp] = any;
  int32_t tmp[16];
  std::memcpy(tmp, e.pins, sizeof(tmp));
  for (int i = 0; i < 4; ++i) tmp[cp * 4 + i] = (int32_t)(in_goal(c.cur[i], goal) ? c.moved[i] : c.cur[i]);
  int8_t tb[kCells];
  set_pins_on_board(tb, tmp, P, e.total);
  bool D[4];
  relative_order_preserved(c.cur, c.moved, bs, D);
  const long long dist10 = bs / 4;
  for (int i = 0; i < 4; ++i) {
    long long x = c.moved[i] - target - mt;
    bool res = has(e, R_CIRCULAR) ? true : !((c.cur[i] <= target) && ((c.moved[i] > target + 4) || (x == 0 && mt)));
    const long long nsb = pymod(floordiv(c.cur[i], dist10) + 1, P), nsa = floordiv(c.fitted[i], dist10);
    const bool trav = e.start[gidx(nsb, P)] == e.start[gidx(nsa, P)];
    const bool pa = pos[gidx(nsa, P)];
    if (has(e, R_START_BLOCK) && trav) res = !pa && res;
    if (mt && has(e, R_START_BLOCK) && trav && pa) x = 0;
    const bool A = has(e, R_CIRCULAR) && res;
    const bool C = has(e, R_JUMP_GOAL) || check_goal_path(-1, x, goal, tb, cp);
    if (4 >= x && x > 0 && c.cur[i] <= target) res = A || C;
    if (in_goal(c.cur[i], goal)) res = (c.moved[i] <= goal[3]) && (has(e, R_JUMP_GOAL) || D[i]);
    const bool mover = c.cur[i] == -1 ? c.moved[i] == -1 : true;
    if (!(res && mover)) return false;
  }
  return true;
}

void val_normal(const muzcpu_dog& e, int move, bool out[4]) {   // dog.py:483-566
  const long long mv[4] = {move, move, move, move};
  Common c = common(e, mv);
  const int cp = c.cp, P = c.P;
  const long long target = e.target[cp], mt = has(e, R_MUST_TRAVERSE) ? 1 : 0, bs = e.board_size;
  const int32_t* goal = e.goal + cp * 4;
  const int8_t* board = e.board;
  const long long dist10 = bs / 4;
  for (int i = 0; i < 4; ++i) {
    const long long cur = c.cur[i], moved = c.moved[i];
    long long x = moved - target - mt;
    bool res = (board[c.fitted[i]] != cp) || has(e, R_FRIENDLY);
    const long long nsb = pymod(floordiv(cur, dist10) + 1, P), nsa = floordiv(c.fitted[i], dist10);
    const bool trav = e.start[gidx(nsb, P)] == e.start[gidx(nsa, P)];
    const bool pa = c.pos[gidx(nsa, P)];
    if (has(e, R_START_BLOCK) && trav) res = (!pa || cur == e.start[cp]) && res;
    if (mt && has(e, R_START_BLOCK) && trav && pa) x = 0;
    if (!has(e, R_CIRCULAR) && cur <= target && (x > 4 || (x == 0 && mt))) res = false;
    const bool A = has(e, R_CIRCULAR) && res;
    const bool B = board[goal[gidx(x - 1, 4)]] != cp;
    const bool C = has(e, R_JUMP_GOAL) || check_goal_path(-1, x, goal, board, cp);
    if (4 >= x && x > 0 && cur <= target) res = A || (B && C);
    const bool D = has(e, R_JUMP_GOAL) || check_goal_path(cur - goal[0], moved - goal[0] + 1, goal, board, cp);
    if (in_goal(cur, goal)) res = (moved <= goal[3]) && (board[gidx(moved, e.total)] != cp) && D;
    if (cur == -1) res = (move == 1 || move == 11 || move == 13) && !c.pos[cp];
    out[i] = res && move > 0;
  }
}

void val_neg(const muzcpu_dog& e, int move, bool out[4]) {   // dog.py:568-615
  const long long mv[4] = {move, move, move, move};
  Common c = common(e, mv);
  const int cp = c.cp, P = c.P;
  const int32_t* goal = e.goal + cp * 4;
  const long long dist10 = e.board_size / 4;
  for (int i = 0; i < 4; ++i) {
    const long long cur = c.cur[i];
    bool res = (e.board[c.fitted[i]] != cp) || has(e, R_FRIENDLY);
    const long long nsb = floordiv(cur, dist10), nsa = pymod(floordiv(c.fitted[i], dist10) + 1, P);
    const bool cond = e.start[gidx(nsb, P)] == e.start[gidx(nsa, P)];
    if (has(e, R_START_BLOCK) && cond) res = (!c.pos[gidx(nsa, P)] || cur == e.start[cp]) && res;
    res = res && (has(e, R_CIRCULAR) || c.moved[i] >= e.start[cp]);
    if (cur == -1 || in_goal(cur, goal)) res = false;
    out[i] = res;
  }
}

void valid_step_actions(const muzcpu_dog& e, uint8_t* out) {   // dog.py:618-691 -> [joker 396 | real 396]
  const int cp = sub_player(e);
  const int8_t* hand = e.hands + cp * kNC;
  bool sw[4][kCells];
  val_swap(e, sw);
  bool hot[120];
  for (int d = 0; d < 120; ++d) hot[d] = val_action_7(e, g_dists[d]);
  bool normal[12][4];
  for (int m = 0; m < 12; ++m) val_normal(e, kNormal[m], normal[m]);
  bool neg[4];
  val_neg(e, -4, neg);
  static constexpr int kMaskCard[12] = {11, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13};
  const bool joker = hand[0] > 0;
  for (int half = 0; half < 2; ++half) {
    uint8_t* o = out + half * kHalf;
    const bool real = half == 1;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < kCells; ++j) o[i * kCells + j] = sw[i][j] && (real ? hand[1] > 0 : joker);
    for (int d = 0; d < 120; ++d) o[kSwapA + d] = hot[d] && (real ? hand[7] > 0 : joker);
    for (int p = 0; p < 4; ++p)
      for (int m = 0; m < 12; ++m) o[kSwapA + 120 + p * 12 + m] = normal[m][p] && (real ? hand[kMaskCard[m]] > 0 : joker);
    for (int p = 0; p < 4; ++p) o[kHalf - 4 + p] = neg[p] && (real ? hand[4] > 0 : joker);
  }
}

void valid_actions(const muzcpu_dog& e, uint8_t* out) {   // dog.py:693-711 -> [806]
  std::memset(out, 0, kActions);
  if (e.phase == 0) {
    valid_step_actions(e, out);
  } else {
    for (int c = 0; c < kNC; ++c) out[kPlay + c] = e.hands[e.current_player * kNC + c] > 0;
  }
}

// --------------------------------------------------------------------------------------- transitions
struct Out {
  int8_t board[kCells];
  int32_t pins[16];
  int reward;
  bool done;
};

void finish(const muzcpu_dog& e, int cp, const int8_t* board, const int32_t* pins, bool invalid, Out& o) {
  bool w[4];
  get_winner(e, board, w);
  std::memcpy(o.board, board, kCells);
  std::memcpy(o.pins, pins, sizeof(o.pins));
  o.done = e.done || w[0] || w[1] || w[2] || w[3];
  o.reward = e.done ? 0 : (invalid ? -1 : (w[cp] ? 1 : 0));
}

void step_swap(const muzcpu_dog& e, int pin_idx, int swap_pos, Out& o) {   // dog.py:755-788
  const int cp = sub_player(e), N = e.total;
  bool sw[4][kCells];
  val_swap(e, sw);
  const bool invalid = !sw[std::min(std::max(pin_idx, 0), 3)][std::min(std::max(swap_pos, 0), N - 1)];
  if (invalid) return finish(e, cp, e.board, e.pins, true, o);
  const int sp = e.board[gidx(swap_pos, N)];
  const int pp = e.pins[cp * 4 + pin_idx];
  int8_t board[kCells];
  std::memcpy(board, e.board, kCells);
  int c = si(swap_pos, N);
  if (c >= 0) board[c] = (int8_t)cp;
  c = si(pp, N);
  if (c >= 0) board[c] = (int8_t)sp;
  int32_t pins[16];
  std::memcpy(pins, e.pins, sizeof(pins));
  pins[cp * 4 + pin_idx] = swap_pos;
  const int row = si(sp, e.num_players);
  if (row >= 0)
    for (int k = 0; k < 4; ++k)
      if (pins[row * 4 + k] == swap_pos) pins[row * 4 + k] = pp;
  finish(e, cp, board, pins, false, o);
}

void capture_move(const muzcpu_dog& e, int cp, int pin, long long nw, bool invalid, Out& o) {   // _capture_move
  int32_t pins[16];
  std::memcpy(pins, e.pins, sizeof(pins));
  const int at = e.board[gidx(nw, e.total)];
  if (at != -1 && (at != cp || has(e, R_FRIENDLY)) && !invalid)
    for (int k = 0; k < 4; ++k)
      if (pins[at * 4 + k] == nw) pins[at * 4 + k] = -1;
  if (!invalid) pins[cp * 4 + pin] = (int32_t)nw;
  int8_t board[kCells];
  if (invalid) std::memcpy(board, e.board, kCells);
  else set_pins_on_board(board, pins, e.num_players, e.total);
  finish(e, cp, board, pins, invalid, o);
}

void step_normal(const muzcpu_dog& e, int pin, int move, Out& o) {   // dog.py:790-859
  const int cp = sub_player(e);
  bool va[4];
  val_normal(e, move, va);
  const bool invalid = !va[pin];
  const long long cur = e.pins[cp * 4 + pin], moved = cur + move, fitted = pymod(moved, e.board_size);
  const long long x = moved - e.target[cp] - (has(e, R_MUST_TRAVERSE) ? 1 : 0);
  const int32_t* goal = e.goal + cp * 4;
  const bool ig = in_goal(cur, goal);
  const bool a = ig ? check_goal_path(cur - goal[0], moved - goal[0] + 1, goal, e.board, cp)
                    : check_goal_path(-1, x, goal, e.board, cp);
  const long long gx = goal[gidx(x - 1, 4)];
  const bool A = (e.board[gx] != cp) && (has(e, R_JUMP_GOAL) || a);
  long long nw;
  if (cur == -1) nw = e.start[cp];
  else if (ig) nw = moved;
  else if (4 >= x && x > 0 && A && cur <= e.target[cp]) nw = gx;
  else nw = fitted;
  capture_move(e, cp, pin, nw, invalid, o);
}

void step_neg(const muzcpu_dog& e, int pin, int move, Out& o) {   // dog.py:861-911
  const int cp = sub_player(e);
  bool va[4];
  val_neg(e, move, va);
  capture_move(e, cp, pin, pymod((long long)e.pins[cp * 4 + pin] + move, e.board_size), !va[pin], o);
}

// utils/utility_funcs.py:237-303 -> bool[4][total]
void path_matrix(const long long* st, const long long* en, long long start_idx, const int32_t* goal, long long target,
                 int bs, int total, bool trav, bool m[4][kCells]) {
  auto rng = [](long long s, long long t, int N, bool same_area, bool* row) {
    for (int i = 0; i < N; ++i) row[i] = false;
    if (s == -1 || t == -1 || (same_area && s == t)) return;
    for (int i = 0; i < N; ++i) row[i] = s <= t ? (i >= s && i <= t) : (i >= s || i <= t);
  };
  bool anydiff = false;
  for (int i = 0; i < 4; ++i) {
    const bool A = in_goal(st[i], goal), B = in_goal(en[i], goal);
    anydiff = anydiff || (A != B);
    for (int j = 0; j < kCells; ++j) m[i][j] = false;
    if (A == B) {
      rng(st[i], en[i], bs, true, m[i]);
    } else {
      rng(st[i], target, bs, false, m[i]);
      bool r2[kCells];
      rng(goal[0], en[i], total, false, r2);
      for (int j = 0; j < total; ++j) m[i][j] = m[i][j] || r2[j];
    }
  }
  if (trav && anydiff)
    for (int i = 0; i < 4; ++i) m[i][start_idx] = true;
}

void step_hot7(const muzcpu_dog& e, const int* dist, Out& o) {   // dog.py:913-985
  const int cp = sub_player(e), P = e.num_players, N = e.total;
  const bool invalid = !val_action_7(e, dist);
  const long long target = e.target[cp], mt = has(e, R_MUST_TRAVERSE) ? 1 : 0;
  const int32_t* goal = e.goal + cp * 4;
  long long cur[4], moved[4], nw[4];
  int32_t tmp[16];
  std::memcpy(tmp, e.pins, sizeof(tmp));
  for (int i = 0; i < 4; ++i) {
    cur[i] = e.pins[cp * 4 + i];
    moved[i] = cur[i] + dist[i];
    tmp[cp * 4 + i] = (int32_t)(in_goal(cur[i], goal) ? moved[i] : cur[i]);
  }
  int8_t tb[kCells];
  set_pins_on_board(tb, tmp, P, N);
  for (int i = 0; i < 4; ++i) {
    const long long x = moved[i] - target - mt;
    const bool ig = in_goal(cur[i], goal);
    const bool A = has(e, R_JUMP_GOAL) || (ig ? true : check_goal_path(-1, x, goal, tb, cp));
    if (cur[i] == -1) nw[i] = -1;
    else if (ig) nw[i] = moved[i];
    else if (4 >= x && x > 0 && A && cur[i] <= target) nw[i] = goal[gidx(x - 1, 4)];
    else nw[i] = pymod(moved[i], e.board_size);
  }
  int32_t pins[16];
  std::memcpy(pins, e.pins, sizeof(pins));
  if (!invalid)
    for (int i = 0; i < 4; ++i) pins[cp * 4 + i] = (int32_t)nw[i];
  bool paths[4][kCells];
  path_matrix(cur, nw, e.start[cp], goal, target, e.board_size, N, true, paths);
  bool anyp[kCells];
  for (int j = 0; j < N; ++j) anyp[j] = paths[0][j] || paths[1][j] || paths[2][j] || paths[3][j];
  bool hit[16];
  for (int k = 0; k < P * 4; ++k) hit[k] = anyp[gidx(e.pins[k], N)];
  for (int i = 0; i < 4; ++i) {   // check_moving_pins_hit (utils 310-319)
    bool other[kCells];
    for (int j = 0; j < N; ++j) {
      other[j] = false;
      for (int r = 0; r < 4; ++r)
        if (r != i) other[j] = other[j] || paths[r][j];
    }
    hit[cp * 4 + i] = other[gidx(cur[i], N)] && other[gidx(nw[i], N)];
  }
  if (!invalid)
    for (int k = 0; k < P * 4; ++k)
      if (hit[k]) pins[k] = -1;
  int8_t board[kCells];
  if (invalid) std::memcpy(board, e.board, kCells);
  else set_pins_on_board(board, pins, P, N);
  finish(e, cp, board, pins, invalid, o);
}

// map_action_to_move (dog.py:1134-1197) -> is_joker, is_swap, d[4]
void map_action(int action, bool& joker, bool& swap, long long d[4]) {
  joker = action - kHalf < 0;
  const int act = (int)pymod(action, kHalf);
  for (int i = 0; i < 4; ++i) d[i] = 0;
  swap = act < kSwapA;
  if (swap) {
    for (int i = 0; i < 4; ++i) d[i] = -1;
    d[act / kCells] = act % kCells;
  } else if (act < kSwapA + 120) {
    for (int i = 0; i < 4; ++i) d[i] = g_dists[act - kSwapA][i];
  } else if (act < kHalf - 4) {
    const int na = act - (kSwapA + 120);
    int mv = na % 12 + 1;
    mv += mv >= 7;
    d[na / 12] = mv;
  } else {
    d[act - (kHalf - 4)] = -4;
  }
}

int action_card(bool joker, bool swap, const long long d[4]) {   // map_action_to_card (dog.py:1241-1262)
  const long long s = d[0] + d[1] + d[2] + d[3];
  if (joker) return 0;
  if (swap) return 1;
  if (s == -4) return 4;
  return s == 1 ? 11 : (int)s;
}

int next_with_cards(const muzcpu_dog& e, const int8_t* hands, long long tot[4]) {   // dog.py:1042-1046
  for (int p = 0; p < e.num_players; ++p) {
    tot[p] = 0;
    for (int c = 0; c < e.num_cards; ++c) tot[p] += hands[p * kNC + c];
  }
  for (int i = 0; i < e.num_players; ++i) {
    const int cand = (e.current_player + i + 1) % e.num_players;
    if (tot[cand] > 0) return cand;
  }
  return -1;
}

void step_play(muzcpu_dog& e, int action, int& reward, int& done) {   // dog.py:987-1063
  const int cp = sub_player(e);
  bool joker, swap;
  long long d[4];
  map_action(action, joker, swap, d);
  const int card = action_card(joker, swap, d);
  const bool valid_card = e.hands[cp * kNC + gidx(card, e.num_cards)] > 0;
  Out o;
  if (!valid_card) {
    std::memcpy(o.board, e.board, kCells);
    std::memcpy(o.pins, e.pins, sizeof(o.pins));
    o.reward = -1;
    o.done = e.done;
  } else if (swap) {
    int p = 0;
    while (p < 3 && d[p] < 0) ++p;
    step_swap(e, p, (int)d[p], o);
  } else if (d[0] + d[1] + d[2] + d[3] == 7) {
    const int dd[4] = {(int)d[0], (int)d[1], (int)d[2], (int)d[3]};
    step_hot7(e, dd, o);
  } else {
    int p = 0;
    while (p < 3 && d[p] == 0) ++p;
    if (d[p] < 0) step_neg(e, p, (int)d[p], o);
    else step_normal(e, p, (int)d[p], o);
  }
  int8_t hands[4 * kNC];
  std::memcpy(hands, e.hands, sizeof(hands));
  if (o.reward != -1) hands[cp * kNC + gidx(card, e.num_cards)] -= 1;
  long long tot[4];
  const int nxt = next_with_cards(e, hands, tot);
  bool all_zero = true;
  for (int p = 0; p < e.num_players; ++p) all_zero = all_zero && tot[p] == 0;
  std::memcpy(e.board, o.board, kCells);
  std::memcpy(e.pins, o.pins, sizeof(o.pins));
  std::memcpy(e.hands, hands, sizeof(hands));
  e.current_player = o.done ? cp : nxt;
  e.reward = o.reward;
  e.done = o.done;
  if ((all_zero || nxt == -1) && !o.done) distribute_cards(e);
  reward = o.reward;
  done = o.done;
}

void step_swap_phase(muzcpu_dog& e, int card, int& reward, int& done) {   // dog.py:1078-1116
  const int P = e.num_players, cp = e.current_player;
  const int ci = si(card, e.num_cards);
  if (ci >= 0) e.hands[cp * kNC + ci] -= 1;
  e.swap_choices[cp] = (int8_t)card;
  const int nxt = (cp + 1) % P;
  const bool complete = nxt == e.round_starter;
  if (complete) {
    static constexpr int partners[4] = {2, 3, 0, 1};
    for (int p = 0; p < P; ++p) {
      const int rc = e.swap_choices[partners[p]];
      if (rc >= 0 && rc < e.num_cards) e.hands[p * kNC + rc] += 1;
    }
    for (int i = 0; i < 4; ++i) e.swap_choices[i] = -1;
  }
  e.current_player = complete ? e.round_starter : nxt;
  if (complete) e.phase = 0;
  e.reward = 0;
  reward = 0;
  done = e.done;
}

void env_step(muzcpu_dog& e, int action, int& reward, int& done) {   // dog.py:1118-1132
  if (e.phase == 1) step_swap_phase(e, action - kPlay, reward, done);
  else step_play(e, action, reward, done);
}

void no_step(muzcpu_dog& e) {   // dog.py:714-753
  for (int c = 0; c < kNC; ++c) e.hands[e.current_player * kNC + c] = 0;
  long long tot[4];
  const int nxt = next_with_cards(e, e.hands, tot);
  bool any = false;
  for (int p = 0; p < e.num_players; ++p) any = any || tot[p] > 0;
  if (any && nxt != -1) {
    e.current_player = nxt;
    return;
  }
  distribute_cards(e);
}

// engine_random_action (csrc/env_dog.hip:k_dog_random_action): the k-th legal action from the counter uniform
int random_action(const uint8_t* mask, uint64_t seed, int game, int turn) {
  int legal[kActions], n = 0;
  for (int a = 0; a < kActions; ++a)
    if (mask[a]) legal[n++] = a;
  if (n == 0) return -1;
  const float u = u24(mix64(game_key(seed ^ kActionStream, game, turn)));
  return legal[std::min((int)(u * (float)n), n - 1)];
}

// ------------------------------------------------------------------------------------- DOG MuZero slice
// The reference's DOG MuZero is a skeleton (MuZero_DOG/muzero_dog.py:85-99 and game_agent.py:52-57 are `pass`);
// this follows the builder-defined slice the device runs and oracle/dog_muzero.py restates: the 34-channel
// encoding, the DOG RepresentationNetwork (LayerNorm head), Dyn4 / Pred4 at A = 806, mctx's Gumbel search.
constexpr int kDogC = 34;

// oracle/dog_muzero.py:encode_board -> out [34][56] (spatial channels 0..5, global features 6..33 broadcast)
void encode_board(const muzcpu_dog& e, float* out) {
  const int cp = e.current_player, bs = e.board_size, dist = bs / 4, ng = e.total - bs;
  const bool teams = has(e, R_TEAMS);
  int b[kCells];
  for (int i = 0; i < bs; ++i) b[i] = e.board[(i + dist * cp) % bs];
  for (int i = 0; i < ng; ++i) b[bs + i] = e.board[bs + (i + 4 * cp) % ng];
  int rolled[4];
  for (int r = 0; r < 4; ++r) rolled[r] = (cp + r) % 4;
  for (int r = 0; r < 4; ++r)
    for (int w = 0; w < kCells; ++w) out[r * kCells + w] = (float)(b[w] == rolled[r]);
  for (int w = 0; w < kCells; ++w) {
    const float* pc = out;
    out[4 * kCells + w] = teams ? pc[w] + pc[2 * kCells + w] : pc[w];
    out[5 * kCells + w] = teams ? pc[kCells + w] + pc[3 * kCells + w] : pc[kCells + w] + pc[2 * kCells + w] + pc[3 * kCells + w];
  }
  const int sub = sub_player(e);
  int g[28] = {0};
  for (int r = 0; r < 4; ++r)
    for (int k = 0; k < 4; ++k) g[r] += e.pins[rolled[r] * 4 + k] == -1;
  for (int c = 0; c < kNC; ++c) g[4 + c] = e.hands[sub * kNC + c];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < kNC; ++c) g[18 + r] += e.hands[rolled[r] * kNC + c];
  g[22] = e.phase;
  g[23] = e.hand_size;
  g[24] = sub != cp;
  for (int c = 0; c < kNC; ++c) g[25] += e.deck[c];
  g[26] = (int)pymod(e.round_starter - cp, 4);
  const int mates[2] = {cp, (cp + 2) % 4};
  for (int m = 0; m < (teams ? 2 : 1); ++m)
    for (int k = 0; k < 4; ++k) g[27] += e.pins[mates[m] * 4 + k] >= bs;
  for (int c = 0; c < 28; ++c)
    for (int w = 0; w < kCells; ++w) out[(6 + c) * kCells + w] = (float)g[c];
}

// recurrent_inference_fn of the slice: DynamicsNetwork4 (MuZero_det_MADN/muzero_deterministic_madn.py:391-457)
// at one-hot width A = net.A, then PredictionNetwork4.  The one-hot products are row gathers (Dense_0: bias +
// W[a]; Dense_6 / Dense_7: the latent rows' fma chain + W[256 + a]), the same roundings as the full products
// with a one-hot operand (every other term adds an exact zero).
void recurrent_wide(const Net& net, const int* action, const float* emb, int B, float* reward, float* discount,
                    float* logits, float* value, float* nxt, Scratch& s) {
  const std::string d = "dynamics/";
  const int A = net.A;
  const float *W0 = net.w(d + "Dense_0/kernel"), *b0 = net.w(d + "Dense_0/bias");
  std::vector<float> e((size_t)B * 64), sc((size_t)B * kLat), shf((size_t)B * kLat);
  for (int b = 0; b < B; ++b) {
    const int a = action[b];
    for (int j = 0; j < 64; ++j) {
      const float v = (a >= 0 && a < A) ? b0[j] + W0[(size_t)a * 64 + j] : b0[j];
      e[(size_t)b * 64 + j] = std::max(v, 0.f);
    }
  }
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
  std::vector<float> h((size_t)B * 64), l3((size_t)B * 3);
  const char* hid[2] = {"Dense_6", "Dense_7"};
  const char* head[2] = {"reward_head", "discount_head"};
  float* out[2] = {reward, discount};
  for (int k = 0; k < 2; ++k) {
    const float* W = net.w(d + hid[k] + "/kernel");
    dense_raw(W, net.w(d + hid[k] + "/bias"), nxt, B, kLat, 64, h.data());   // the latent rows of [nxt, one-hot]
    for (int b = 0; b < B; ++b) {
      const int a = action[b];
      for (int j = 0; j < 64; ++j) {
        float v = h[(size_t)b * 64 + j];
        if (a >= 0 && a < A) v += W[(size_t)(kLat + a) * 64 + j];
        h[(size_t)b * 64 + j] = std::max(v, 0.f);
      }
    }
    dense(net, d + head[k], h.data(), B, 64, 3, l3.data());
    for (int b = 0; b < B; ++b) out[k][b] = support3(&l3[(size_t)b * 3]);
  }
  prediction(net, nxt, B, logits, value, s);
}

struct DogRec {
  const Net& net;
  Scratch& s;
  void operator()(const int* action, const float* emb, int B, float* reward, float* discount, float* logits,
                  float* value, float* nxt) const {
    recurrent_wide(net, action, emb, B, reward, discount, logits, value, nxt, s);
  }
};

// One self-play turn of `n` DOG lanes (MuZero_det_MADN/game_agent.py:64-192's turn at A = 806, as
// game_agent_dog.DogSelfPlay.turn runs it): legal mask -> (no legal action: no_step) -> encode -> root inference
// -> Gumbel search with the engine's noise of (seed, game id, turn) -> env_step.  act_out[i] = the action (-1:
// no_step).  Returns the number of searched games.
struct DogTurn {
  Search sr;
  Scratch s;
  std::vector<Tree<kActions>> trees;
  std::vector<float> obs, lg, v, e, gum, w, rv;
  std::vector<int> act, search;
  std::unique_ptr<bool[]> inv;
  void init(int n, int S, int D) {
    sr.init(S, D);
    obs.resize((size_t)n * kDogC * kCells);
    lg.resize((size_t)n * kActions);
    v.resize(n);
    e.resize((size_t)n * kLat);
    gum.resize((size_t)n * kActions);
    w.resize((size_t)n * kActions);
    rv.resize(n);
    act.resize(n);
    inv.reset(new bool[(size_t)n * kActions]);
  }
  int run(const Net& net, muzcpu_dog* envs, const int* gid, int n, int turn, float temp, uint64_t seed, int* act_out) {
    search.clear();
    uint8_t mask[kActions];
    for (int i = 0; i < n; ++i) {
      valid_actions(envs[i], mask);
      bool any = false;
      for (int a = 0; a < kActions; ++a) any = any || mask[a];
      act_out[i] = -1;
      if (!any) continue;
      const int k = (int)search.size();
      for (int a = 0; a < kActions; ++a) inv[(size_t)k * kActions + a] = !mask[a];
      encode_board(envs[i], &obs[(size_t)k * kDogC * kCells]);
      gumbel_noise<kActions>(seed, gid[i], turn, temp, &gum[(size_t)k * kActions]);
      search.push_back(i);
    }
    const int B = (int)search.size();
    if (B) {
      representation(net, obs.data(), B, e.data(), s);
      prediction(net, e.data(), B, lg.data(), v.data(), s);
      gumbel_search<kActions>(sr, B, lg.data(), v.data(), e.data(), inv.get(), gum.data(), trees, act.data(), w.data(),
                              rv.data(), DogRec{net, s});
      for (int k = 0; k < B; ++k) act_out[search[k]] = act[k];
    }
    for (int i = 0; i < n; ++i) {
      int r, d;
      if (act_out[i] < 0) no_step(envs[i]);
      else env_step(envs[i], act_out[i], r, d);
    }
    return B;
  }
};

}  // namespace

extern "C" {

void muzcpu_dog_reset(muzcpu_dog* e, int P, int rules, uint64_t seed, int game) { env_reset(*e, P, rules, seed, game); }
void muzcpu_dog_valid_actions(const muzcpu_dog* e, uint8_t* out806) { valid_actions(*e, out806); }
void muzcpu_dog_step(muzcpu_dog* e, int action, int* reward, int* done) { env_step(*e, action, *reward, *done); }
void muzcpu_dog_no_step(muzcpu_dog* e) { no_step(*e); }

// one step_* call (the reference's golden step tests, DOG/test.py): kind 0 normal (a = pin, b = move),
// 1 neg (pin, move), 2 swap (pin, pos), 3 hot 7 (dist); writes board / pins into *e, returns reward, done
void muzcpu_dog_step_kind(muzcpu_dog* e, int kind, int a, int b, const int* dist, int* reward, int* done) {
  Out o;
  if (kind == 0) step_normal(*e, a, b, o);
  else if (kind == 1) step_neg(*e, a, b, o);
  else if (kind == 2) step_swap(*e, a, b, o);
  else step_hot7(*e, dist, o);
  std::memcpy(e->board, o.board, kCells);
  std::memcpy(e->pins, o.pins, sizeof(o.pins));
  *reward = o.reward;
  *done = o.done;
}

// The bench's CPU loop on one thread (bench.py's former NumPy sample, exactly): n games with ids 0..n-1, each
// turn every game takes the counter-RNG random legal action (or no_step) and a finished game is replaced by a
// fresh one with the next id before its turn.  Records the actions [turns][n]; returns env-steps.
int64_t muzcpu_dog_play(int P, int rules, int n, int turns, uint64_t seed, int32_t* actions) {
  std::vector<muzcpu_dog> envs(n);
  std::vector<int> gid(n);
  for (int i = 0; i < n; ++i) env_reset(envs[i], P, rules, seed, gid[i] = i);
  int next = n;
  uint8_t mask[kActions];
  int64_t steps = 0;
  for (int t = 0; t < turns; ++t)
    for (int i = 0; i < n; ++i) {
      if (envs[i].done) env_reset(envs[i], P, rules, seed, gid[i] = next++);
      valid_actions(envs[i], mask);
      const int a = random_action(mask, seed, gid[i], t);
      int r, d;
      if (a < 0) no_step(envs[i]);
      else env_step(envs[i], a, r, d);
      if (actions) actions[(size_t)t * n + i] = a;
      ++steps;
    }
  return steps;
}

// The config (d) CPU baseline: `threads` OpenMP threads, each advancing `lanes` games by the loop above until
// `seconds` have passed.  Returns env-steps (games finished through *games_out).
int64_t muzcpu_dog_bench(int P, int rules, int lanes, uint64_t seed, int threads, double seconds, int64_t* games_out,
                         double* elapsed_out) {
  std::atomic<int> next_game{0};
  std::atomic<int64_t> steps{0}, games{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
#pragma omp parallel num_threads(threads)
  {
    std::vector<muzcpu_dog> envs(lanes);
    std::vector<int> gid(lanes);
    for (int i = 0; i < lanes; ++i) env_reset(envs[i], P, rules, seed, gid[i] = next_game.fetch_add(1));
    uint8_t mask[kActions];
    int64_t mine = 0, fin = 0;
    for (int t = 0; elapsed() < seconds; ++t) {
      for (int i = 0; i < lanes; ++i) {
        if (envs[i].done) {
          env_reset(envs[i], P, rules, seed, gid[i] = next_game.fetch_add(1));
          ++fin;
        }
        valid_actions(envs[i], mask);
        const int a = random_action(mask, seed, gid[i], t);
        int r, d;
        if (a < 0) no_step(envs[i]);
        else env_step(envs[i], a, r, d);
      }
      mine += lanes;
    }
    steps += mine;
    games += fin;
  }
  if (games_out) *games_out = games.load();
  if (elapsed_out) *elapsed_out = elapsed();
  return steps.load();
}

// ---- DOG MuZero slice (see DogTurn) ------------------------------------------------------------------------------
void muzcpu_dog_encode(const muzcpu_dog* e, float* out) { encode_board(*e, out); }

// recurrent inference of a DOG net (muzcpu_net_create with the slice's parameters: A = 806)
void muzcpu_dog_recurrent(void* net, const int* action, const float* emb, int B, float* reward, float* discount,
                          float* logits, float* value, float* nxt) {
  Scratch s;
  recurrent_wide(*(Net*)net, action, emb, B, reward, discount, logits, value, nxt, s);
}

// one batched gumbel_muzero_policy at A = 806 from given root outputs (invalid: uint8 [B][806], gumbel: scaled
// noise [B][806]) -> action [B], action_weights [B][806], root value [B]
void muzcpu_dog_search(void* net, int B, int S, int D, const float* logits, const float* value, const float* emb,
                       const uint8_t* invalid, const float* gumbel, int* action, float* weights, float* root_value) {
  Search sr;
  sr.init(S, D);
  Scratch s;
  std::vector<Tree<kActions>> trees(B);
  std::unique_ptr<bool[]> inv(new bool[(size_t)B * kActions]);
  for (size_t i = 0; i < (size_t)B * kActions; ++i) inv[i] = invalid[i] != 0;
  gumbel_search<kActions>(sr, B, logits, value, emb, inv.get(), gumbel, trees, action, weights, root_value,
                          DogRec{*(Net*)net, s});
}

// n lanes of DOG MuZero self-play on one thread for `turns` turns: lane i starts game i, a finished game is
// replaced before its lane's next turn by a fresh one with the next game id (deal keys and Gumbel noise of that
// id).  actions [turns][n] (-1 = no_step).  Returns the number of searches.
int64_t muzcpu_dog_mz_play(void* netp, int rules, int n, int turns, int S, int D, float temp, uint64_t seed,
                           int32_t* actions) {
  const Net& net = *(Net*)netp;
  std::vector<muzcpu_dog> envs(n);
  std::vector<int> gid(n), act(n);
  for (int i = 0; i < n; ++i) env_reset(envs[i], 4, rules, seed, gid[i] = i);
  int next = n;
  DogTurn dt;
  dt.init(n, S, D);
  int64_t searches = 0;
  for (int t = 0; t < turns; ++t) {
    for (int i = 0; i < n; ++i)
      if (envs[i].done) env_reset(envs[i], 4, rules, seed, gid[i] = next++);
    searches += dt.run(net, envs.data(), gid.data(), n, t, temp, seed, act.data());
    for (int i = 0; i < n; ++i) actions[(size_t)t * n + i] = act[i];
  }
  return searches;
}

// The DOG MuZero CPU baseline (config (d), MuZero policy): `threads` OpenMP threads, each playing `lanes` games
// turn by turn as muzcpu_dog_mz_play (fresh game ids from a shared counter) until `seconds` have passed.  Returns
// env-steps (lanes x turns, no_step turns included, as the device bench counts them); searches, finished games
// and elapsed seconds through the pointers.
int64_t muzcpu_dog_mz_bench(void* netp, int rules, int lanes, int S, int D, float temp, uint64_t seed, int threads,
                            double seconds, int64_t* searches_out, int64_t* games_out, double* elapsed_out) {
  const Net& net = *(Net*)netp;
  std::atomic<int> next_game{0};
  std::atomic<int64_t> steps{0}, searches{0}, games{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
#pragma omp parallel num_threads(threads)
  {
    std::vector<muzcpu_dog> envs(lanes);
    std::vector<int> gid(lanes), act(lanes);
    for (int i = 0; i < lanes; ++i) env_reset(envs[i], 4, rules, seed, gid[i] = next_game.fetch_add(1));
    DogTurn dt;
    dt.init(lanes, S, D);
    int64_t my_steps = 0, my_searches = 0, my_games = 0;
    for (int t = 0; elapsed() < seconds; ++t) {
      for (int i = 0; i < lanes; ++i)
        if (envs[i].done) {
          env_reset(envs[i], 4, rules, seed, gid[i] = next_game.fetch_add(1));
          ++my_games;
        }
      my_searches += dt.run(net, envs.data(), gid.data(), lanes, t, temp, seed, act.data());
      my_steps += lanes;
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
