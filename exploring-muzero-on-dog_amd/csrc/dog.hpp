// DOG rules as device functions over one game's state staged in LDS (DOG/dog.py + utils/utility_funcs.py).
//
// Layout of the work: a wavefront owns a game.  The 792 play actions decompose into 396 base checks
// (224 swaps, 120 hot-7 distributions, 48 normal moves, 4 "-4" moves); the lanes evaluate them in
// parallel and the joker / real-card copies are gated by the hand afterwards.  Transitions run on one
// lane; a deal (distribute_cards) ranks its 120 shuffle keys on all 64 lanes.
// Every JAX quirk of the reference is kept (see oracle/dog.py): clamped gathers, the substituted
// player's hand, the swap phase without validity check, the negative-index column of val_swap.
#pragma once
#include "detmadn.hpp"
#include "rng.hpp"

#ifndef MUZ_DOG_GOAL_CHAIN
#define MUZ_DOG_GOAL_CHAIN 1   // 0: closed-form goal cells (A/B r5m: checks -8 %, env_step +33 %, bench 0.7 % slower)
#endif

namespace muz {

constexpr int kDogCards = 14;
constexpr int kDogBase = 396;                 // one copy (joker or real) of the play actions
constexpr int kDogPlay = 2 * kDogBase;        // 792
constexpr int kDogActions = kDogPlay + kDogCards;   // 806
constexpr int kDogWords = (kDogActions + 31) / 32;  // 26
constexpr int kDogSwaps = 4 * kCells;         // 224
constexpr int kDogHot = 120;
constexpr int kDogNormalBase = kDogSwaps + kDogHot;     // 344
constexpr int kDogNegBase = kDogBase - 4;     // 392
constexpr int kMaxPool = 120;
constexpr unsigned long long kDealStream = 0xDEA1C0DE5EEDull;

__constant__ int8_t c_dists7[kDogHot][4];   // all_pin_distributions(7), filled from the host

struct DogG {   // one game in LDS
  int8_t board[kCells];
  int8_t pins[16];
  int8_t hands[4][kDogCards];
  int8_t deck[kDogCards];
  int8_t swap_choices[4];
  int cp, round_starter, phase, hand_size, done, reward;
  unsigned deal;
  // scratch of a deal
  float key[kMaxPool];
  int8_t pool[kMaxPool];
  int8_t shuffled[kMaxPool];
  unsigned long long wb[7];     // base validity bits by checking slot (env_dog.hip: dog_check_of)
  unsigned long long wj[7], wr[7];   // k_dog_play: legal joker / real-card copies by checking slot
  int need_deal;
};

// (DOG keeps the plain select chains: k_dog_play runs at 64 VGPRs, where rsel / goal_of's VGPR guards add
// spills -- its lane-0 transitions index wave-uniform values)
// Goal cells: the host fills goal[p][g] = goal[p][0] + g for p < P and kTrack for p >= P (host_consts.hpp), so a
// goal cell is a 4-way select of the seat's first goal cell plus g, and "pos in p's goal" a range test -- instead of
// 16-way select chains over the kernarg table, which made the legality checks SALU-bound (k_dog_play's check phase).
// (g in [0, 4) at every call site.)
__device__ __forceinline__ int dgoal0(const DetConsts& c, int p) {
  int r = c.goal[0][0];
  r = p == 1 ? c.goal[1][0] : r;
  r = p == 2 ? c.goal[2][0] : r;
  r = p == 3 ? c.goal[3][0] : r;
  return r;
}
__device__ __forceinline__ int dgoal(const DetConsts& c, int p, int g) {
#if MUZ_DOG_GOAL_CHAIN
  int r = c.goal[0][0];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int h = 0; h < 4; ++h) r = (p == q && g == h) ? c.goal[q][h] : r;
  return r;
#else
  return p < c.P ? dgoal0(c, p) + g : kTrack;
#endif
}

__device__ __forceinline__ int dcst(const int (&a)[4], int i) {
  int r = a[0];
#pragma unroll
  for (int j = 1; j < 4; ++j) r = (i == j) ? a[j] : r;
  return r;
}

__device__ __forceinline__ bool dog_player_done(const DetConsts& c, const int8_t* board, int p) {
  if (p >= c.P) return false;
  bool all = true;
#pragma unroll
  for (int g = 0; g < 4; ++g) all &= board[dgoal(c, p, g)] >= 0;
  return all;
}

__device__ __forceinline__ uint32_t dog_winners(const DetConsts& c, const int8_t* board) {
  uint32_t d = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) d |= dog_player_done(c, board, p) ? (1u << p) : 0u;
  if (!has(c.flags, R_TEAMS)) return d;
  const bool t0 = (d & 1u) && (d & 4u), t1 = (d & 2u) && (d & 8u);
  if ((t0 && t1) || !(t0 || t1)) return 0u;
  return t0 ? 0x5u : 0xAu;
}

__device__ __forceinline__ int dog_sub(const DetConsts& c, const DogG& s) {
  return (has(c.flags, R_TEAMS) && dog_player_done(c, s.board, s.cp)) ? (s.cp + 2) % 4 : s.cp;
}

__device__ __forceinline__ int dpin(const DogG& s, int p, int k) { return s.pins[p * 4 + k]; }

__device__ __forceinline__ bool in_goal_p(const DetConsts& c, int p, int pos) {
#if MUZ_DOG_GOAL_CHAIN
  return pos == dgoal(c, p, 0) || pos == dgoal(c, p, 1) || pos == dgoal(c, p, 2) || pos == dgoal(c, p, 3);
#else
  return p < c.P ? (unsigned)(pos - dgoal0(c, p)) < 4u : pos == kTrack;
#endif
}

// all(board[goal[cp][g]] != cp  for lo < g < hi)
__device__ __forceinline__ bool dog_goal_free(const DetConsts& c, const int8_t* board, int cp, int lo, int hi) {
  bool ok = true;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    if (lo < g && g < hi) ok &= board[dgoal(c, cp, g)] != cp;
  return ok;
}

__device__ __forceinline__ bool pos_on_start(const DetConsts& c, const int8_t* board, int q) {
  return q < c.P && board[dcst(c.start, q)] == q;
}

// ---- val_swap (dog.py:317-348): bit [pin, pos] -------------------------------------------------
__device__ __forceinline__ bool dog_val_swap(const DetConsts& c, const DogG& s, int cp, int pin, int pos) {
  const uint32_t F = c.flags;
  const int b = s.board[pos];
  bool ok = !(b == -1 || b == cp);                       // cond_a
  bool is_start = false;
  for (int q = 0; q < c.P; ++q)
    if (dcst(c.start, q) == pos) {                        // cond_b (start columns)
      is_start = true;
      ok = !((s.board[pos] == q) && has(F, R_START_BLOCK)) && (s.board[pos] != -1);
    }
  (void)is_start;
  for (int k = 0; k < 4; ++k) {                          // cond_c: own pins' columns (-1 -> column 55)
    const int p = dpin(s, cp, k);
    if ((p < 0 ? p + kCells : p) == pos) ok = false;
  }
  for (int q = 0; q < c.P; ++q)                           // condA: every goal column
    if (in_goal_p(c, q, pos)) ok = false;
  const int cur = dpin(s, cp, pin);                       // condB: disallowed pin positions
  const bool dis = cur == -1 || (has(F, R_START_BLOCK) && cur == dcst(c.start, cp)) || in_goal_p(c, cp, cur);
  return ok && !dis;
}

// ---- val_action_normal_move (dog.py:483-566) ----------------------------------------------------
__device__ __forceinline__ bool dog_val_normal(const DetConsts& c, const DogG& s, int cp, int pin, int move) {
  const uint32_t F = c.flags;
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = dcst(c.target, cp);
  const int g0 = dgoal(c, cp, 0), g3 = dgoal(c, cp, 3);
  const int cur = dpin(s, cp, pin);
  if (cur == -1) return (move == 1 || move == 11 || move == 13) && !pos_on_start(c, s.board, cp) && move > 0;
  const int moved = cur + move;
  const int fitted = fmodp(moved, kTrack);
  int x = moved - tgt - mt;
  bool res = (s.board[fitted] != cp) || has(F, R_FRIENDLY);
  const int nsb_j = jidx(fmodp(fdiv(cur, kDist) + 1, c.P), c.P);
  const int nsa_j = jidx(fdiv(fitted, kDist), c.P);
  const bool trav = dcst(c.start, nsb_j) == dcst(c.start, nsa_j);
  const bool pa = pos_on_start(c, s.board, nsa_j);
  if (has(F, R_START_BLOCK) && trav) res = (!pa || cur == dcst(c.start, cp)) && res;
  if (mt && has(F, R_START_BLOCK) && trav && pa) x = 0;
  if (!has(F, R_CIRCULAR) && cur <= tgt && (x > 4 || (x == 0 && mt))) res = false;
  if (4 >= x && x > 0 && cur <= tgt) {
    const bool A = has(F, R_CIRCULAR) && res;
    const bool B = s.board[dgoal(c, cp, jidx(x - 1, 4))] != cp;
    const bool C = has(F, R_JUMP_GOAL) || dog_goal_free(c, s.board, cp, -1, x);
    res = A || (B && C);
  }
  if (in_goal_p(c, cp, cur)) {
    const bool D = has(F, R_JUMP_GOAL) || dog_goal_free(c, s.board, cp, cur - g0, moved - g0 + 1);
    res = (moved <= g3) && (s.board[jidx(moved, kCells)] != cp) && D;
  }
  return res && move > 0;
}

// ---- val_neg_move (dog.py:568-614); the action space only uses move = -4 --------------------------
__device__ __forceinline__ bool dog_val_neg(const DetConsts& c, const DogG& s, int cp, int pin, int move = -4) {
  const uint32_t F = c.flags;
  const int cur = dpin(s, cp, pin);
  if (cur == -1 || in_goal_p(c, cp, cur)) return false;
  const int moved = cur + move;
  const int fitted = fmodp(moved, kTrack);
  bool res = (s.board[fitted] != cp) || has(F, R_FRIENDLY);
  const int nsb_j = jidx(fdiv(cur, kDist), c.P);
  const int nsa_j = jidx(fmodp(fdiv(fitted, kDist) + 1, c.P), c.P);
  const bool cond = dcst(c.start, nsb_j) == dcst(c.start, nsa_j);
  if (has(F, R_START_BLOCK) && cond) res = (!pos_on_start(c, s.board, nsa_j) || cur == dcst(c.start, cp)) && res;
  return res && (has(F, R_CIRCULAR) || moved >= dcst(c.start, cp));
}

// ---- val_action_7 (dog.py:350-481) for one distribution ------------------------------------------
__device__ __forceinline__ bool dog_val7(const DetConsts& c, const DogG& s, int cp, const int (&d)[4]) {
  const uint32_t F = c.flags;
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = dcst(c.target, cp);
  const int g3 = dgoal(c, cp, 3);
  int cur[4], moved[4];
  bool ing[4];
  bool pos_cp = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    cur[k] = dpin(s, cp, k);
    moved[k] = cur[k] + d[k];
    ing[k] = in_goal_p(c, cp, cur[k]);
    pos_cp |= (cur[k] == dcst(c.start, cp)) && (moved[k] == dcst(c.start, cp));
  }
  // goal cells of cp occupied by cp after the in-goal pins moved (tmp_board)
  bool occ[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bool o = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) o |= (ing[k] ? moved[k] : cur[k]) == dgoal(c, cp, g);
    occ[g] = o;
  }
  bool all = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int fitted = fmodp(moved[k], kTrack);
    int x = moved[k] - tgt - mt;
    bool res = has(F, R_CIRCULAR) ? true : !((cur[k] <= tgt) && ((moved[k] > tgt + 4) || (x == 0 && mt)));
    const int nsb_j = jidx(fmodp(fdiv(cur[k], kDist) + 1, c.P), c.P);
    const int nsa_j = jidx(fdiv(fitted, kDist), c.P);
    const bool trav = dcst(c.start, nsb_j) == dcst(c.start, nsa_j);
    const bool pa = (nsa_j == cp) ? pos_cp : pos_on_start(c, s.board, nsa_j);
    if (has(F, R_START_BLOCK) && trav) res = !pa && res;
    if (mt && has(F, R_START_BLOCK) && trav && pa) x = 0;
    if (4 >= x && x > 0 && cur[k] <= tgt) {
      const bool A = has(F, R_CIRCULAR) && res;
      bool C = has(F, R_JUMP_GOAL);
      if (!C) {
        C = true;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (-1 < g && g < x) C &= !occ[g];
      }
      res = A || C;
    }
    if (ing[k]) {
      bool D = has(F, R_JUMP_GOAL);
      if (!D) {   // check_relative_order_preserved: pairwise order among in-goal pins kept
        D = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!(cur[j] >= kTrack)) continue;
          const int so = (cur[k] > cur[j]) - (cur[k] < cur[j]);
          const int sn = (moved[k] > moved[j]) - (moved[k] < moved[j]);
          D &= so == sn;
        }
      }
      res = (moved[k] <= g3) && D;
    }
    const bool mover = cur[k] == -1 ? moved[k] == -1 : true;
    all &= res && mover;
  }
  return all;
}

// Base action i in [0, 396) (one copy): swap [0,224), hot-7 [224,344), normal [344,392), -4 [392,396).
__device__ __forceinline__ bool dog_base_valid(const DetConsts& c, const DogG& s, int cp, int i) {
  if (i < kDogSwaps) return dog_val_swap(c, s, cp, i / kCells, i % kCells);
  if (i < kDogNormalBase) {
    int d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = c_dists7[i - kDogSwaps][k];
    return dog_val7(c, s, cp, d);
  }
  if (i < kDogNegBase) {
    const int na = i - kDogNormalBase;
    int mv = na % 12 + 1;
    mv += mv >= 7 ? 1 : 0;
    return dog_val_normal(c, s, cp, na / 12, mv);
  }
  return dog_val_neg(c, s, cp, i - kDogNegBase);
}

// Card a base action needs (map_action_to_card of the real copy).
__device__ __forceinline__ int dog_base_card(int i) {
  if (i < kDogSwaps) return 1;
  if (i < kDogNormalBase) return 7;
  if (i < kDogNegBase) {
    int mv = (i - kDogNormalBase) % 12 + 1;
    mv += mv >= 7 ? 1 : 0;
    return mv == 1 ? 11 : mv;
  }
  return 4;
}

}  // namespace muz
