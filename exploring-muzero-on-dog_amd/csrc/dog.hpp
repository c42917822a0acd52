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

// ---- k_dog_play's legality checks, lean form (MUZ_DOG_LEAN_CHECKS) ------------------------------------------------
// The same predicates as dog_val_swap / dog_val7 / dog_val_normal / dog_val_neg (dog.py:350-615), with everything
// that depends only on the mover -- its pins, target, goal cells, the seats' start cells, which starts are occupied
// by their owners, the goal-cell occupancy -- gathered once per check phase into DogCtx in LDS instead of being
// recomputed inside every check through select chains over the kernarg tables and runtime-P modulos.  Seat geometry
// facts used (host_consts.hpp): goal[p][g] = goal[p][0] + g for p < P; starts are distinct.  (Held in registers,
// built by every wave, it cost 224 SGPR spills and made the phase slower than the select chains it replaced.)
struct DogCtx {
  int P, cp, tgt, g0, start_cp;
  bool circ, sb, jump, friendly;
  int mt;
  int start[4];          // seat start cells (p >= P: the host's 0)
  int cur[4];            // the mover's pins
  int nsb_start[4];      // dog_val7 / dog_val_normal: start cell of the seat after the pin's section
  unsigned posbits;      // bit q: q < P and board[start[q]] == q (pos_on_start)
  unsigned gocc;         // bit g: board[goal[cp][g]] == cp
  unsigned ingbits;      // bit k: pin k in the mover's goal
  unsigned long long goal_cells;   // bit c: c is a goal cell of some seat q < P
  // per-launch copies of the rule constants the per-turn build reads (LDS instead of dependent kernarg loads)
  bool teams;
  int goal0[4];          // goal[q][0] (q >= P: unused)
  int target[4];
};

// dog_ctx in LDS, in two parts: the rule constants once per launch (dog_ctx_static, one lane), and the mover's
// facts once per turn by one full wave (dog_ctx_turn: lane q computes seat / pin / goal-cell q's facts, the bit sets
// are ballots) reading only LDS -- a few dependent LDS round trips instead of one lane's serial chain of kernarg and
// LDS loads (measured ~4.5k cycles per turn with tid 0 building all of dog_ctx, ~2.3k with the wave on kernarg).
__device__ __forceinline__ void dog_ctx_static(const DetConsts& c, DogCtx* out) {
  const uint32_t F = c.flags;
  out->P = c.P;
  out->circ = has(F, R_CIRCULAR);
  out->sb = has(F, R_START_BLOCK);
  out->jump = has(F, R_JUMP_GOAL);
  out->friendly = has(F, R_FRIENDLY);
  out->teams = has(F, R_TEAMS);
  out->mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  unsigned long long gc = 0ull;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    out->start[p] = c.start[p];
    out->goal0[p] = c.goal[p][0];
    out->target[p] = c.target[p];
    if (p < c.P) gc |= 0xFull << c.goal[p][0];
  }
  out->goal_cells = gc;
}

// dog_sub (dog.hpp) on the LDS constants: the teammate moves for a seat whose pins are all home
__device__ __forceinline__ int dog_sub_lean(const DogCtx& x, const DogG& s) {
  const int p = s.cp;
  if (!x.teams || p >= x.P) return p;
  const int g = x.goal0[p];
  const bool done = s.board[g] >= 0 && s.board[g + 1] >= 0 && s.board[g + 2] >= 0 && s.board[g + 3] >= 0;
  return done ? (p + 2) % 4 : p;
}

__device__ __forceinline__ void dog_ctx_turn(const DogG& s, int lane, DogCtx* out) {
  const DogCtx& x = *out;
  const int P = x.P;
  const int cp = dog_sub_lean(x, s);
  const int q = lane & 3;
  const int start_q = x.start[q];
  const int g0 = cp < P ? x.goal0[cp] : kTrack;
  const int cur = dpin(s, cp, q);
  const bool pos_q = lane < 4 && q < P && s.board[start_q] == q;
  const bool occ_g = lane < 4 && s.board[g0 + q] == cp;
  const bool ing_k = lane < 4 && (unsigned)(cur - g0) < 4u;
  const unsigned posbits = (unsigned)__ballot(pos_q) & 0xFu;
  const unsigned gocc = (unsigned)__ballot(occ_g) & 0xFu;
  const unsigned ingbits = (unsigned)__ballot(ing_k) & 0xFu;
  const int nsb = x.start[mod_small(fdiv(cur, kDist) + 1, P)];
  const int tgt = x.target[cp], start_cp = x.start[cp];
  __builtin_amdgcn_wave_barrier();   // every lane has read the static part before lane 0 writes the turn part
  if (lane < 4) {
    out->cur[q] = cur;
    out->nsb_start[q] = nsb;
  }
  if (lane == 0) {
    out->cp = cp;
    out->tgt = tgt;
    out->g0 = g0;
    out->start_cp = start_cp;
    out->posbits = posbits;
    out->gocc = gocc;
    out->ingbits = ingbits;
  }
}

// val_swap (dog.py:317-348), pin / pos per lane
__device__ __forceinline__ bool dog_val_swap_lean(const DogCtx& x, const DogG& s, int pin, int pos) {
  const int b = s.board[pos];
  bool ok = !(b == -1 || b == x.cp);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < x.P && x.start[q] == pos) ok = !((b == q) && x.sb) && (b != -1);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = x.cur[k];
    if ((p < 0 ? p + kCells : p) == pos) ok = false;
  }
  if ((x.goal_cells >> pos) & 1ull) ok = false;
  const int cur = x.cur[pin];
  const bool dis = cur == -1 || (x.sb && cur == x.start_cp) || (unsigned)(cur - x.g0) < 4u;
  return ok && !dis;
}

// val_action_7 (dog.py:393-481) for distribution d
__device__ __forceinline__ bool dog_val7_lean(const DogCtx& x, const int (&d)[4]) {
  int moved[4];
  bool pos_cp = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    moved[k] = x.cur[k] + d[k];
    pos_cp |= (x.cur[k] == x.start_cp) && (d[k] == 0);
  }
  unsigned occ = 0u;   // goal cells of the mover occupied after its in-goal pins moved
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = ((x.ingbits >> k) & 1u) ? moved[k] : x.cur[k];
    if ((unsigned)(v - x.g0) < 4u) occ |= 1u << (v - x.g0);
  }
  const int g3 = x.g0 + 3;
  bool all = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int cur = x.cur[k], mv = moved[k];
    const int fitted = mv < 0 ? mv + kTrack : (mv >= kTrack ? mv - kTrack : mv);   // mv in [-1, 62]
    int xx = mv - x.tgt - x.mt;
    bool res = x.circ ? true : !((cur <= x.tgt) && ((mv > x.tgt + 4) || (xx == 0 && x.mt)));
    const int nsa = (fitted >= 10) + (fitted >= 20) + (fitted >= 30);
    const int nsa_j = nsa < x.P - 1 ? nsa : x.P - 1;
    const bool trav = x.nsb_start[k] == x.start[nsa_j];
    const bool pa = (nsa_j == x.cp) ? pos_cp : ((x.posbits >> nsa_j) & 1u) != 0u;
    if (x.sb && trav) res = !pa && res;
    if (x.mt && x.sb && trav && pa) xx = 0;
    if (4 >= xx && xx > 0 && cur <= x.tgt) {
      const bool A = x.circ && res;
      const bool C = x.jump || (occ & ((1u << xx) - 1u)) == 0u;   // !occ[g] for 0 <= g < xx
      res = A || C;
    }
    if ((x.ingbits >> k) & 1u) {
      bool D = x.jump;
      if (!D) {
        D = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!(x.cur[j] >= kTrack)) continue;
          const int so = (cur > x.cur[j]) - (cur < x.cur[j]);
          const int sn = (mv > moved[j]) - (mv < moved[j]);
          D &= so == sn;
        }
      }
      res = (mv <= g3) && D;
    }
    const bool mover = cur == -1 ? mv == -1 : true;
    all &= res && mover;
  }
  return all;
}

// val_action_normal_move (dog.py:483-566)
__device__ __forceinline__ bool dog_val_normal_lean(const DogCtx& x, const DogG& s, int pin, int move) {
  const int cur = x.cur[pin];
  if (cur == -1) return (move == 1 || move == 11 || move == 13) && !((x.posbits >> x.cp) & 1u) && move > 0;
  const int moved = cur + move;                                  // in [0, 68]
  const int fitted = moved >= kTrack ? moved - kTrack : moved;
  int xx = moved - x.tgt - x.mt;
  bool res = (s.board[fitted] != x.cp) || x.friendly;
  const int nsa = (fitted >= 10) + (fitted >= 20) + (fitted >= 30);
  const int nsa_j = nsa < x.P - 1 ? nsa : x.P - 1;
  const bool trav = x.nsb_start[pin] == x.start[nsa_j];
  const bool pa = ((x.posbits >> nsa_j) & 1u) != 0u;
  if (x.sb && trav) res = (!pa || cur == x.start_cp) && res;
  if (x.mt && x.sb && trav && pa) xx = 0;
  if (!x.circ && cur <= x.tgt && (xx > 4 || (xx == 0 && x.mt))) res = false;
  if (4 >= xx && xx > 0 && cur <= x.tgt) {
    const bool A = x.circ && res;
    const bool B = ((x.gocc >> (xx - 1)) & 1u) == 0u;             // jidx(x - 1, 4) = x - 1 here
    const bool C = x.jump || (x.gocc & ((1u << xx) - 1u)) == 0u;   // goal_free(cp, -1, x)
    res = A || (B && C);
  }
  if ((unsigned)(cur - x.g0) < 4u) {
    const int lo = cur - x.g0, hi = moved - x.g0 + 1;            // goal_free(cp, lo, hi): lo < g < hi
    unsigned m = 0u;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (lo < g && g < hi) m |= 1u << g;
    const bool D = x.jump || (x.gocc & m) == 0u;
    res = (moved <= x.g0 + 3) && (s.board[moved < kCells ? moved : kCells - 1] != x.cp) && D;
  }
  return res && move > 0;
}

// val_neg_move (dog.py:568-614), move = -4
__device__ __forceinline__ bool dog_val_neg_lean(const DogCtx& x, const DogG& s, int pin) {
  const int cur = x.cur[pin];
  if (cur == -1 || (unsigned)(cur - x.g0) < 4u) return false;
  const int moved = cur - 4;                                     // cur in [0, 39]: moved in [-4, 35]
  const int fitted = moved < 0 ? moved + kTrack : moved;
  bool res = (s.board[fitted] != x.cp) || x.friendly;
  const int nsb = (cur >= 10) + (cur >= 20) + (cur >= 30);
  const int nsb_j = nsb < x.P - 1 ? nsb : x.P - 1;
  const int nsa_j = mod_small((fitted >= 10) + (fitted >= 20) + (fitted >= 30) + 1, x.P);
  const bool cond = x.start[nsb_j] == x.start[nsa_j];
  if (x.sb && cond) res = (!((x.posbits >> nsa_j) & 1u) || cur == x.start_cp) && res;
  return res && (x.circ || moved >= x.start_cp);
}

// dog_base_valid on the lean predicates (base action i in [0, 396)); d7: the 120 distributions packed one per u32
// (byte k = pin k's share) in LDS, or null for the __constant__ table (a per-lane global load)
__device__ __forceinline__ bool dog_base_valid_lean(const DogCtx& x, const DogG& s, int i, const uint32_t* d7) {
  if (i < kDogSwaps) return dog_val_swap_lean(x, s, i / kCells, i % kCells);
  if (i < kDogNormalBase) {
    int d[4];
    if (d7) {
      const uint32_t w = d7[i - kDogSwaps];
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k] = (int)((w >> (8 * k)) & 0xFFu);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k] = c_dists7[i - kDogSwaps][k];
    }
    return dog_val7_lean(x, d);
  }
  if (i < kDogNegBase) {
    const int na = i - kDogNormalBase;
    int mv = na % 12 + 1;
    mv += mv >= 7 ? 1 : 0;
    return dog_val_normal_lean(x, s, na / 12, mv);
  }
  return dog_val_neg_lean(x, s, i - kDogNegBase);
}

}  // namespace muz

