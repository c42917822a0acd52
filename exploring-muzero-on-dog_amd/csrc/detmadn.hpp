// Deterministic MADN rules as per-lane device functions (one board per wavefront lane).
//
// Restates MADN/deterministic_madn.py (reference) for the GPU:
//   valid_action 299-393, env_step 170-257, no_step 283-297, encode_board 395-438,
//   set_pins_on_board 259-271, refill_action_set 273-281, is_player_done/get_winner 122-168,
//   check_goal_path_for_pin{,2} utils/utility_funcs.py:142-184.
// Pins / action sets / player live in VGPRs; the board of each lane is staged in LDS
// ([cell][lane] bytes) so the data-dependent board lookups are LDS reads, not scratch.
#pragma once
#include "common.hpp"

namespace muz {

constexpr int kCells = 56;     // 4*distance + 16, distance fixed at 10
constexpr int kTrack = 40;     // board_size
constexpr int kDist = 10;

enum : uint32_t {
  R_TEAMS = 1u << 0,
  R_FREE_PIN = 1u << 1,
  R_CIRCULAR = 1u << 2,
  R_START_BLOCK = 1u << 3,
  R_JUMP_GOAL = 1u << 4,
  R_FRIENDLY = 1u << 5,
  R_START_ON_1 = 1u << 6,
  R_BONUS_6 = 1u << 7,
  R_MUST_TRAVERSE = 1u << 8,
  R_DICE_RETHROW = 1u << 9,   // classic only
};

// Rule constants after env_reset's layout fix-up (deterministic_madn.py:62-78).
struct DetConsts {
  int P;
  int starting_player;
  uint32_t flags;
  int start[4];
  int target[4];
  int goal[4][4];
};

struct DetLane {
  int pins[16];   // [p*4 + k]
  int aset[24];   // [p*6 + m]
  int cp;         // current_player (unsubstituted)
  int done;
  int reward;
};

// LDS view of one lane's board: cell c of this lane at base[c * bs].
struct BoardView {
  int8_t* base;
  int bs;
  __device__ __forceinline__ int at(int cell) const { return base[cell * bs]; }
  __device__ __forceinline__ void set(int cell, int v) const { base[cell * bs] = (int8_t)v; }
};

__device__ __forceinline__ bool has(uint32_t f, uint32_t bit) { return (f & bit) != 0; }

__device__ __forceinline__ int pin_of(const DetLane& s, int p, int k) { return rsel(s.pins, p * 4 + k); }
__device__ __forceinline__ int aset_of(const DetLane& s, int p, int m) { return rsel(s.aset, p * 6 + m); }

// A game's pins and action set kept in an LDS row (pins [0, 16), action set [16, 40)) instead of registers, read
// and written by index: the G-lane env round (k_det_round_g) runs legal_ctx, the encode and env_step on it
// without holding all 40 values in VGPRs.  The rule functions below take either lane type through these
// accessors (static index j: lane_pin / lane_aset; dynamic index: pin_of / aset_of / set_pin / set_aset).
struct LdsLane {
  int8_t* row;
  int cp, done, reward;
};
__device__ __forceinline__ int pin_of(const LdsLane& s, int p, int k) { return s.row[p * 4 + k]; }
__device__ __forceinline__ int aset_of(const LdsLane& s, int p, int m) { return s.row[16 + p * 6 + m]; }
__device__ __forceinline__ int lane_pin(const DetLane& s, int j) { return s.pins[j]; }
__device__ __forceinline__ int lane_aset(const DetLane& s, int j) { return s.aset[j]; }
__device__ __forceinline__ void lane_set_pin(DetLane& s, int j, int v) { s.pins[j] = v; }
__device__ __forceinline__ void lane_set_aset(DetLane& s, int j, int v) { s.aset[j] = v; }
__device__ __forceinline__ void set_pin(DetLane& s, int idx, int v) { rset(s.pins, idx, v); }
__device__ __forceinline__ void set_aset(DetLane& s, int idx, int v) { rset(s.aset, idx, v); }
__device__ __forceinline__ int lane_pin(const LdsLane& s, int j) { return s.row[j]; }
__device__ __forceinline__ int lane_aset(const LdsLane& s, int j) { return s.row[16 + j]; }
__device__ __forceinline__ void lane_set_pin(LdsLane& s, int j, int v) { s.row[j] = (int8_t)v; }
__device__ __forceinline__ void lane_set_aset(LdsLane& s, int j, int v) { s.row[16 + j] = (int8_t)v; }
__device__ __forceinline__ void set_pin(LdsLane& s, int idx, int v) { s.row[idx] = (int8_t)v; }
__device__ __forceinline__ void set_aset(LdsLane& s, int idx, int v) { s.row[16 + idx] = (int8_t)v; }

__device__ __forceinline__ int cst(const int (&a)[4], int i) { return rsel(a, i); }

__device__ __forceinline__ int goal_of(const DetConsts& c, int p, int g) {
  int r = c.goal[0][0];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      r = (p == q && g == h) ? c.goal[q][h] : r;
      asm volatile("" : "+v"(r));   // (see rsel: keeps the consts out of scratch)
    }
  return r;
}

// is_player_done (deterministic_madn.py:122-137): all four goal cells of `p` hold a pin.
__device__ __forceinline__ bool player_done(const DetConsts& c, const BoardView& b, int p) {
  if (p >= c.P) return false;
  bool all = true;
#pragma unroll
  for (int g = 0; g < 4; ++g) all &= b.at(goal_of(c, p, g)) >= 0;
  return all;
}

// Team substitution (deterministic_madn.py:184, 310).
__device__ __forceinline__ int sub_player(const DetConsts& c, const BoardView& b, int cp0) {
  return (has(c.flags, R_TEAMS) && player_done(c, b, cp0)) ? (cp0 + 2) % 4 : cp0;
}

// get_winner (deterministic_madn.py:139-168) as a 4-bit mask.
__device__ __forceinline__ uint32_t winners(const DetConsts& c, const BoardView& b) {
  uint32_t d = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) d |= player_done(c, b, p) ? (1u << p) : 0u;
  if (!has(c.flags, R_TEAMS)) return d;
  bool t0 = (d & 1u) && (d & 4u);
  bool t1 = (d & 2u) && (d & 8u);
  if ((t0 && t1) || !(t0 || t1)) return 0u;
  return t0 ? 0x5u : 0xAu;
}

// all(board[goal[g]] != cp for lo < g < hi)   (check_goal_path_for_pin{,2})
__device__ __forceinline__ bool goal_path_free(const DetConsts& c, const BoardView& b, int cp, int lo, int hi) {
  bool ok = true;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    if (lo < g && g < hi) ok &= b.at(goal_of(c, cp, g)) != cp;
  return ok;
}

// valid_action (deterministic_madn.py:299-393), split into the per-state prelude (LegalCtx) and the check of one
// (pin i, move m) (legal_one): det_legal runs all 24 checks in one lane, k_det_round_g 24 / G checks per lane.
struct LegalCtx {
  int cp0, cp, tgt, g0, g3, mt, start_cp;
  bool home_ok;
  bool pos[4];
  uint32_t avail;   // moves m with action_set[cp][m-1] > 0, bit m-1
};
template <class Lane>
__device__ __forceinline__ LegalCtx legal_ctx(const DetConsts& c, const Lane& s, const BoardView& b) {
  LegalCtx x;
  const uint32_t F = c.flags;
  x.cp0 = s.cp;
  x.cp = sub_player(c, b, x.cp0);
  x.tgt = cst(c.target, x.cp);
  x.g0 = goal_of(c, x.cp, 0);
  x.g3 = goal_of(c, x.cp, 3);
  x.mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  x.start_cp = cst(c.start, x.cp);
  x.home_ok = b.at(x.start_cp) != x.cp0;   // compares the UNSUBSTITUTED player (line 390)
#pragma unroll
  for (int q = 0; q < 4; ++q) x.pos[q] = (q < c.P) ? (b.at(cst(c.start, q)) == q) : false;
  x.avail = 0;
#pragma unroll
  for (int m = 0; m < 6; ++m) x.avail |= (aset_of(s, x.cp, m) > 0) ? (1u << m) : 0u;
  return x;
}
// the rule checks of pin i (current cell `cur`) with move m, before the action-set gate
__device__ __forceinline__ bool legal_one(const DetConsts& c, const BoardView& b, const LegalCtx& x, int cur, int m) {
  const uint32_t F = c.flags;
  const int cp = x.cp, tgt = x.tgt, mt = x.mt;
  const bool in_goal = (cur == goal_of(c, cp, 0)) | (cur == goal_of(c, cp, 1)) | (cur == goal_of(c, cp, 2)) |
                       (cur == goal_of(c, cp, 3));
  const int nsb = mod_small(fdiv(cur, kDist) + 1, c.P);   // fdiv(cur, 10) + 1 in [0, 6]
  bool res;
  if (cur == -1) {
    res = (m == 6 || (m == 1 && has(F, R_START_ON_1))) && x.home_ok;
  } else {
    const int moved = cur + m;
    const int fitted = fmodp(moved, kTrack);
    int xx = moved - tgt - mt;
    res = (b.at(fitted) != cp) || has(F, R_FRIENDLY);
    const int nsa = fdiv(fitted, kDist);
    const int nsa_j = jidx(nsa, c.P);
    const bool trav = cst(c.start, jidx(nsb, c.P)) == cst(c.start, nsa_j);
    const bool pos_a = x.pos[0] & (nsa_j == 0) | x.pos[1] & (nsa_j == 1) | x.pos[2] & (nsa_j == 2) |
                       x.pos[3] & (nsa_j == 3);
    if (has(F, R_START_BLOCK) && trav) res = (!pos_a || cur == x.start_cp) && res;
    if (mt && has(F, R_START_BLOCK) && trav && pos_a) xx = 0;
    if (!has(F, R_CIRCULAR) && cur <= tgt && (xx > 4 || (xx == 0 && mt))) res = false;
    if (4 >= xx && xx > 0 && cur <= tgt) {
      const bool A = has(F, R_CIRCULAR) && res;
      const bool B = b.at(goal_of(c, cp, jidx(xx - 1, 4))) != cp;
      const bool C = has(F, R_JUMP_GOAL) || goal_path_free(c, b, cp, -1, xx);
      res = A || (B && C);
    }
    if (in_goal) {
      const bool D = has(F, R_JUMP_GOAL) || goal_path_free(c, b, cp, cur - x.g0, moved - x.g0 + 1);
      res = (moved <= x.g3) && (b.at(jidx(moved, kCells)) != cp) && D;
    }
  }
  return res;
}
// -> 24-bit mask, bit pin*6 + (move-1)
__device__ __forceinline__ uint32_t det_legal(const DetConsts& c, const DetLane& s, const BoardView& b) {
  const LegalCtx x = legal_ctx(c, s, b);
  uint32_t mask = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cur = pin_of(s, x.cp, i);
#pragma unroll
    for (int m = 1; m <= 6; ++m)
      if (legal_one(c, b, x, cur, m)) mask |= 1u << (i * 6 + (m - 1));
  }
  // & valid_actions (action_set > 0) per move column
  uint32_t col = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) col |= x.avail << (i * 6);
  return mask & col;
}

// The legality mask of a game held in LDS by G lanes (G = 4, 8, 16 or 32; lane a of the game, t = threadIdx.x):
// lane a checks actions a, a + G, ... (legal_one) and each ballot delivers the game's G bits.  Every lane of the
// game must call it; lanes of other games in the wave may be inactive (they contribute zero bits).
template <int G>
__device__ __forceinline__ uint32_t det_legal_g(const DetConsts& c, const LdsLane& s, const BoardView& b, int a, int t) {
  static_assert(G == 4 || G == 8 || G == 16 || G == 32, "lanes per game");
  const LegalCtx x = legal_ctx(c, s, b);
  const int gw = (t & 63) / G;   // this game's slot in the wave
  uint32_t mask = 0;
#pragma unroll
  for (int it = 0; it < (24 + G - 1) / G; ++it) {
    const int act = a + G * it;
    const int i = act / 6, m = act % 6 + 1;
    const bool ok = act < 24 && legal_one(c, b, x, pin_of(s, x.cp, i < 4 ? i : 0), m) && ((x.avail >> (m - 1)) & 1u);
    const unsigned long long bal = __ballot(ok);
    mask |= (uint32_t)((bal >> (G * gw)) & ((1ull << G) - 1ull)) << (G * it);
  }
  return mask & 0xFFFFFFu;
}

// `games` consecutive games' SoA rows (from game g0) to LDS, transposed per game: board[gi][cell] and the
// state row [gi][kStateRow] (pins [0, 16), action set [16, 40), cp 40, done 41, reward 42); consecutive threads
// on consecutive games of one SoA row, so the global loads are coalesced.  det_rows_store is the way back.
constexpr int kStateRow = 48;
template <int NG>
__device__ __forceinline__ void det_rows_load(const DetConsts& c, const muz_detmadn_soa& st, int g0, int games,
                                              int8_t (*sboard)[kCells], int8_t (*sstate)[kStateRow], int t, int nt) {
  const int S = st.stride, P = c.P;
  for (int i = t; i < kCells * NG; i += nt) {
    const int row = i / NG, gi = i - row * NG;
    if (gi < games) sboard[gi][row] = st.board[row * S + g0 + gi];
  }
  for (int i = t; i < kStateRow * NG; i += nt) {
    const int row = i / NG, gi = i - row * NG;
    if (gi >= games) continue;
    int8_t v = 0;
    if (row < 16) v = row < 4 * P ? st.pins[row * S + g0 + gi] : (int8_t)-1;
    else if (row < 40) v = row - 16 < 6 * P ? st.action_set[(row - 16) * S + g0 + gi] : (int8_t)0;
    else if (row == 40) v = st.current_player[g0 + gi];
    else if (row == 41) v = st.done[g0 + gi] ? 1 : 0;
    else if (row == 42) v = st.reward[g0 + gi];
    sstate[gi][row] = v;
  }
}
template <int NG>
__device__ __forceinline__ void det_rows_store(const DetConsts& c, const muz_detmadn_soa& st, int g0, int games,
                                               const int8_t (*sboard)[kCells], const int8_t (*sstate)[kStateRow],
                                               int t, int nt) {
  const int S = st.stride, P = c.P;
  for (int i = t; i < kCells * NG; i += nt) {
    const int row = i / NG, gi = i - row * NG;
    if (gi < games) st.board[row * S + g0 + gi] = sboard[gi][row];
  }
  for (int i = t; i < kStateRow * NG; i += nt) {
    const int row = i / NG, gi = i - row * NG;
    if (gi >= games) continue;
    const int8_t v = sstate[gi][row];
    if (row < 16) {
      if (row < 4 * P) st.pins[row * S + g0 + gi] = v;
    } else if (row < 40) {
      if (row - 16 < 6 * P) st.action_set[(row - 16) * S + g0 + gi] = v;
    } else if (row == 40) {
      st.current_player[g0 + gi] = v;
    } else if (row == 41) {
      st.done[g0 + gi] = (uint8_t)v;
    } else if (row == 42) {
      st.reward[g0 + gi] = v;
    }
  }
}

constexpr int kEncStride = 96;   // per game: rel[56] + constant channel values at [56 + ch]
// Observation bytes from a staged game (the env rounds' phase 2, the self-play encode): per game at
// senc + gl * kEncStride, rel[56] = the rolled cell's owner relative to the current player (kRelEmpty for an empty
// cell), then the constant channels' values at [56 + ch] (det_enc_stage).  A game's C x 56 = 16 (28P + 7) bytes
// split into halves of 8 cells of one channel (56 = 7 x 8), two per 16-byte chunk.  A board channel's 4 output bytes are ONE byte permute of the 4 staged rel bytes through the
// channel's 4-entry table (byte r = 1 if relative owner r is on the channel); kRelEmpty = 12 is v_perm_b32's
// constant-zero selector.  (Per-byte predicates compiled to ~700 divergent-branch instructions per chunk and
// made this phase ~80 % of the launch: profiles/r3_env_breakdown.log.)
constexpr uint32_t kRelEmpty = 12u;
__device__ __forceinline__ uint32_t det_obs_table(int ch, int P, bool teams) {
  const uint32_t player = 1u << (8 * (ch & 3));                                        // ch < P: one-hot
  const uint32_t own = teams ? 0x00010001u : 0x00000001u;                              // ch == P
  const uint32_t opp = teams ? 0x01000100u : (P == 2 ? 0x00000100u : P == 3 ? 0x00010100u : 0x01010100u);
  return ch < P ? player : ch == P ? own : opp;
}
__device__ __forceinline__ uint2 det_obs_half(const uint8_t* e, int m, int P, bool teams) {
  const int ch = m / 7, w0 = (m - ch * 7) * 8;
  const uint2 rw = *reinterpret_cast<const uint2*>(e + w0);
  const uint32_t tab = det_obs_table(ch, P, teams);
  const uint32_t cv = (uint32_t)e[kCells + ch] * 0x01010101u;   // constant channel (ignored below P + 2)
  const bool board = ch < P + 2;
  return make_uint2(board ? __builtin_amdgcn_perm(0u, tab, rw.x) : cv, board ? __builtin_amdgcn_perm(0u, tab, rw.y) : cv);
}
// Stage one game's encode inputs into e (kEncStride bytes) with G lanes (lane a: cells a, a + G, ... and constant
// channels P + 2 + a, ...): encode_board (deterministic_madn.py:395-438) split into the board part and the rest.
template <int G, class Lane>
__device__ __forceinline__ void det_enc_stage(const DetConsts& c, const Lane& s, const BoardView& b, uint8_t* e, int a) {
  const int P = c.P, C = 8 * P + 2;
  for (int w = a; w < kCells; w += G) {
    const int src = (w < kTrack) ? fmodp(w + kDist * s.cp, kTrack) : kTrack + fmodp((w - kTrack) + 4 * s.cp, 16);
    const int v = b.at(src);
    e[w] = v < 0 ? (uint8_t)kRelEmpty : (uint8_t)mod_small(v - s.cp, P);
  }
  auto none = [](int) { return 0; };
  for (int ch = P + 2 + a; ch < C; ch += G) e[kCells + ch] = (uint8_t)det_encode_value(c, s, ch, 0, none);
}

// set_pins_on_board (deterministic_madn.py:259-271) into the lane's LDS board.
template <class Lane>
__device__ __forceinline__ void rebuild_board(const DetConsts& c, const Lane& s, const BoardView& b) {
  for (int cell = 0; cell < kCells; ++cell) b.set(cell, -1);
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (p < c.P) {
        const int pos = lane_pin(s, p * 4 + k);
        if (pos >= 0 && pos < kCells) b.set(pos, p);
      }
}

// env_step (deterministic_madn.py:170-257) with (pin, move), given the state's legal mask (valid_action of
// the same state; callers that already hold it skip the second legality pass).  Updates s and the LDS board.
// Returns the reward; s.done / s.reward / s.cp updated like the reference.
template <class Lane>
__device__ __forceinline__ int det_step_masked(const DetConsts& c, Lane& s, const BoardView& b, int pin, int move,
                                               const uint32_t legal) {
  const uint32_t F = c.flags;
  const int player_id = s.cp;
  const int cp = sub_player(c, b, player_id);
  const int mi = jidx(move - 1, 6);
  const int pi = jidx(pin, 4);
  const bool invalid = ((legal >> (pi * 6 + mi)) & 1u) == 0u;
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = cst(c.target, cp);
  const int g0 = goal_of(c, cp, 0);
  const int cur = pin_of(s, cp, pi);
  const int moved = cur + move;
  const int fitted = fmodp(moved, kTrack);
  const int x = moved - tgt - mt;
  const bool in_goal = (cur == g0) | (cur == goal_of(c, cp, 1)) | (cur == goal_of(c, cp, 2)) |
                       (cur == goal_of(c, cp, 3));
  const bool a = in_goal ? goal_path_free(c, b, cp, cur - g0, moved - g0 + 1) : goal_path_free(c, b, cp, -1, x);
  const int gx = goal_of(c, cp, jidx(x - 1, 4));
  const bool A = (b.at(gx) != cp) && (has(F, R_JUMP_GOAL) || a);
  int new_pos;
  if (cur == -1)
    new_pos = cst(c.start, cp);
  else if (in_goal)
    new_pos = moved;
  else if (4 >= x && x > 0 && A && cur <= tgt)
    new_pos = gx;
  else
    new_pos = fitted;
  const int pin_at = b.at(jidx(new_pos, kCells));
  if (!invalid) {
    if (pin_at != -1 && (pin_at != cp || has(F, R_FRIENDLY))) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int pj = lane_pin(s, j);
        int x = ((j >> 2) == pin_at && pj == new_pos) ? -1 : pj;
        asm volatile("" : "+v"(x));
        lane_set_pin(s, j, x);
      }
    }
    set_pin(s, cp * 4 + pi, new_pos);
    rebuild_board(c, s, b);
  }
  // action set: decrement [cp, move-1]; if the row empties, refill row current_player of the
  // PRE-step set (refill_action_set, lines 235-240 + 281).
  const int curr = aset_of(s, cp, mi);
  const int nv = (invalid || curr == 0) ? curr : curr - 1;
  bool row_empty = true;
#pragma unroll
  for (int m = 0; m < 6; ++m) row_empty &= ((m == mi) ? nv : aset_of(s, cp, m)) == 0;
  if (row_empty) {
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      int x = (j / 6 == player_id) ? 4 : lane_aset(s, j);
      asm volatile("" : "+v"(x));
      lane_set_aset(s, j, x);
    }
  } else {
    set_aset(s, cp * 6 + mi, nv);
  }
  const uint32_t w = winners(c, b);
  const int reward = s.done ? 0 : (invalid ? -1 : (int)((w >> cp) & 1u));
  const int done = (s.done || w != 0u) ? 1 : 0;
  s.cp = (done || (has(F, R_BONUS_6) && move == 6)) ? player_id : mod_small(player_id + 1, c.P);
  s.done = done;
  s.reward = reward;
  return reward;
}

__device__ __forceinline__ int det_step(const DetConsts& c, DetLane& s, const BoardView& b, int pin, int move) {
  return det_step_masked(c, s, b, pin, move, det_legal(c, s, b));
}

// no_step (deterministic_madn.py:283-297).
template <class Lane>
__device__ __forceinline__ void det_nostep(const DetConsts& c, Lane& s) {
#pragma unroll
  for (int j = 0; j < 24; ++j) {
    int x = (j / 6 == s.cp) ? 4 : lane_aset(s, j);
    asm volatile("" : "+v"(x));
    lane_set_aset(s, j, x);
  }
  s.cp = mod_small(s.cp + 1, c.P);
}

// ---- SoA load / store -----------------------------------------------------------------
__device__ __forceinline__ void det_load(const DetConsts& c, const muz_detmadn_soa& st, int g, DetLane& s,
                                         const BoardView& b) {
  const int S = st.stride;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = st.pins[min(j, c.P * 4 - 1) * S + g];
    s.pins[j] = (j < c.P * 4) ? v : -1;
  }
#pragma unroll
  for (int j = 0; j < 24; ++j) {
    const int v = st.action_set[min(j, c.P * 6 - 1) * S + g];
    s.aset[j] = (j < c.P * 6) ? v : 0;
  }
  s.cp = st.current_player[g];
  s.done = st.done[g] ? 1 : 0;
  s.reward = st.reward[g];
  for (int cell = 0; cell < kCells; ++cell) b.set(cell, st.board[cell * S + g]);
}

__device__ __forceinline__ void det_store(const DetConsts& c, const muz_detmadn_soa& st, int g, const DetLane& s,
                                          const BoardView& b, bool board_dirty) {
  const int S = st.stride;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (j < c.P * 4) st.pins[j * S + g] = (int8_t)s.pins[j];
#pragma unroll
  for (int j = 0; j < 24; ++j)
    if (j < c.P * 6) st.action_set[j * S + g] = (int8_t)s.aset[j];
  st.current_player[g] = (int8_t)s.cp;
  st.done[g] = (uint8_t)s.done;
  st.reward[g] = (int8_t)s.reward;
  if (board_dirty)
    for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = (int8_t)b.at(cell);
}

// encode_board value of channel ch at cell w (deterministic_madn.py:395-438).
// C = P + 2 + P + 6P; board cell lookups go through `cell_owner(src)`.
template <class Lane, class CellFn>
__device__ __forceinline__ int det_encode_value(const DetConsts& c, const Lane& s, int ch, int w,
                                                CellFn cell_owner) {
  const int P = c.P, cp = s.cp;
  const int src = (w < kTrack) ? fmodp(w + kDist * cp, kTrack) : kTrack + fmodp((w - kTrack) + 4 * cp, 16);
  const int v = cell_owner(src);
  auto rolled = [&](int i) { return mod_small(i + cp, P); };
  if (ch < P) return v == rolled(ch) ? 1 : 0;
  if (ch == P) {  // team channel
    if (has(c.flags, R_TEAMS)) return (v == rolled(0) ? 1 : 0) + (v == rolled(2) ? 1 : 0);
    return v == rolled(0) ? 1 : 0;
  }
  if (ch == P + 1) {  // opponent channel
    if (has(c.flags, R_TEAMS)) return (v == rolled(1) ? 1 : 0) + (v == rolled(3) ? 1 : 0);
    int n = 0;
    for (int i = 1; i < P; ++i) n += (v == rolled(i)) ? 1 : 0;
    return n;
  }
  if (ch < 2 * P + 2) {  // pins at home of rolled player
    const int p = rolled(ch - P - 2);
    int n = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) n += (pin_of(s, p, k) == -1) ? 1 : 0;
    return n;
  }
  const int a = ch - (2 * P + 2);
  return aset_of(s, rolled(a / 6), a % 6);
}

}  // namespace muz
