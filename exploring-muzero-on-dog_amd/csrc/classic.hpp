// Classic MADN rules as per-lane device functions (one board per wavefront lane).
//
// Restates MADN/classic_madn.py (reference) for the GPU: valid_action 367-461, env_step 257-337,
// no_step 353-365, encode_board 463-497, is_soft_locked 180-206, dice_probabilities 208-228,
// throw_die 230-242 (jax.random.choice with p, uniform made explicit).  Shares the rule constants,
// board view, winner and goal-path helpers with the deterministic variant (detmadn.hpp): the two
// reference files implement those identically.
#pragma once
#include "detmadn.hpp"

namespace muz {

struct ClsLane {
  int pins[16];   // [p*4 + k]
  int cp;         // current_player (unsubstituted)
  int done;
  int reward;
  int die;
};

__device__ __forceinline__ int cpin(const ClsLane& s, int p, int k) { return rsel(s.pins, p * 4 + k); }

__device__ __forceinline__ bool in_goal_of(const DetConsts& c, int p, int pos) {
  return (pos == goal_of(c, p, 0)) | (pos == goal_of(c, p, 1)) | (pos == goal_of(c, p, 2)) | (pos == goal_of(c, p, 3));
}

// valid_action (classic_madn.py:367-461) -> 4-bit mask over the (substituted) player's pins.
__device__ __forceinline__ uint32_t cls_legal(const DetConsts& c, const ClsLane& s, const BoardView& b) {
  const uint32_t F = c.flags;
  const int cp = sub_player(c, b, s.cp);
  const int tgt = cst(c.target, cp);
  const int g0 = goal_of(c, cp, 0), g3 = goal_of(c, cp, 3);
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int start_cp = cst(c.start, cp);
  const int die = s.die;
  bool pos[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pos[q] = (q < c.P) ? (b.at(cst(c.start, q)) == q) : false;
  const bool pos_cp = pos[0] & (cp == 0) | pos[1] & (cp == 1) | pos[2] & (cp == 2) | pos[3] & (cp == 3);
  // pins at home: die in {1, 6} (start_on_1) or {-1, 6}, and own start not occupied by own pin (455-459)
  const bool home_ok = (die == 6 || (die == 1 && has(F, R_START_ON_1))) && !pos_cp;
  uint32_t mask = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cur = cpin(s, cp, i);
    bool res;
    if (cur == -1) {
      res = home_ok;
    } else {
      const int moved = cur + die;
      const int fitted = fmodp(moved, kTrack);
      int x = moved - tgt - mt;
      res = (b.at(fitted) != cp) || has(F, R_FRIENDLY);
      const int nsb = mod_small(fdiv(cur, kDist) + 1, c.P);   // fdiv(cur, 10) + 1 in [0, 6]
      const int nsa_j = jidx(fdiv(fitted, kDist), c.P);
      const bool trav = cst(c.start, jidx(nsb, c.P)) == cst(c.start, nsa_j);
      const bool pos_a = pos[0] & (nsa_j == 0) | pos[1] & (nsa_j == 1) | pos[2] & (nsa_j == 2) | pos[3] & (nsa_j == 3);
      if (has(F, R_START_BLOCK) && trav) res = (!pos_a || cur == start_cp) && res;
      if (mt && has(F, R_START_BLOCK) && trav && pos_a) x = 0;
      if (!has(F, R_CIRCULAR) && cur <= tgt && (x > 4 || (x == 0 && mt))) res = false;
      if (4 >= x && x > 0 && cur <= tgt) {
        const bool A = has(F, R_CIRCULAR) && res;
        const bool B = b.at(goal_of(c, cp, jidx(x - 1, 4))) != cp;
        const bool C = has(F, R_JUMP_GOAL) || goal_path_free(c, b, cp, -1, x);
        res = A || (B && C);
      }
      if (in_goal_of(c, cp, cur)) {
        const bool D = has(F, R_JUMP_GOAL) || goal_path_free(c, b, cp, cur - g0, moved - g0 + 1);
        res = (moved <= g3) && (b.at(jidx(moved, kCells)) != cp) && D;
      }
    }
    if (res) mask |= 1u << i;
  }
  return mask;
}

__device__ __forceinline__ void cls_rebuild_board(const DetConsts& c, const ClsLane& s, const BoardView& b) {
  for (int cell = 0; cell < kCells; ++cell) b.set(cell, -1);
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (p < c.P) {
        const int pos = s.pins[p * 4 + k];
        if (pos >= 0 && pos < kCells) b.set(pos, p);
      }
}

// env_step (classic_madn.py:257-337): move pin `pin` of the substituted player by s.die, given the state's
// legal mask (valid_action of the same state and die; cls_step computes it).
__device__ __forceinline__ int cls_step_masked(const DetConsts& c, ClsLane& s, const BoardView& b, int pin,
                                               const uint32_t legal) {
  const uint32_t F = c.flags;
  const int player_id = s.cp;
  const int cp = sub_player(c, b, player_id);
  const int pi = jidx((int)(int8_t)pin, 4);
  const bool invalid = ((legal >> pi) & 1u) == 0u;
  const int move = s.die;
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = cst(c.target, cp);
  const int g0 = goal_of(c, cp, 0);
  const int cur = cpin(s, cp, pi);
  const int moved = cur + move;
  const int fitted = fmodp(moved, kTrack);
  const int x = moved - tgt - mt;
  const bool in_goal = in_goal_of(c, cp, cur);
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
      for (int j = 0; j < 16; ++j) {   // (selects + asm guard: a folded a[i] store demotes pins to scratch)
        int x = ((j >> 2) == pin_at && s.pins[j] == new_pos) ? -1 : s.pins[j];
        asm volatile("" : "+v"(x));
        s.pins[j] = x;
      }
    }
    rset(s.pins, cp * 4 + pi, new_pos);
    cls_rebuild_board(c, s, b);
  }
  const uint32_t w = winners(c, b);
  const int reward = s.done ? 0 : (invalid ? -1 : (int)((w >> cp) & 1u));
  const int done = (s.done || w != 0u) ? 1 : 0;
  s.cp = (done || (has(F, R_BONUS_6) && move == 6)) ? player_id : mod_small(player_id + 1, c.P);
  s.done = done;
  s.reward = reward;
  return reward;
}

__device__ __forceinline__ int cls_step(const DetConsts& c, ClsLane& s, const BoardView& b, int pin) {
  return cls_step_masked(c, s, b, pin, cls_legal(c, s, b));
}

// is_soft_locked (classic_madn.py:180-206): the UNSUBSTITUTED current player's pins out of the house
// all sit on the last goal cells.
__device__ __forceinline__ bool cls_soft_locked(const DetConsts& c, const ClsLane& s, const BoardView& b) {
  const int cp = s.cp;
  int out = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) out += (cpin(s, cp, k) != -1) ? 1 : 0;
  if (out == 0) return true;
  bool locked = true;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    if (g >= 4 - out) locked &= b.at(goal_of(c, cp, g)) == cp;
  return locked;
}

// dice_probabilities (classic_madn.py:208-228), the reference's fp32 constants (12-18).
__device__ __forceinline__ void cls_dice_probs(const DetConsts& c, bool soft_locked, float (&p)[6]) {
  if (soft_locked && has(c.flags, R_DICE_RETHROW)) {
    if (has(c.flags, R_START_ON_1)) {
      const float e = (float)(76.0 / 216.0), m = (float)(16.0 / 216.0);
      p[0] = e; p[1] = m; p[2] = m; p[3] = m; p[4] = m; p[5] = e;
    } else {
      const float e = (float)(91.0 / 216.0), m = (float)(25.0 / 216.0);
      p[0] = m; p[1] = m; p[2] = m; p[3] = m; p[4] = m; p[5] = e;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 6; ++i) p[i] = (float)(1.0 / 6.0);
  }
}

// jax.random.choice([1..6], p=p) from an explicit uniform u in [0, 1):
// cum = cumsum(p); r = cum[5] * (1 - u); die = 1 + searchsorted_left(cum, r).
__device__ __forceinline__ int cls_choice(const float (&p)[6], float u) {
  float cum[6];
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    acc = acc + p[i];
    cum[i] = acc;
  }
  const float r = cum[5] * (1.0f - u);
  int idx = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) idx += (cum[i] < r) ? 1 : 0;
  return (idx > 5 ? 5 : idx) + 1;
}

// ---- SoA load / store -----------------------------------------------------------------
__device__ __forceinline__ void cls_load(const DetConsts& c, const muz_classic_soa& st, int g, ClsLane& s,
                                         const BoardView& b) {
  const int S = st.stride;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = st.pins[min(j, c.P * 4 - 1) * S + g];
    s.pins[j] = (j < c.P * 4) ? v : -1;
  }
  s.cp = st.current_player[g];
  s.done = st.done[g] ? 1 : 0;
  s.reward = st.reward[g];
  s.die = st.die[g];
  for (int cell = 0; cell < kCells; ++cell) b.set(cell, st.board[cell * S + g]);
}

__device__ __forceinline__ void cls_store(const DetConsts& c, const muz_classic_soa& st, int g, const ClsLane& s,
                                          const BoardView& b) {
  const int S = st.stride;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (j < c.P * 4) st.pins[j * S + g] = (int8_t)s.pins[j];
  st.current_player[g] = (int8_t)s.cp;
  st.done[g] = (uint8_t)s.done;
  st.reward[g] = (int8_t)s.reward;
  for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = (int8_t)b.at(cell);
}

// encode_board value of channel ch at cell w (classic_madn.py:463-497); C = 2P + 3.
template <class CellFn>
__device__ __forceinline__ int cls_encode_value(const DetConsts& c, const ClsLane& s, int ch, int w, CellFn cell_owner) {
  const int P = c.P, cp = s.cp;
  const int src = (w < kTrack) ? fmodp(w + kDist * cp, kTrack) : kTrack + fmodp((w - kTrack) + 4 * cp, 16);
  const int v = cell_owner(src);
  auto rolled = [&](int i) { return mod_small(i + cp, P); };
  if (ch < P) return v == rolled(ch) ? 1 : 0;
  if (ch == P) {
    if (has(c.flags, R_TEAMS)) return (v == rolled(0) ? 1 : 0) + (v == rolled(2) ? 1 : 0);
    return v == rolled(0) ? 1 : 0;
  }
  if (ch == P + 1) {
    if (has(c.flags, R_TEAMS)) return (v == rolled(1) ? 1 : 0) + (v == rolled(3) ? 1 : 0);
    int n = 0;
    for (int i = 1; i < P; ++i) n += (v == rolled(i)) ? 1 : 0;
    return n;
  }
  if (ch < 2 * P + 2) {
    const int p = rolled(ch - P - 2);
    int n = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) n += (cpin(s, p, k) == -1) ? 1 : 0;
    return n;
  }
  return s.die;
}

}  // namespace muz
