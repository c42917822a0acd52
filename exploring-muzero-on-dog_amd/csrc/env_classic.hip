// Batched classic-MADN environment kernels + their C ABI (include/muz.h).
// One board per lane; 256-lane workgroups; the lane's board is staged in LDS.
#include "classic.hpp"
#include "host_consts.hpp"
#include "rng.hpp"

namespace muz {

constexpr int kClsBlock = 256;

__global__ __launch_bounds__(kClsBlock) void k_cls_reset(DetConsts c, muz_classic_soa st, int n,
                                                       const int32_t* seeds = nullptr) {
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const bool fp = has(c.flags, R_FREE_PIN);
  for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = -1;
  for (int p = 0; p < c.P; ++p) {
    for (int k = 0; k < 4; ++k) st.pins[(p * 4 + k) * S + g] = (int8_t)((fp && k == 0) ? c.start[p] : -1);
    if (fp) st.board[c.start[p] * S + g] = (int8_t)p;
  }
  st.current_player[g] =
      (int8_t)(c.starting_player >= 0 ? c.starting_player : start_seat((unsigned long long)(uint32_t)seeds[g], c.P));
  st.reward[g] = 0;
  st.done[g] = 0;
  st.die[g] = 0;
}

__global__ __launch_bounds__(kClsBlock) void k_cls_set_die(muz_classic_soa st, const int32_t* die, int n) {
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g < n) st.die[g] = (int8_t)die[g];
}

// Pins, current player and the 4 goal cells of that player are all the soft-lock test needs, so the
// dice kernels read the board straight from HBM (no LDS staging).
__device__ __forceinline__ bool cls_soft_locked_soa(const DetConsts& c, const muz_classic_soa& st, int g) {
  const int S = st.stride;
  const int cp = st.current_player[g];
  int out = 0;
  for (int k = 0; k < 4; ++k) out += (st.pins[(cp * 4 + k) * S + g] != -1) ? 1 : 0;
  if (out == 0) return true;
  bool locked = true;
  for (int k = 4 - out; k < 4; ++k) locked &= st.board[goal_of(c, cp, k) * S + g] == cp;
  return locked;
}

__global__ __launch_bounds__(kClsBlock) void k_cls_dice_probs(DetConsts c, muz_classic_soa st, float* probs,
                                                              uint8_t* soft, int n) {
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  const bool sl = cls_soft_locked_soa(c, st, g);
  float p[6];
  cls_dice_probs(c, sl, p);
  for (int i = 0; i < 6; ++i) probs[(size_t)g * 6 + i] = p[i];
  if (soft) soft[g] = sl ? 1 : 0;
}

__global__ __launch_bounds__(kClsBlock) void k_cls_throw_die(DetConsts c, muz_classic_soa st, const float* uniform,
                                                             int32_t* die_out, int n) {
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  float p[6];
  cls_dice_probs(c, cls_soft_locked_soa(c, st, g), p);
  const int d = cls_choice(p, uniform[g]);
  st.die[g] = (int8_t)d;
  if (die_out) die_out[g] = d;
}

__global__ __launch_bounds__(kClsBlock) void k_cls_legal(DetConsts c, muz_classic_soa st, uint32_t* legal, int n) {
  __shared__ int8_t sboard[kCells * kClsBlock];
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  BoardView b{sboard + threadIdx.x, kClsBlock};
  ClsLane s;
  cls_load(c, st, g, s, b);
  legal[g] = cls_legal(c, s, b);
}

__global__ __launch_bounds__(kClsBlock) void k_cls_step(DetConsts c, muz_classic_soa st, const int32_t* pin,
                                                        int8_t* reward, uint8_t* done, int n) {
  __shared__ int8_t sboard[kCells * kClsBlock];
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  BoardView b{sboard + threadIdx.x, kClsBlock};
  ClsLane s;
  cls_load(c, st, g, s, b);
  const int r = cls_step(c, s, b, pin[g]);
  cls_store(c, st, g, s, b);
  if (reward) reward[g] = (int8_t)r;
  if (done) done[g] = (uint8_t)s.done;
}

__global__ __launch_bounds__(kClsBlock) void k_cls_nostep(DetConsts c, muz_classic_soa st, int8_t* reward,
                                                          uint8_t* done, int n) {
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  st.current_player[g] = (int8_t)((st.current_player[g] + 1) % c.P);
  if (reward) reward[g] = 0;
  if (done) done[g] = st.done[g];
}

// One thread per (game, cell): coalesced obs writes along the cell axis.
template <typename T>
__global__ __launch_bounds__(64) void k_cls_encode(DetConsts c, muz_classic_soa st, T* obs, int n) {
  const int g = blockIdx.x;
  const int w = threadIdx.x;
  if (g >= n || w >= kCells) return;
  const int S = st.stride;
  ClsLane s;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = st.pins[min(j, c.P * 4 - 1) * S + g];
    s.pins[j] = (j < c.P * 4) ? v : -1;
  }
  s.cp = st.current_player[g];
  s.die = st.die[g];
  const int C = 2 * c.P + 3;
  T* out = obs + (size_t)g * C * kCells;
  auto owner = [&](int cell) { return (int)st.board[cell * S + g]; };
  for (int ch = 0; ch < C; ++ch) out[ch * kCells + w] = (T)cls_encode_value(c, s, ch, w, owner);
}

// ---- evaluation agents (MuZero_Classic_MADN/evaluate_agent_stochastic.py play_eval_loop_jitted) -----------------
// mode 0: the random agent (do_random, 800-804: jax.random.categorical over 0 / -1e9 logits of the legal pins);
// mode 1: the rule-based agent (do_rule_based, 806-866): per pin i a score
//   goal_bonus  if the pin (not yet in the goal area) lands on one of the player's goal cells
//   + out_many / out_few (>= 2 / < 2 pins at home) if a home pin moves to the start
//   + hit_bonus if the pin moves onto an opponent pin (teams: the partner is no opponent)
// (base score 0) with the landing cell of cur + die (the UNSUBSTITUTED current player's pins, as written); illegal
// pins -inf; action = argmax(score / temperature + gumbel) with the counter Gumbel draws of det's agents
// (policy_gumbel, actions 0..3).  -1 when no pin is legal.
__global__ __launch_bounds__(kClsBlock) void k_cls_policy(DetConsts c, muz_classic_soa st, const uint32_t* legal,
                                                          int mode, muz_rule_agent ag, unsigned long long seed, int turn,
                                                          const int32_t* game_id, int32_t* action, int n) {
  const int g = blockIdx.x * kClsBlock + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const uint32_t lb = legal[g] & 15u;
  if (lb == 0u) {
    action[g] = -1;
    return;
  }
  const unsigned long long key = game_key(seed ^ kPolicyStream, game_id ? game_id[g] : g, turn);
  int best = -1;
  float bv = -INFINITY;
  if (mode == 0) {
    for (int a = 0; a < 4; ++a) {
      const float v = (((lb >> a) & 1u) ? 0.0f : -1e9f) + policy_gumbel(key, a);
      if (v > bv) {
        bv = v;
        best = a;
      }
    }
    action[g] = best;
    return;
  }
  const int P = c.P, cp = st.current_player[g], die = st.die[g];
  const int mt = has(c.flags, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = cst(c.target, cp), start = cst(c.start, cp);
  int pins[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) pins[j] = j < P * 4 ? st.pins[min(j, P * 4 - 1) * S + g] : -1;
  int home = 0;
  for (int k = 0; k < 4; ++k) home += rsel(pins, cp * 4 + k) < 0 ? 1 : 0;
  const int partner = has(c.flags, R_TEAMS) ? (cp + 2) % 4 : -1;
  for (int i = 0; i < 4; ++i) {
    if (((lb >> i) & 1u) == 0u) continue;
    const int cur = rsel(pins, cp * 4 + i);
    const int moved = cur + die;
    const int x = moved - tgt - mt;
    int np;
    if (cur < 0) np = start;
    else if (cur >= kTrack) np = moved;
    else if (4 >= x && x > 0 && cur <= tgt) np = goal_of(c, cp, jidx(x - 1, 4));
    else np = fmodp(moved, kTrack);
    bool in_goal = false;
#pragma unroll
    for (int h = 0; h < 4; ++h) in_goal |= np == goal_of(c, cp, h);
    const float gb = (in_goal && cur < kTrack) ? ag.goal_bonus : 0.0f;
    const float ob = (cur < 0 && np == start) ? (home >= 2 ? ag.out_many : ag.out_few) : 0.0f;
    bool hit = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int p = j >> 2;
      hit |= p < P && p != cp && p != partner && pins[j] == np;
    }
    const float hb = (np != cur && hit) ? ag.hit_bonus : 0.0f;
    const float score = ((0.0f + gb) + ob) + hb;
    const float v = score / ag.temperature + policy_gumbel(key, i);
    if (v > bv) {
      bv = v;
      best = i;
    }
  }
  action[g] = best;
}

}  // namespace muz

using namespace muz;

static inline unsigned cls_blocks(int n) { return (unsigned)((n + kClsBlock - 1) / kClsBlock); }

#define CLS_PROLOGUE(extra)                          \
  DetConsts c;                                       \
  int rc = make_det_consts(rules, &c);               \
  if (rc) return rc;                                 \
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && extra); \
  if (n == 0) return MUZ_OK;

extern "C" {

int muz_classic_reset(const muz_rules* rules, muz_classic_soa st, int32_t n, void* stream) {
  CLS_PROLOGUE(true)
  k_cls_reset<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, n);
  return muz_last_launch_error();
}

int muz_classic_reset_seeded(const muz_rules* rules, muz_classic_soa st, const int32_t* seeds, int32_t n,
                             void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c, true);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && seeds);
  if (n == 0) return MUZ_OK;
  k_cls_reset<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, n, seeds);
  return muz_last_launch_error();
}

int muz_classic_set_die(const muz_rules* rules, muz_classic_soa st, const int32_t* die, int32_t n, void* stream) {
  CLS_PROLOGUE(die != nullptr)
  k_cls_set_die<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(st, die, n);
  return muz_last_launch_error();
}

int muz_classic_dice_probs(const muz_rules* rules, muz_classic_soa st, float* probs, uint8_t* soft_locked, int32_t n,
                           void* stream) {
  CLS_PROLOGUE(probs != nullptr)
  k_cls_dice_probs<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, probs, soft_locked, n);
  return muz_last_launch_error();
}

int muz_classic_throw_die(const muz_rules* rules, muz_classic_soa st, const float* uniform, int32_t* die_out, int32_t n,
                          void* stream) {
  CLS_PROLOGUE(uniform != nullptr)
  k_cls_throw_die<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, uniform, die_out, n);
  return muz_last_launch_error();
}

int muz_classic_legal(const muz_rules* rules, muz_classic_soa st, uint32_t* legal, int32_t n, void* stream) {
  CLS_PROLOGUE(legal != nullptr)
  k_cls_legal<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, legal, n);
  return muz_last_launch_error();
}

int muz_classic_step(const muz_rules* rules, muz_classic_soa st, const int32_t* pin, int8_t* reward, uint8_t* done,
                     int32_t n, void* stream) {
  CLS_PROLOGUE(pin != nullptr)
  k_cls_step<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, pin, reward, done, n);
  return muz_last_launch_error();
}

int muz_classic_nostep(const muz_rules* rules, muz_classic_soa st, int8_t* reward, uint8_t* done, int32_t n,
                       void* stream) {
  CLS_PROLOGUE(true)
  k_cls_nostep<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, reward, done, n);
  return muz_last_launch_error();
}

int muz_classic_policy_action(const muz_rules* rules, muz_classic_soa st, const uint32_t* legal_bits, int32_t mode,
                              const muz_rule_agent* agent, uint64_t seed, int32_t turn, const int32_t* game_id,
                              int32_t* action, int32_t n, void* stream) {
  CLS_PROLOGUE(legal_bits && action && (mode == 0 || mode == 1) && (mode == 0 || agent))
  muz_rule_agent ag{};
  if (mode == 1) {
    ag = *agent;
    MUZ_HOST_CHECK(ag.temperature > 0.f);
  }
  k_cls_policy<<<cls_blocks(n), kClsBlock, 0, (hipStream_t)stream>>>(c, st, legal_bits, mode, ag,
                                                                     (unsigned long long)seed, turn, game_id, action, n);
  return muz_last_launch_error();
}

int muz_classic_encode_f32(const muz_rules* rules, muz_classic_soa st, float* obs, int32_t n, void* stream) {
  CLS_PROLOGUE(obs != nullptr)
  k_cls_encode<float><<<n, 64, 0, (hipStream_t)stream>>>(c, st, obs, n);
  return muz_last_launch_error();
}

int muz_classic_encode_i8(const muz_rules* rules, muz_classic_soa st, int8_t* obs, int32_t n, void* stream) {
  CLS_PROLOGUE(obs != nullptr)
  k_cls_encode<int8_t><<<n, 64, 0, (hipStream_t)stream>>>(c, st, obs, n);
  return muz_last_launch_error();
}

}  // extern "C"
