// Batched deterministic-MADN environment kernels + their C ABI (include/muz.h).
// One board per lane; 256-lane workgroups; the lane's board is staged in LDS.
#include "detmadn.hpp"
#include "host_consts.hpp"
#include "rng.hpp"

namespace muz {

constexpr int kEnvBlock = 256;

__global__ __launch_bounds__(kEnvBlock) void k_det_reset(DetConsts c, muz_detmadn_soa st, int n,
                                                       const int32_t* seeds = nullptr) {
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const bool fp = has(c.flags, R_FREE_PIN);
  for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = -1;
  for (int p = 0; p < c.P; ++p) {
    for (int k = 0; k < 4; ++k) st.pins[(p * 4 + k) * S + g] = (int8_t)((fp && k == 0) ? c.start[p] : -1);
    for (int m = 0; m < 6; ++m) st.action_set[(p * 6 + m) * S + g] = 4;
    if (fp) st.board[c.start[p] * S + g] = (int8_t)p;
  }
  st.current_player[g] =
      (int8_t)(c.starting_player >= 0 ? c.starting_player : start_seat((unsigned long long)(uint32_t)seeds[g], c.P));
  st.reward[g] = 0;
  st.done[g] = 0;
}

__global__ __launch_bounds__(kEnvBlock) void k_det_legal(DetConsts c, muz_detmadn_soa st, uint32_t* legal, int n) {
  __shared__ int8_t sboard[kCells * kEnvBlock];
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  BoardView b{sboard + threadIdx.x, kEnvBlock};
  DetLane s;
  det_load(c, st, g, s, b);
  legal[g] = det_legal(c, s, b);
}

// mode 0: action index (map_action), mode 1: explicit (pin, move)
__global__ __launch_bounds__(kEnvBlock) void k_det_step(DetConsts c, muz_detmadn_soa st, const int32_t* a0,
                                                        const int32_t* a1, int mode, int8_t* reward, uint8_t* done,
                                                        uint32_t* next_legal, int n) {
  __shared__ int8_t sboard[kCells * kEnvBlock];
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  BoardView b{sboard + threadIdx.x, kEnvBlock};
  DetLane s;
  det_load(c, st, g, s, b);
  int pin, move;
  if (mode == 0) {
    const int a = a0[g];
    pin = fdiv(a, 6);
    move = fmodp(a, 6) + 1;
  } else {
    pin = a0[g];
    move = a1[g];
  }
  const int r = det_step(c, s, b, pin, move);
  det_store(c, st, g, s, b, true);
  if (reward) reward[g] = (int8_t)r;
  if (done) done[g] = (uint8_t)s.done;
  if (next_legal) next_legal[g] = det_legal(c, s, b);
}

__global__ __launch_bounds__(kEnvBlock) void k_det_nostep(DetConsts c, muz_detmadn_soa st, int8_t* reward,
                                                          uint8_t* done, int n) {
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const int cp = st.current_player[g];
  for (int m = 0; m < 6; ++m) st.action_set[(cp * 6 + m) * S + g] = 4;
  st.current_player[g] = (int8_t)((cp + 1) % c.P);
  if (reward) reward[g] = 0;
  if (done) done[g] = st.done[g];
}

// One thread per (game, cell): coalesced obs writes along the cell axis.
template <typename T>
__global__ __launch_bounds__(64) void k_det_encode(DetConsts c, muz_detmadn_soa st, T* obs, int n) {
  const int g = blockIdx.x;
  const int w = threadIdx.x;
  if (g >= n || w >= kCells) return;
  const int S = st.stride;
  DetLane s;
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
  const int C = 8 * c.P + 2;
  T* out = obs + (size_t)g * C * kCells;
  auto owner = [&](int cell) { return (int)st.board[cell * S + g]; };
  for (int ch = 0; ch < C; ++ch) out[ch * kCells + w] = (T)det_encode_value(c, s, ch, w, owner);
}


// ---- random-play env round (SURVEY §8(d)(b'): the env-only micro-benchmark, and a random-play actor) -----
// One env-step per game: the k-th legal action of the mask left by the previous round (k = floor(u * count),
// u from the counter RNG of (seed ^ kDetRandomStream, game, turn)), env_step -- or no_step when nothing is
// legal --, an in-place env_reset of a game that finished, the next legal mask, and the int8 observation of
// the state the next round acts on (encode_board, deterministic_madn.py:395-438).
// Phase 1 is lane per game (256 games per workgroup; SoA loads / stores coalesced) and stages per game, in
// LDS, each rolled cell's owner relative to the current player (rel = (owner - cp) mod P, kRelEmpty empty)
// and the constant channels (home counts, action sets).  Phase 2 (det_obs_write) writes the workgroup's
// 256 x C x 56 contiguous observation bytes as 16-byte chunks, consecutive threads on consecutive chunks.
constexpr int kRoundBlock = 256;
constexpr unsigned long long kDetRandomStream = 0xD37A11D0ull;

// Phase 2 of the env rounds (the staging and chunk helpers are in detmadn.hpp): `games` consecutive games'
// int8 observations, contiguous in `out`, one 16-byte chunk per thread and iteration.
__device__ __forceinline__ void det_obs_write(const DetConsts& c, const uint8_t* senc, int games, int8_t* out, int t,
                                              int nthreads) {
  const int P = c.P, C = 8 * P + 2;
  const bool teams = has(c.flags, R_TEAMS);
  const int per = C * 7 / 2;   // 16-byte chunks per game
  const float inv = 1.0f / (float)per;
  uint4* o = reinterpret_cast<uint4*>(out);
  for (int q = t; q < games * per; q += nthreads) {
    int gl = (int)(((float)q + 0.5f) * inv);
    gl -= gl * per > q ? 1 : 0;
    gl += (gl + 1) * per <= q ? 1 : 0;
    const int m = 2 * (q - gl * per);
    const uint8_t* e = senc + gl * kEncStride;
    const uint2 lo = det_obs_half(e, m, P, teams), hi = det_obs_half(e, m + 1, P, teams);
    o[q] = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

__global__ __launch_bounds__(kRoundBlock) void k_det_round(DetConsts c, muz_detmadn_soa st, uint32_t* legal,
                                                           unsigned long long seed, int turn, int8_t* obs,
                                                           int8_t* reward, uint8_t* done, int n) {
  __shared__ int8_t sboard[kCells * kRoundBlock];
  __shared__ __attribute__((aligned(16))) uint8_t senc[kRoundBlock * kEncStride];
  const int g = blockIdx.x * kRoundBlock + threadIdx.x;
  const int P = c.P, C = 8 * P + 2;
  if (g < n) {
    BoardView b{sboard + threadIdx.x, kRoundBlock};
    DetLane s;
    det_load(c, st, g, s, b);
    const uint32_t lb = legal[g];
    const int cnt = __popc(lb);
    int r = 0;
    if (cnt == 0) {
      det_nostep(c, s);
    } else {
      const float u = u24(mix64(game_key(seed ^ kDetRandomStream, g, turn)));
      int k = (int)(u * (float)cnt);
      k = k >= cnt ? cnt - 1 : k;
      uint32_t x = lb;
      for (int j = 0; j < k; ++j) x &= x - 1;   // drop the k lowest set bits
      const int a = __ffs(x) - 1;
      r = det_step_masked(c, s, b, a / 6, a % 6 + 1, lb);   // lb: this state's mask (the round contract)
    }
    const int fin = s.done;
    if (fin) {   // env_reset in place with the batch's rules (deterministic_madn.py:42-120)
      const bool fp = has(c.flags, R_FREE_PIN);
      for (int cell = 0; cell < kCells; ++cell) b.set(cell, -1);
#pragma unroll
      for (int j = 0; j < 16; ++j) s.pins[j] = (fp && (j & 3) == 0 && (j >> 2) < P) ? c.start[j >> 2] : -1;
#pragma unroll
      for (int j = 0; j < 24; ++j) s.aset[j] = j < 6 * P ? 4 : 0;
      if (fp)
        for (int p = 0; p < P; ++p) b.set(c.start[p], p);
      s.cp = c.starting_player;
      s.done = 0;
      s.reward = 0;
    }
    det_store(c, st, g, s, b, true);
    legal[g] = det_legal(c, s, b);
    if (reward) reward[g] = (int8_t)r;
    if (done) done[g] = (uint8_t)fin;
    if (obs) {   // stage this game's encode inputs
      uint8_t* e = senc + threadIdx.x * kEncStride;
      uint32_t wv = 0;
      for (int w = 0; w < kCells; ++w) {
        const int src = (w < kTrack) ? fmodp(w + kDist * s.cp, kTrack) : kTrack + fmodp((w - kTrack) + 4 * s.cp, 16);
        const int v = b.at(src);
        const uint32_t rel = v < 0 ? kRelEmpty : (uint32_t)mod_small(v - s.cp, P);
        wv |= rel << (8 * (w & 3));
        if ((w & 3) == 3) {
          *reinterpret_cast<uint32_t*>(e + (w & ~3)) = wv;
          wv = 0;
        }
      }
      auto none = [](int) { return 0; };
      for (int ch = P + 2; ch < C; ++ch) e[kCells + ch] = (uint8_t)det_encode_value(c, s, ch, 0, none);
    }
  }
  if (!obs) return;
  __syncthreads();
  const int g0 = blockIdx.x * kRoundBlock;
  det_obs_write(c, senc, min(kRoundBlock, n - g0), obs + (size_t)g0 * C * kCells, threadIdx.x, kRoundBlock);
}

// The same round with one game per G lanes (G = 4, 8, 16 or 32), for batches too small to fill the GPU one game per
// lane (4096 games = 16 workgroups of k_det_round on 16 of 256 CUs) and to shorten each lane's serial chain: the
// workgroup copies its NG = 256 / G games' SoA rows into LDS with coalesced, game-contiguous loads (transposed to a
// per-game row), lane 0 of a game picks the action and applies env_step / no_step / env_reset (the same device
// functions as k_det_round, on the game's LDS copy), lane a checks actions a, a + G, ... (legal_one, the body of
// det_legal; one ballot per G actions forms the mask), stages cells a, a + G, ... and constant channels P + 2 + a,
// ... of the encode, and the workgroup writes the state rows back and its NG x C x 56 contiguous observation bytes
// as 8-byte chunks, both fully coalesced.  Same results, bit for bit.
constexpr int kWideBlock = 256;

template <int G>
__global__ __launch_bounds__(kWideBlock) void k_det_round_g(DetConsts c, muz_detmadn_soa st, uint32_t* legal,
                                                            unsigned long long seed, int turn, int8_t* obs,
                                                            int8_t* reward, uint8_t* done, int n) {
  static_assert(G == 4 || G == 8 || G == 16 || G == 32, "lanes per game");
  constexpr int NG = kWideBlock / G;
  __shared__ int8_t sboard[NG][kCells];
  __shared__ int8_t sstate[NG][kStateRow];
  __shared__ __attribute__((aligned(16))) uint8_t senc[NG][kEncStride];
  const int t = threadIdx.x;
  const int lg = t / G, a = t % G;
  const int g0 = blockIdx.x * NG;
  const int games = min(NG, n - g0);
  const int g = g0 + lg;
  const bool valid = lg < games;   // uniform over the game's G lanes
  const int P = c.P, C = 8 * P + 2;
  det_rows_load<NG>(c, st, g0, games, sboard, sstate, t, kWideBlock);
  int8_t* sp = sstate[lg];
  const BoardView b{sboard[lg], 1};
  const uint32_t lb = valid ? legal[g] : 0u;
  __syncthreads();
  if (valid && a == 0) {   // the game's step on its LDS rows (pins / action set by index, not in VGPRs)
    LdsLane s{sp, sp[40], sp[41], sp[42]};
    const int cnt = __popc(lb);
    int r = 0;
    if (cnt == 0) {
      det_nostep(c, s);
    } else {
      const float u = u24(mix64(game_key(seed ^ kDetRandomStream, g, turn)));
      int k = (int)(u * (float)cnt);
      k = k >= cnt ? cnt - 1 : k;
      uint32_t x = lb;
      for (int j = 0; j < k; ++j) x &= x - 1;
      const int act = __ffs(x) - 1;
      r = det_step_masked(c, s, b, act / 6, act % 6 + 1, lb);
    }
    const int fin = s.done;
    if (fin) {   // env_reset in place (as k_det_round)
      const bool fp = has(c.flags, R_FREE_PIN);
      for (int cell = 0; cell < kCells; ++cell) b.set(cell, -1);
#pragma unroll
      for (int j = 0; j < 16; ++j) sp[j] = (int8_t)((fp && (j & 3) == 0 && (j >> 2) < P) ? c.start[j >> 2] : -1);
#pragma unroll
      for (int j = 0; j < 24; ++j) sp[16 + j] = (int8_t)(j < 6 * P ? 4 : 0);
      if (fp)
        for (int p = 0; p < P; ++p) b.set(c.start[p], p);
      s.cp = c.starting_player;
      s.done = 0;
      s.reward = 0;
    }
    sp[40] = (int8_t)s.cp;
    sp[41] = (int8_t)s.done;
    sp[42] = (int8_t)s.reward;
    if (reward) reward[g] = (int8_t)r;
    if (done) done[g] = (uint8_t)fin;
  }
  __syncthreads();
  if (valid) {
    const LdsLane s{sp, sp[40], 0, 0};
    // next legal mask: lane a checks actions a, a + G, ...; the game's G bits of each ballot
    const uint32_t mask = det_legal_g<G>(c, s, b, a, t);
    if (a == 0) legal[g] = mask;
    // encode staging: rolled cells' owner relative to cp, constant channels
    if (obs) det_enc_stage<G>(c, s, b, senc[lg], a);
  }
  // (lanes of invalid games, last workgroup only, skip the ballots: inactive lanes contribute zero bits)
  __syncthreads();
  det_rows_store<NG>(c, st, g0, games, sboard, sstate, t, kWideBlock);   // LDS -> SoA rows, coalesced
  if (!obs) return;
  det_obs_write(c, &senc[0][0], games, obs + (size_t)g0 * C * kCells, t, kWideBlock);
}

// ---- evaluation agents (MuZero_det_MADN/evaluate_agent.py) --------------------------------------------
// mode 0: the random agent (do_random, 770-775: jax.random.categorical over 0 / -1e9 logits of the legal
// actions); mode 1: the rule-based agent (do_rule_based, 777-864): per action pin*6 + m a score
//   base  = abundance[a // 4]   (jnp.repeat(counts / max(sum counts, 1), 4): indexed by a // 4, as written)
//   + goal_bonus  if the pin (not yet in the goal area) lands on one of the player's goal cells
//   + out_many / out_few (>= 2 / < 2 pins at home) if a home pin moves to the start
//   + hit_bonus   if the pin moves onto an opponent pin (teams: the partner is no opponent)
// with landing cells from cur + m, m = 0..5 (jnp.arange(6), as written) and the UNSUBSTITUTED current
// player; illegal actions -inf; action = argmax(score / temperature + gumbel) -- jax.random.categorical,
// the Gumbel draw from the engine's counter RNG (seed ^ kPolicyStream, game, turn, action).  -1 when
// nothing is legal.
__global__ __launch_bounds__(256) void k_det_policy(DetConsts c, muz_detmadn_soa st, const uint32_t* legal, int mode,
                                                    muz_rule_agent ag, unsigned long long seed, int turn,
                                                    const int32_t* game_id, int32_t* action, int n) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const uint32_t lb = legal[g];
  if (lb == 0u) {
    action[g] = -1;
    return;
  }
  const int gid = game_id ? game_id[g] : g;
  const unsigned long long key = game_key(seed ^ kPolicyStream, gid, turn);
  auto gum = [&](int a) { return policy_gumbel(key, a); };
  int best = -1;
  float bv = -INFINITY;
  if (mode == 0) {
    for (int a = 0; a < 24; ++a) {
      const float l = ((lb >> a) & 1u) ? 0.0f : -1e9f;
      const float v = l + gum(a);
      if (v > bv) {
        bv = v;
        best = a;
      }
    }
    action[g] = best;
    return;
  }
  const int P = c.P, cp = st.current_player[g];
  const int mt = has(c.flags, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = cst(c.target, cp), start = cst(c.start, cp);
  int pins[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) pins[j] = j < P * 4 ? st.pins[min(j, P * 4 - 1) * S + g] : -1;
  int home = 0;
  for (int k = 0; k < 4; ++k) home += rsel(pins, cp * 4 + k) < 0 ? 1 : 0;
  int counts[6];
  int total = 0;
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    counts[m] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) counts[m] += (lb >> (i * 6 + m)) & 1u;
    total += counts[m];
  }
  const float denom = fmaxf((float)total, 1.0f);
  const int partner = has(c.flags, R_TEAMS) ? (cp + 2) % 4 : -1;
  for (int i = 0; i < 4; ++i) {
    const int cur = rsel(pins, cp * 4 + i);
    for (int m = 0; m < 6; ++m) {
      const int a = i * 6 + m;
      if (((lb >> a) & 1u) == 0u) continue;
      const int moved = cur + m;
      const int x = moved - tgt - mt;
      int np;
      if (cur < 0) np = start;
      else if (cur >= kTrack) np = moved;
      else if (4 >= x && x > 0 && cur <= tgt) np = goal_of(c, cp, jidx(x - 1, 4));
      else np = fmodp(moved, kTrack);
      const int ab = a >> 2;   // jnp.repeat(action_abundance, 4)[a]
      int cab = 0;
#pragma unroll
      for (int q = 0; q < 6; ++q) cab = q == ab ? counts[q] : cab;
      const float base = (float)cab / denom;
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
      const float score = ((base + gb) + ob) + hb;
      const float v = score / ag.temperature + gum(a);
      if (v > bv) {
        bv = v;
        best = a;
      }
    }
  }
  action[g] = best;
}

// variant 0 = by batch size, 1 = one game per lane (k_det_round), 2 / 3 / 4 / 5 = one game per 32 / 8 / 4 / 16
// lanes (k_det_round_g).  The lane kernel needs >= 256 workgroups of 256 games to fill 256 CUs; below kWideMaxGames
// the G-lane kernel spreads the same games over G x the lanes: G = 32 up to kWide32MaxGames, G = 4 above
// (every variant at 4096 / 65 536 / 2^20 games: profiles/r3_env_variants.log).
constexpr int kWide32MaxGames = 1 << 13;
constexpr int kWideMaxGames = 1 << 16;
static inline unsigned nblocks(int n, int b) { return (unsigned)((n + b - 1) / b); }

int launch_det_round(const DetConsts& c, const muz_detmadn_soa& st, uint32_t* legal, unsigned long long seed, int turn,
                     int8_t* obs, int8_t* reward, uint8_t* done, int n, int variant, hipStream_t s) {
  if (variant == 0) variant = n <= kWide32MaxGames ? 2 : n <= kWideMaxGames ? 4 : 1;
  switch (variant) {
    case 2:
      k_det_round_g<32><<<nblocks(n, kWideBlock / 32), kWideBlock, 0, s>>>(c, st, legal, seed, turn, obs, reward, done, n);
      break;
    case 3:
      k_det_round_g<8><<<nblocks(n, kWideBlock / 8), kWideBlock, 0, s>>>(c, st, legal, seed, turn, obs, reward, done, n);
      break;
    case 4:
      k_det_round_g<4><<<nblocks(n, kWideBlock / 4), kWideBlock, 0, s>>>(c, st, legal, seed, turn, obs, reward, done, n);
      break;
    case 5:
      k_det_round_g<16><<<nblocks(n, kWideBlock / 16), kWideBlock, 0, s>>>(c, st, legal, seed, turn, obs, reward, done, n);
      break;
    default:
      k_det_round<<<nblocks(n, kRoundBlock), kRoundBlock, 0, s>>>(c, st, legal, seed, turn, obs, reward, done, n);
  }
  return muz_last_launch_error();
}

}  // namespace muz

using namespace muz;


extern "C" {

int muz_detmadn_reset(const muz_rules* rules, muz_detmadn_soa st, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n);
  if (n == 0) return MUZ_OK;
  k_det_reset<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, n);
  return muz_last_launch_error();
}

int muz_detmadn_reset_seeded(const muz_rules* rules, muz_detmadn_soa st, const int32_t* seeds, int32_t n,
                             void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c, true);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && seeds);
  if (n == 0) return MUZ_OK;
  k_det_reset<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, n, seeds);
  return muz_last_launch_error();
}

int muz_detmadn_legal(const muz_rules* rules, muz_detmadn_soa st, uint32_t* legal, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && legal);
  if (n == 0) return MUZ_OK;
  k_det_legal<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, legal, n);
  return muz_last_launch_error();
}

int muz_detmadn_step(const muz_rules* rules, muz_detmadn_soa st, const int32_t* action, int8_t* reward,
                     uint8_t* done, uint32_t* next_legal, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && action);
  if (n == 0) return MUZ_OK;
  k_det_step<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, action, nullptr, 0, reward, done,
                                                                            next_legal, n);
  return muz_last_launch_error();
}

int muz_detmadn_step_pin_move(const muz_rules* rules, muz_detmadn_soa st, const int32_t* pin, const int32_t* move,
                              int8_t* reward, uint8_t* done, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && pin && move);
  if (n == 0) return MUZ_OK;
  k_det_step<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, pin, move, 1, reward, done,
                                                                            nullptr, n);
  return muz_last_launch_error();
}

int muz_detmadn_nostep(const muz_rules* rules, muz_detmadn_soa st, int8_t* reward, uint8_t* done, int32_t n,
                       void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n);
  if (n == 0) return MUZ_OK;
  k_det_nostep<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, reward, done, n);
  return muz_last_launch_error();
}

int muz_detmadn_encode_f32(const muz_rules* rules, muz_detmadn_soa st, float* obs, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && obs);
  if (n == 0) return MUZ_OK;
  k_det_encode<float><<<n, 64, 0, (hipStream_t)stream>>>(c, st, obs, n);
  return muz_last_launch_error();
}

int muz_detmadn_encode_i8(const muz_rules* rules, muz_detmadn_soa st, int8_t* obs, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && obs);
  if (n == 0) return MUZ_OK;
  k_det_encode<int8_t><<<n, 64, 0, (hipStream_t)stream>>>(c, st, obs, n);
  return muz_last_launch_error();
}

int muz_detmadn_random_round(const muz_rules* rules, muz_detmadn_soa st, uint32_t* legal_bits, uint64_t seed,
                             int32_t turn, int8_t* obs, int8_t* reward, uint8_t* done, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && legal_bits && ((uintptr_t)obs & 15u) == 0);
  if (n == 0) return MUZ_OK;
  return launch_det_round(c, st, legal_bits, seed, turn, obs, reward, done, n, 0, (hipStream_t)stream);
}

int muz_detmadn_random_round_variant(const muz_rules* rules, muz_detmadn_soa st, uint32_t* legal_bits, uint64_t seed,
                                     int32_t turn, int8_t* obs, int8_t* reward, uint8_t* done, int32_t n,
                                     int32_t variant, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && legal_bits && ((uintptr_t)obs & 15u) == 0 && variant >= 0 && variant <= 5);
  if (n == 0) return MUZ_OK;
  return launch_det_round(c, st, legal_bits, seed, turn, obs, reward, done, n, variant, (hipStream_t)stream);
}

int muz_detmadn_policy_action(const muz_rules* rules, muz_detmadn_soa st, const uint32_t* legal_bits, int32_t mode,
                              const muz_rule_agent* agent, uint64_t seed, int32_t turn, const int32_t* game_id,
                              int32_t* action, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && legal_bits && action && (mode == 0 || mode == 1));
  MUZ_HOST_CHECK(mode == 0 || (agent && agent->temperature > 0.f));
  if (n == 0) return MUZ_OK;
  const muz_rule_agent ag = agent ? *agent : muz_rule_agent{1.f, 0.f, 0.f, 0.f, 0.f};
  k_det_policy<<<nblocks(n, 256), 256, 0, (hipStream_t)stream>>>(c, st, legal_bits, mode, ag, seed, turn, game_id,
                                                                 action, n);
  return muz_last_launch_error();
}

}  // extern "C"
