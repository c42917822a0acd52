// Native self-play driver for deterministic MADN: play_n_games_v3 / play_batch_of_games_jitted
// (MuZero_det_MADN/game_agent.py:50-192) as a host loop of stream-ordered HIP launches.
//
// Per turn: legal masks + active flags for every game -> deterministic device compaction of the
// games that search (has a legal move) -> encode their observations -> root inference ->
// persistent Gumbel search -> env_step / no_step + trajectory records.  Unlike the reference's
// vmap-of-cond, finished games and no-move turns cost no network work, and there is no host round
// trip inside a turn: batch sizes live on the device (`counts`), surplus workgroups exit early.
// The host checks the active-game count two turns late (pinned memory + events), so the GPU queue
// never drains; the at most two trailing turns it launches find no active game and record nothing.
#include "detmadn.hpp"
#include "host_consts.hpp"
#include "launch.hpp"
#include "turn_ledger.hpp"
#include "compact.hpp"

#include <algorithm>

namespace muz {

// lane kernels' workgroup size; 64 / 128 measured within noise of 256 (profiles/r1g_sp_block_ab.log)
constexpr int kSpBlock = 256;
#ifndef MUZ_SP_FUSED_HEAD
#define MUZ_SP_FUSED_HEAD 1   // the turn head as one launch (k_sp_head); 0: refill / flags / compact / encode (A/B)
#endif

// Legal masks + flags of every lane, one game per kFlagLanes lanes (a lane per game would leave a 4096-game batch
// on 16 of 256 CUs, its launch one lane's 24 serial legality checks): the workgroup copies its games' SoA rows into
// LDS (coalesced), and each game's lanes run its checks in parallel (det_legal_g, one ballot per 32 actions).
// lane_game (streaming driver only): game number of each lane, -1 = idle; a game whose record is full
// (idx == T, the reference's max_steps) stops like a finished one.
constexpr int kFlagLanes = 32;
__global__ __launch_bounds__(kSpBlock) void k_sp_flags_g(DetConsts c, muz_detmadn_soa st, uint32_t* legal,
                                                         int32_t* flag, int n, const int32_t* lane_game,
                                                         const int32_t* idx, int T) {
  constexpr int G = kFlagLanes, NG = kSpBlock / G;
  __shared__ int8_t sboard[NG][kCells];
  __shared__ int8_t sstate[NG][kStateRow];
  const int t = threadIdx.x, lg = t / G, a = t % G;
  const int g0 = blockIdx.x * NG, games = min(NG, n - g0), g = g0 + lg;
  det_rows_load<NG>(c, st, g0, games, sboard, sstate, t, kSpBlock);
  __syncthreads();
  if (lg >= games) return;   // (uniform over a game's lanes)
  if (sstate[lg][41] || (lane_game && (lane_game[g] < 0 || idx[lane_game[g]] >= T))) {
    if (a == 0) {
      flag[g] = 0;
      legal[g] = 0;
    }
    return;
  }
  const LdsLane s{sstate[lg], sstate[lg][40], 0, 0};
  const uint32_t l = det_legal_g<G>(c, s, BoardView{sboard[lg], 1}, a, t);
  if (a == 0) {
    legal[g] = l;
    flag[g] = l ? 1 : 2;
  }
}

// Observation of every searching game (compacted order: slot sl plays lane list[sl]) as fp32 for root inference +
// its int8 trajectory record; one game per kFlagLanes lanes: the game's lanes gather its SoA bytes into LDS, stage
// the encode (det_enc_stage: rel[56] + constant channels) and write both outputs from the staging -- fp32 as
// float4 per 4 cells of a channel (56 = 14 x 4; 4 bytes = one v_perm_b32 through the channel table), int8 as
// 16-byte chunks -- consecutive lanes on consecutive chunks of the game's contiguous block.
__global__ __launch_bounds__(kSpBlock) void k_sp_encode_g(DetConsts c, muz_detmadn_soa st, const int32_t* list,
                                                          const int32_t* counts, const uint32_t* legal,
                                                          uint32_t* legal_c, float* obs, int8_t* traj_obs,
                                                          const int32_t* idx, int T, const int32_t* lane_game) {
  constexpr int G = kFlagLanes, NG = kSpBlock / G;
  __shared__ int8_t sboard[NG][kCells];
  __shared__ int8_t sstate[NG][kStateRow];
  __shared__ __attribute__((aligned(16))) uint8_t senc[NG][kEncStride];
  const int cnt = counts[0];
  if ((int)blockIdx.x * NG >= cnt) return;   // (uniform over the workgroup)
  const int t = threadIdx.x, lg = t / G, a = t % G;
  const int sl = blockIdx.x * NG + lg;
  const bool valid = sl < cnt;   // uniform over a game's lanes
  const int S = st.stride, P = c.P, C = 8 * P + 2;
  const int g = valid ? list[sl] : 0;
  if (valid) {
    for (int cell = a; cell < kCells; cell += G) sboard[lg][cell] = st.board[cell * S + g];
    if (a < 16) sstate[lg][a] = a < 4 * P ? st.pins[a * S + g] : (int8_t)-1;
    if (a < 24) sstate[lg][16 + a] = a < 6 * P ? st.action_set[a * S + g] : (int8_t)0;
    if (a == 0) {
      sstate[lg][40] = st.current_player[g];
      legal_c[sl] = legal[g];
    }
  }
  __syncthreads();
  if (valid) det_enc_stage<G>(c, LdsLane{sstate[lg], sstate[lg][40], 0, 0}, BoardView{sboard[lg], 1}, senc[lg], a);
  __syncthreads();
  if (!valid) return;
  const bool teams = has(c.flags, R_TEAMS);
  const uint8_t* e = senc[lg];
  float4* o = reinterpret_cast<float4*>(obs + (size_t)sl * C * kCells);
  for (int q = a; q < C * 14; q += G) {   // 4 cells of one channel per float4
    const int ch = q / 14, w0 = (q - ch * 14) * 4;
    const uint32_t rel4 = *reinterpret_cast<const uint32_t*>(e + w0);
    const uint32_t v4 = ch < P + 2 ? __builtin_amdgcn_perm(0u, det_obs_table(ch, P, teams), rel4)
                                   : (uint32_t)e[kCells + ch] * 0x01010101u;
    o[q] = make_float4((float)(v4 & 0xFFu), (float)((v4 >> 8) & 0xFFu), (float)((v4 >> 16) & 0xFFu),
                       (float)(v4 >> 24));
  }
  const int gn = lane_game ? lane_game[g] : g;   // trajectory row of this lane's game
  uint4* to = reinterpret_cast<uint4*>(traj_obs + ((size_t)gn * T + idx[gn]) * C * kCells);
  for (int q = a; q < C * 7 / 2; q += G) {
    const uint2 lo = det_obs_half(e, 2 * q, P, teams), hi = det_obs_half(e, 2 * q + 1, P, teams);
    to[q] = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// Apply the searched action (env_step) or no_step, and write the trajectory record (game_agent.py:79-141): one
// game per kFlagLanes lanes, like k_sp_flags_g -- the workgroup's SoA rows go through LDS both ways (coalesced),
// lane 0 of a game steps it on its LDS rows (LdsLane), its lanes copy the 24 action weights into the record.
// The apply of one game's searched action (or no_step) on its LDS rows and its trajectory record; lane a of the
// game's G lanes, f / sl / leg: the game's flag, slot and legal mask of the turn being applied.
template <int G>
__device__ __forceinline__ void sp_apply_game(const DetConsts& c, int8_t* sp, int8_t* board, int f, int sl, uint32_t leg,
                                              int gn, int tt, const int32_t* s_action, const float* s_weights,
                                              const float* s_value, const muz_traj& tr, int a) {
  const int T = tr.max_steps;
  const size_t rec = (size_t)gn * T + tt;
  if (f == 1 && a < MUZ_DET_ACTIONS)
    tr.pol[rec * MUZ_DET_ACTIONS + a] = s_weights[(size_t)sl * MUZ_DET_ACTIONS + a];
  if (f != 0 && a == 0) {
    LdsLane s{sp, sp[40], sp[41], sp[42]};
    const BoardView b{board, 1};
    const bool teams = has(c.flags, R_TEAMS);
    const int cp_before = s.cp;
    const int team_before = teams ? cp_before % 2 : -1;
    int act, rew_cls, disc_cls;
    float val, mask;
    if (f == 1) {
      act = s_action[sl];
      // leg: this state's mask from the flags pass (the state is unchanged since), so no second legality pass
      const int r = det_step_masked(c, s, b, fdiv(act, 6), fmodp(act, 6) + 1, leg);
      const bool nd = s.done != 0;
      const int next_player = s.cp;
      const int next_team = teams ? next_player % 2 : -1;
      rew_cls = (nd && r > 0) ? 2 : ((nd && r < 0) ? 0 : 1);
      disc_cls = nd ? 1 : (teams ? (team_before == next_team ? 2 : 0) : (cp_before == next_player ? 2 : 0));
      val = s_value[sl];
      mask = 1.f;
    } else {
      det_nostep(c, s);   // obs / policy records stay zero (buffers are zeroed per call)
      act = -1;
      rew_cls = 1;
      disc_cls = 1;
      val = 0.f;
      mask = 0.f;
    }
    sp[40] = (int8_t)s.cp;
    sp[41] = (int8_t)s.done;
    sp[42] = (int8_t)s.reward;
    tr.act[rec] = act;
    tr.rew[rec] = rew_cls;
    tr.val[rec] = val;
    tr.mask[rec] = mask;
    tr.player[rec] = cp_before;
    tr.team[rec] = team_before;
    tr.discount[rec] = disc_cls;
    tr.idx[gn] = tt + 1;
  }
}

__global__ __launch_bounds__(kSpBlock) void k_sp_apply_g(DetConsts c, muz_detmadn_soa st, const int32_t* flag,
                                                         const int32_t* slot, const int32_t* s_action,
                                                         const float* s_weights, const float* s_value, muz_traj tr,
                                                         int n, const int32_t* lane_game, const uint32_t* legal) {
  constexpr int G = kFlagLanes, NG = kSpBlock / G;
  __shared__ int8_t sboard[NG][kCells];
  __shared__ int8_t sstate[NG][kStateRow];
  const int t = threadIdx.x, lg = t / G, a = t % G;
  const int g0 = blockIdx.x * NG, games = min(NG, n - g0), g = g0 + lg;
  det_rows_load<NG>(c, st, g0, games, sboard, sstate, t, kSpBlock);
  const int f = lg < games ? flag[g] : 0;
  const int gn = f ? (lane_game ? lane_game[g] : g) : 0;
  const int tt = f ? tr.idx[gn] : 0;   // read by every lane of the game before lane 0 advances it
  __syncthreads();
  if (f) sp_apply_game<G>(c, sstate[lg], sboard[lg], f, slot[g], legal[g], gn, tt, s_action, s_weights, s_value, tr, a);
  __syncthreads();
  det_rows_store<NG>(c, st, g0, games, sboard, sstate, t, kSpBlock);
}

__device__ void det_reset_lane(const DetConsts& c, const muz_detmadn_soa& st, int g) {
  const int S = st.stride;
  const bool fp = has(c.flags, R_FREE_PIN);
  for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = -1;
  for (int p = 0; p < c.P; ++p) {
    for (int k = 0; k < 4; ++k) st.pins[(p * 4 + k) * S + g] = (int8_t)((fp && k == 0) ? c.start[p] : -1);
    for (int m = 0; m < 6; ++m) st.action_set[(p * 6 + m) * S + g] = 4;
    if (fp) st.board[c.start[p] * S + g] = (int8_t)p;
  }
  st.current_player[g] = (int8_t)c.starting_player;
  st.reward[g] = 0;
  st.done[g] = 0;
}

__global__ void k_det_reset_sp(DetConsts c, muz_detmadn_soa st, int n) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  det_reset_lane(c, st, g);
}

// Streaming refill (one workgroup, deterministic): every lane whose game ended (done, or its record is
// full) takes the next unplayed game number in lane order and is reset; lanes left without a game go
// idle (-1).  next[0] = next unplayed game number.
__global__ __launch_bounds__(kScanThreads) void k_ss_refill(DetConsts c, muz_detmadn_soa st, int32_t* lane_game,
                                                            const int32_t* idx, int T, int32_t* next, int num_games,
                                                            int W) {
  __shared__ int part[kScanThreads];
  const int t = threadIdx.x;
  const int chunk = (W + kScanThreads - 1) / kScanThreads;
  const int lo = min(W, t * chunk), hi = min(W, lo + chunk);
  auto ended = [&](int l) {
    const int gn = lane_game[l];
    return gn >= 0 && (st.done[l] || idx[gn] >= T);
  };
  int cnt = 0;
  for (int l = lo; l < hi; ++l) cnt += ended(l);
  part[t] = cnt;
  __syncthreads();
  for (int off = 1; off < kScanThreads; off <<= 1) {
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int base = next[0];
  int r = part[t] - cnt;
  for (int l = lo; l < hi; ++l) {
    if (!ended(l)) continue;
    const int gn = base + r++;
    if (gn < num_games) {
      lane_game[l] = gn;
      det_reset_lane(c, st, l);
    } else {
      lane_game[l] = -1;
    }
  }
  __syncthreads();
  if (t == kScanThreads - 1) next[0] = min(num_games, base + part[t]);
}

// ---- the turn head as one launch (MUZ_SP_FUSED_HEAD, default): refill + flags + compaction + encode ------------
// The four launches above cost ~37 us per turn at 4096 lanes, most of it two single-workgroup scans and kernel
// boundaries (profiles/r5s_kernel_stats.csv).  Here every workgroup (8 lanes) loads its rows once and takes its
// share of the two lane-order counts the head needs -- refilled lanes' game numbers, searching games' slots -- with
// one device atomic each.  The workgroups' order among themselves then decides which lane takes which new game
// number and which slot a searching game gets, but no result: a game's search, records and noise depend on its
// game number and its own step count only (key_game / key_turn), never on its lane or its slot, and the set of game
// numbers handed out per turn is the same (tests/test_gpu_selfplay.py: stream == batch, oracle parity).  (Ordered
// alternatives measured: a decoupled look-back over the 512 workgroups, 262 us serial / 69 us 64-wide -- each poll
// an agent-scope load across XCDs.)
// counts: this turn's [searching, active, -, arrivals]; the next turn's four (the other parity) are zeroed here.
// 32 games per workgroup (128 workgroups at 4096 lanes): the same-address atomics serialise, so fewer, larger
// workgroups take fewer of them.
constexpr int kHeadBlock = 1024;

struct SpHead {
  uint32_t* legal;
  int32_t* flag;
  int32_t* list;
  int32_t* slot;
  int32_t* counts;        // this turn's four counters (zeroed by the previous turn's head or the driver)
  int32_t* counts_next;   // the next turn's four, zeroed here
  uint32_t* legal_c;
  float* obs;
  int8_t* traj_obs;
  int32_t* host_counts;   // the turn's pinned ledger slot (device-visible), or null
  // APPLY: the previous turn's search results, applied first (what k_sp_apply_g did at the end of that turn)
  const int32_t* s_action;
  const float* s_weights;
  const float* s_value;
  muz_traj tr;
};

// STREAM: k_ss_refill's lane refill first (lane_game / next); otherwise lane g plays game g.
// APPLY: the previous turn's apply first (k_sp_apply_g, on the rows this launch loads anyway): one launch and one
// round trip of the rows fewer per turn.
template <bool STREAM, bool APPLY>
__global__ __launch_bounds__(kHeadBlock) void k_sp_head(DetConsts c, muz_detmadn_soa st, int n, const int32_t* idx, int T,
                                                      int32_t* lane_game, int32_t* next, int num_games, SpHead o) {
  constexpr int G = kFlagLanes, NG = kHeadBlock / G;
  __shared__ int8_t sboard[NG][kCells];
  __shared__ int8_t sstate[NG][kStateRow];
  __shared__ __attribute__((aligned(16))) uint8_t senc[NG][kEncStride];
  __shared__ int s_gn[NG], s_f[NG], s_pre, s_reset;
  const int t = threadIdx.x, lg = t / G, a = t % G;
  const int b = blockIdx.x, nb = gridDim.x;
  const int g0 = b * NG, games = min(NG, n - g0), g = g0 + lg;
  det_rows_load<NG>(c, st, g0, games, sboard, sstate, t, kHeadBlock);
  int fprev = 0, slprev = 0, gnprev = 0, ttprev = 0;
  uint32_t legprev = 0;
  if (APPLY && lg < games) {   // the previous turn's flag / slot / mask, read before this turn's passes rewrite them
    fprev = o.flag[g];
    if (fprev) {
      slprev = o.slot[g];
      legprev = o.legal[g];
      gnprev = STREAM ? lane_game[g] : g;
      ttprev = idx[gnprev];
    }
  }
  if (t < NG) {
    s_gn[t] = -1;
    s_f[t] = 0;
  }
  if (t == 0) s_reset = 0;
  if (b == 0 && t < 4) o.counts_next[t] = 0;
  __syncthreads();
  if (APPLY) {
    if (fprev)
      sp_apply_game<G>(c, sstate[lg], sboard[lg], fprev, slprev, legprev, gnprev, ttprev, o.s_action, o.s_weights,
                       o.s_value, o.tr, a);
    __syncthreads();   // (the refill below reads the advanced idx and the new done flags)
  }
  if constexpr (STREAM) {
    // refill (k_ss_refill): every lane whose game ended takes the next unplayed game number (next[0] counts the
    // numbers handed out, possibly past num_games: those lanes go idle)
    if (t < games) {
      const int gn = lane_game[g0 + t];
      s_gn[t] = gn;
      s_f[t] = gn >= 0 && (sstate[t][41] || idx[gn] >= T);
    }
    __syncthreads();
    if (t == 0) {
      int cnt = 0;
      for (int i = 0; i < games; ++i) cnt += s_f[i];
      int r = cnt ? atomicAdd(next, cnt) : 0;
      for (int i = 0; i < games; ++i)
        if (s_f[i]) {
          s_gn[i] = r < num_games ? r : -1;
          s_reset |= r < num_games;
          ++r;
        }
    }
    __syncthreads();
    if (t < games && s_f[t]) lane_game[g0 + t] = s_gn[t];
    if (s_reset) {   // det_reset_lane on the LDS rows of the refilled lanes (stored back below)
      const bool fp = has(c.flags, R_FREE_PIN);
      for (int i = t; i < NG * kCells; i += kHeadBlock) {
        const int gi = i / kCells, cell = i % kCells;
        if (gi < games && s_f[gi] && s_gn[gi] >= 0) {
          int v = -1;
          for (int p = 0; p < c.P; ++p)
            if (fp && cell == c.start[p]) v = p;
          sboard[gi][cell] = (int8_t)v;
        }
      }
      for (int i = t; i < NG * kStateRow; i += kHeadBlock) {
        const int gi = i / kStateRow, r = i % kStateRow;
        if (gi < games && s_f[gi] && s_gn[gi] >= 0) {
          int8_t v = sstate[gi][r];
          if (r < 16) v = r < 4 * c.P ? (int8_t)((fp && (r & 3) == 0) ? c.start[r >> 2] : -1) : (int8_t)-1;
          else if (r < 40) v = r - 16 < 6 * c.P ? (int8_t)4 : (int8_t)0;
          else if (r == 40) v = (int8_t)c.starting_player;
          else if (r == 41 || r == 42) v = 0;
          sstate[gi][r] = v;
        }
      }
    }
    __syncthreads();
    if (t < NG) s_f[t] = 0;
    __syncthreads();
  }
  // flags (k_sp_flags_g): 1 = searches (a legal move), 2 = no move (no_step), 0 = idle
  if (lg < games) {
    const int gn = STREAM ? s_gn[lg] : g;
    const bool idle = sstate[lg][41] || (STREAM && (gn < 0 || idx[gn] >= T));
    uint32_t l = 0;
    int f = 0;
    if (!idle) {   // (uniform over the game's lanes)
      l = det_legal_g<G>(c, LdsLane{sstate[lg], sstate[lg][40], 0, 0}, BoardView{sboard[lg], 1}, a, t);
      f = l ? 1 : 2;
    }
    if (a == 0) {
      o.legal[g] = l;
      o.flag[g] = f;
      s_f[lg] = f;
    }
  }
  __syncthreads();
  // compaction (k_sp_compact): slots of the searching games; counts = (searching, active); the last workgroup to
  // arrive hands the totals to the host ledger
  if (t == 0) {
    int c1 = 0, c2 = 0;
    for (int i = 0; i < games; ++i) {
      c1 += s_f[i] == 1;
      c2 += s_f[i] != 0;
    }
    // (searching, active) as one 64-bit add: counts[0] the low word, counts[1] the high word
    const unsigned long long add = ((unsigned long long)(unsigned)c2 << 32) | (unsigned)c1;
    s_pre = add ? (int)(unsigned)atomicAdd(reinterpret_cast<unsigned long long*>(o.counts), add) : 0;
    if (o.host_counts) {
      __threadfence();
      if (atomicAdd(&o.counts[3], 1) == nb - 1) {
        __threadfence();
        const int tot1 = __hip_atomic_load(&o.counts[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int tot2 = __hip_atomic_load(&o.counts[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&o.host_counts[0], tot1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&o.host_counts[1], tot2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  int sl = -1;
  if (lg < games && s_f[lg] == 1) {
    sl = s_pre;
    for (int i = 0; i < lg; ++i) sl += s_f[i] == 1;
  }
  if (a == 0 && lg < games) {
    o.slot[g] = sl;
    if (sl >= 0) {
      o.list[sl] = g;
      o.legal_c[sl] = o.legal[g];
    }
  }
  // encode (k_sp_encode_g) of this workgroup's searching games at their slots
  if (sl >= 0) det_enc_stage<G>(c, LdsLane{sstate[lg], sstate[lg][40], 0, 0}, BoardView{sboard[lg], 1}, senc[lg], a);
  __syncthreads();
  if (sl >= 0) {
    const int P = c.P, C = 8 * P + 2;
    const bool teams = has(c.flags, R_TEAMS);
    const uint8_t* e = senc[lg];
    float4* ob = reinterpret_cast<float4*>(o.obs + (size_t)sl * C * kCells);
    // channels >= 6 are constant planes (the global features): root inference reads them at cell 0 only
    // (k_root_dense: x[:, 6:, 0]; k_repr_conv reads channels 0..5), so only their first float4 is written
    const int nq = 6 * 14 + (C - 6);
    for (int u = a; u < nq; u += G) {
      const int q = u < 6 * 14 ? u : (u - 6 * 14 + 6) * 14;
      const int ch = q / 14, w0 = (q - ch * 14) * 4;
      const uint32_t rel4 = *reinterpret_cast<const uint32_t*>(e + w0);
      const uint32_t v4 = ch < P + 2 ? __builtin_amdgcn_perm(0u, det_obs_table(ch, P, teams), rel4)
                                     : (uint32_t)e[kCells + ch] * 0x01010101u;
      ob[q] = make_float4((float)(v4 & 0xFFu), (float)((v4 >> 8) & 0xFFu), (float)((v4 >> 16) & 0xFFu),
                          (float)(v4 >> 24));
    }
    const int gn = STREAM ? s_gn[lg] : g;
    uint4* to = reinterpret_cast<uint4*>(o.traj_obs + ((size_t)gn * T + idx[gn]) * C * kCells);
    for (int q = a; q < C * 7 / 2; q += G) {
      const uint2 lo = det_obs_half(e, 2 * q, P, teams), hi = det_obs_half(e, 2 * q + 1, P, teams);
      to[q] = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  }
  if (APPLY || (STREAM && s_reset)) det_rows_store<NG>(c, st, g0, games, sboard, sstate, t, kHeadBlock);
}

struct SpWs {
  void* tree;
  float* conv;
  float* obs;
  uint32_t* legal;
  uint32_t* legal_c;
  int32_t* flag;
  int32_t* slot;
  int32_t* list;
  float* root_logits;
  float* root_value;
  float* root_emb;
  int32_t* action;
  float* weights;
  float* value;
  int32_t* counts;
  int32_t* lane_game;   // streaming driver: game number per lane
  int32_t* next_game;
};

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t sp_carve(char* base, int n, int C, int S, SpWs* w) {
  const size_t n16 = (size_t)((n + 15) / 16 * 16);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += al256(bytes);
    return p;
  };
  SpWs t;
  t.tree = take((size_t)search_workspace_bytes(n, S));
  t.conv = (float*)take(n16 * kConvRowFloats * 4);
  t.obs = (float*)take(n16 * C * kCells * 4);
  t.legal = (uint32_t*)take((size_t)n * 4);
  t.legal_c = (uint32_t*)take((size_t)n * 4);
  t.flag = (int32_t*)take((size_t)n * 4);
  t.slot = (int32_t*)take((size_t)n * 4);
  t.list = (int32_t*)take((size_t)n * 4);
  t.root_logits = (float*)take(n16 * MUZ_DET_ACTIONS * 4);
  t.root_value = (float*)take(n16 * 4);
  t.root_emb = (float*)take(n16 * 256 * 4);
  t.action = (int32_t*)take(n16 * 4);
  t.weights = (float*)take(n16 * MUZ_DET_ACTIONS * 4);
  t.value = (float*)take(n16 * 4);
  t.counts = (int32_t*)take(64);
  t.lane_game = (int32_t*)take((size_t)n * 4);
  t.next_game = (int32_t*)take(64);
  if (w) *w = t;
  return off;
}

__global__ void k_ss_init(DetConsts c, muz_detmadn_soa st, int32_t* lane_game, int32_t* next, int num_games, int W) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l == 0) next[0] = min(num_games, W);
  if (l >= W) return;
  lane_game[l] = l < num_games ? l : -1;
  det_reset_lane(c, st, l);
}

// The turn loop shared by the batch and the streaming driver.  Batch: lane g plays game g for at most T
// turns.  Streaming (lane_game != null): lanes are refilled with the next game number when theirs ends,
// until num_games games have been played.
static int sp_turns(const DetConsts& c, const muz_net_w* w, const muz_search_cfg* cfg, muz_detmadn_soa st, muz_traj tr,
                    int n, const SpWs& ws, const int32_t* lane_game, int num_games, int max_turns, muz_sp_stats* stats,
                    hipStream_t s) {
  const int T = tr.max_steps;
  int rc = MUZ_OK;
  SearchArgs sa;
  sa.S = cfg->num_simulations;
  sa.D = cfg->max_depth;
  sa.max_considered = cfg->max_num_considered;
  sa.value_scale = cfg->value_scale;
  sa.maxvisit_init = cfg->maxvisit_init;
  sa.gumbel_scale = cfg->gumbel_scale;
  sa.seed = cfg->seed;
  sa.key_turn = tr.idx;   // the game's own step count (== the turn for every game of a batch)
  sa.key_game = lane_game;

  TurnLedger led(s, stats != nullptr);
  if ((rc = led.begin())) return rc;
  MUZ_HIP_RET(hipMemsetAsync(ws.counts, 0, 8 * sizeof(int32_t), s));   // both parities of k_sp_head's counters
  int turns = 0;
  bool pending = false;   // a turn's searched actions not applied yet
  rc = MUZ_OK;
  for (int turn = 0; turn < max_turns; ++turn) {
    if (!led.proceed(turn)) break;
    const int nbk = (n + kSpBlock / kFlagLanes - 1) / (kSpBlock / kFlagLanes);
#if MUZ_SP_FUSED_HEAD
    const int nbh = (n + kHeadBlock / kFlagLanes - 1) / (kHeadBlock / kFlagLanes);
    int32_t* const counts = ws.counts + 4 * (turn & 1);   // (the other parity: the next turn's, zeroed by the head)
    // (the ledger's counts reach the host through root inference's first kernel: no last-arrival ticket here)
    int32_t* const host_counts = led.device_slot(turn);
    const SpHead h{ws.legal, ws.flag, ws.list, ws.slot, counts, ws.counts + 4 * ((turn + 1) & 1), ws.legal_c, ws.obs,
                   tr.obs, nullptr, ws.action, ws.weights, ws.value, tr};
    if (lane_game) {
      if (pending)
        k_sp_head<true, true><<<nbh, kHeadBlock, 0, s>>>(c, st, n, tr.idx, T, ws.lane_game, ws.next_game, num_games, h);
      else
        k_sp_head<true, false><<<nbh, kHeadBlock, 0, s>>>(c, st, n, tr.idx, T, ws.lane_game, ws.next_game, num_games, h);
    } else {
      if (pending)
        k_sp_head<false, true><<<nbh, kHeadBlock, 0, s>>>(c, st, n, tr.idx, T, nullptr, nullptr, num_games, h);
      else
        k_sp_head<false, false><<<nbh, kHeadBlock, 0, s>>>(c, st, n, tr.idx, T, nullptr, nullptr, num_games, h);
    }
    pending = false;
    if (!host_counts) led.counts(turn, counts);
#else
    int32_t* const host_counts = nullptr;
    int32_t* const counts = ws.counts;
    if (lane_game)
      k_ss_refill<<<1, kScanThreads, 0, s>>>(c, st, ws.lane_game, tr.idx, T, ws.next_game, num_games, n);
    k_sp_flags_g<<<nbk, kSpBlock, 0, s>>>(c, st, ws.legal, ws.flag, n, lane_game, tr.idx, T);
    k_sp_compact<<<1, kScanThreads, 0, s>>>(ws.flag, n, ws.list, ws.slot, ws.counts);
    led.counts(turn, ws.counts);
    k_sp_encode_g<<<nbk, kSpBlock, 0, s>>>(c, st, ws.list, ws.counts, ws.legal, ws.legal_c, ws.obs, tr.obs, tr.idx,
                                           T, lane_game);
#endif
    if ((rc = muz_last_launch_error())) break;
    if ((rc = launch_root_inference(*w, ws.obs, n, counts, ws.conv, ws.root_logits, ws.root_value, ws.root_emb,
                                    s, host_counts)))
      break;
    if (host_counts) led.counts_written(turn);
    sa.turn = turn;
    led.search_begin(turn);
    if ((rc = launch_gumbel_search(*w, sa, ws.root_logits, ws.root_value, ws.root_emb, ws.legal_c, nullptr, ws.list, n, counts, ws.tree, ws.action, ws.weights,
                                   ws.value, s)))
      break;
    led.search_end(turn);
#if MUZ_SP_FUSED_HEAD
    pending = true;   // applied by the next turn's head (or after the loop)
#else
    k_sp_apply_g<<<nbk, kSpBlock, 0, s>>>(c, st, ws.flag, ws.slot, ws.action, ws.weights, ws.value, tr, n, lane_game,
                                          ws.legal);
#endif
    if ((rc = muz_last_launch_error())) break;
    ++turns;
  }
  if (pending && rc == MUZ_OK) {   // the last launched turn's apply
    k_sp_apply_g<<<(n + kSpBlock / kFlagLanes - 1) / (kSpBlock / kFlagLanes), kSpBlock, 0, s>>>(
        c, st, ws.flag, ws.slot, ws.action, ws.weights, ws.value, tr, n, lane_game, ws.legal);
    rc = muz_last_launch_error();
  }
  led.finish(turns, stats);
  return rc;
}

}  // namespace muz

using namespace muz;

extern "C" {

int64_t muz_selfplay_workspace_bytes(int32_t n, int32_t obs_channels, const muz_search_cfg* cfg) {
  if (!cfg || n < 0) return -1;
  return (int64_t)sp_carve(nullptr, n, obs_channels, cfg->num_simulations, nullptr);
}

int muz_detmadn_selfplay(const muz_rules* rules, const muz_net_w* w, const muz_search_cfg* cfg, muz_detmadn_soa st,
                         muz_traj tr, int32_t n, void* workspace, int64_t workspace_bytes, muz_sp_stats* stats,
                         void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  if (!w || !cfg) return MUZ_E_INVALID;
  if (w->obs_channels != 8 * c.P + 2 || w->num_actions != MUZ_DET_ACTIONS) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && workspace && tr.max_steps > 0 && tr.obs && tr.act && tr.rew &&
                 tr.val && tr.pol && tr.mask && tr.player && tr.team && tr.discount && tr.idx);
  MUZ_HOST_CHECK(((uintptr_t)tr.obs & 15u) == 0 && ((uintptr_t)workspace & 15u) == 0);
  if (cfg->num_simulations < 1 || cfg->num_simulations > 100 || cfg->max_depth < 1 || cfg->max_depth > 64)
    return MUZ_E_UNSUPPORTED;
  if (stats) *stats = muz_sp_stats{};
  MUZ_HOST_CHECK(workspace_bytes >= (int64_t)sp_carve(nullptr, n, w->obs_channels, cfg->num_simulations, nullptr));
  if (n == 0) return MUZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int C = w->obs_channels;
  const int T = tr.max_steps;
  SpWs ws;
  sp_carve((char*)workspace, n, C, cfg->num_simulations, &ws);

  // play_n_games_v3: batch_reset + zeroed buffers (init_buffers, game_agent.py:158-169)
  k_det_reset_sp<<<(n + 255) / 256, 256, 0, s>>>(c, st, n);
  const size_t nt = (size_t)n * T;
  MUZ_HIP_RET(hipMemsetAsync(tr.obs, 0, nt * C * kCells, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.act, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.rew, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.val, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.pol, 0, nt * MUZ_DET_ACTIONS * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.mask, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.player, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.team, 0xFF, nt * 4, s));   // jnp.full(..., -1)
  MUZ_HIP_RET(hipMemsetAsync(tr.discount, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.idx, 0, (size_t)n * 4, s));

  return sp_turns(c, w, cfg, st, tr, n, ws, nullptr, n, T, stats, s);
}

int muz_detmadn_selfplay_stream(const muz_rules* rules, const muz_net_w* w, const muz_search_cfg* cfg,
                                muz_detmadn_soa st, muz_traj tr, int32_t num_games, int32_t lanes, void* workspace,
                                int64_t workspace_bytes, muz_sp_stats* stats, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  if (!w || !cfg) return MUZ_E_INVALID;
  if (w->obs_channels != 8 * c.P + 2 || w->num_actions != MUZ_DET_ACTIONS) return MUZ_E_UNSUPPORTED;
  const int n = lanes;
  MUZ_HOST_CHECK(n >= 0 && num_games >= 0 && st.stride >= n && workspace && tr.max_steps > 0 && tr.obs && tr.act &&
                 tr.rew && tr.val && tr.pol && tr.mask && tr.player && tr.team && tr.discount && tr.idx);
  MUZ_HOST_CHECK(((uintptr_t)tr.obs & 15u) == 0 && ((uintptr_t)workspace & 15u) == 0);
  if (cfg->num_simulations < 1 || cfg->num_simulations > 100 || cfg->max_depth < 1 || cfg->max_depth > 64)
    return MUZ_E_UNSUPPORTED;
  if (stats) *stats = muz_sp_stats{};
  MUZ_HOST_CHECK(workspace_bytes >= (int64_t)sp_carve(nullptr, n, w->obs_channels, cfg->num_simulations, nullptr));
  if (n == 0 || num_games == 0) return MUZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int C = w->obs_channels;
  const int T = tr.max_steps;
  SpWs ws;
  sp_carve((char*)workspace, n, C, cfg->num_simulations, &ws);
  const size_t nt = (size_t)num_games * T;
  MUZ_HIP_RET(hipMemsetAsync(tr.obs, 0, nt * C * kCells, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.act, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.rew, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.val, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.pol, 0, nt * MUZ_DET_ACTIONS * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.mask, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.player, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.team, 0xFF, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.discount, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.idx, 0, (size_t)num_games * 4, s));
  // lane l starts game l (l < num_games); later games are handed out by k_ss_refill in lane order
  k_ss_init<<<(n + 255) / 256, 256, 0, s>>>(c, st, ws.lane_game, ws.next_game, num_games, n);
  MUZ_HIP_RET(hipGetLastError());
  // turns: at most ceil(num_games / lanes) generations of T turns each
  const long long gens = ((long long)num_games + n - 1) / n;
  const int max_turns = (int)std::min<long long>(gens * T + 1, 1 << 30);
  return sp_turns(c, w, cfg, st, tr, n, ws, ws.lane_game, num_games, max_turns, stats, s);
}

}  // extern "C"
