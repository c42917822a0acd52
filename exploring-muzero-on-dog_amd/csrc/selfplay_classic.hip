// Native self-play driver for classic MADN with Stochastic MuZero: play_n_games_v3 /
// play_batch_of_games_jitted of MuZero_Classic_MADN/game_agent_stochastic.py:52-257, as a host loop of
// stream-ordered HIP launches (same structure as the det driver, selfplay.hip).
//
// Per turn: throw the die of every active game (counter RNG -> throw_die) + legal masks + flags ->
// device compaction of the games that search -> encode -> root inference -> stochastic search ->
// env_step / no_step + trajectory records (incl. the die and the next state's dice distribution).
#include "classic.hpp"
#include "compact.hpp"
#include "host_consts.hpp"
#include "launch.hpp"
#include "turn_ledger.hpp"
#include "rng.hpp"

#include <algorithm>

namespace muz {

constexpr int kCsBlock = 256;
constexpr unsigned long long kDieStream = 0xD1CE5EEDF00DULL;

// Die of the turn: u = U[0,1) from (seed ^ kDieStream, game, turn), die = throw_die(env, u).
__device__ __forceinline__ float die_uniform(unsigned long long seed, int g, int turn) {
  return u24(mix64(game_key(seed ^ kDieStream, g, turn)));
}

// The die of lane g's game: its game number (lane_game, streaming driver) and own step count (== the
// turn in a batch) key the draw, so a game throws the same dice in whichever lane it is played.
__global__ __launch_bounds__(kCsBlock) void k_cs_flags(DetConsts c, muz_classic_soa st, unsigned long long seed,
                                                       const int32_t* idx, int T, const int32_t* lane_game,
                                                       uint32_t* legal, int32_t* flag, int n) {
  __shared__ int8_t sboard[kCells * kCsBlock];
  const int g = blockIdx.x * kCsBlock + threadIdx.x;
  if (g >= n) return;
  const int gn = lane_game ? lane_game[g] : g;
  if (st.done[g] || gn < 0 || idx[gn] >= T) {   // do_skip_step: nothing happens to a finished game
    flag[g] = 0;
    legal[g] = 0;
    return;
  }
  BoardView b{sboard + threadIdx.x, kCsBlock};
  ClsLane s;
  cls_load(c, st, g, s, b);
  float p[6];
  cls_dice_probs(c, cls_soft_locked(c, s, b), p);
  s.die = cls_choice(p, die_uniform(seed, gn, idx[gn]));
  st.die[g] = (int8_t)s.die;
  const uint32_t l = cls_legal(c, s, b);
  legal[g] = l;
  flag[g] = l ? 1 : 2;
}

// Observation (after the die) of every searching game, compacted order, + its int8 record.
__global__ __launch_bounds__(64) void k_cs_encode(DetConsts c, muz_classic_soa st, const int32_t* list,
                                                  const int32_t* counts, const uint32_t* legal, uint32_t* legal_c,
                                                  float* obs, int8_t* traj_obs, const int32_t* idx, int T,
                                                  const int32_t* lane_game) {
  const int sl = blockIdx.x;
  if (sl >= counts[0]) return;
  const int w = threadIdx.x;
  if (w >= kCells) return;
  const int g = list[sl];
  if (w == 0) legal_c[sl] = legal[g];
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
  float* o = obs + (size_t)sl * C * kCells;
  const int gn = lane_game ? lane_game[g] : g;
  int8_t* to = traj_obs + ((size_t)gn * T + idx[gn]) * C * kCells;
  auto owner = [&](int cell) { return (int)st.board[cell * S + g]; };
  for (int ch = 0; ch < C; ++ch) {
    const int v = cls_encode_value(c, s, ch, w, owner);
    o[ch * kCells + w] = (float)v;
    to[ch * kCells + w] = (int8_t)v;
  }
}

// do_mcts / do_skip + the buffer update (game_agent_stochastic.py:104-174).
__global__ __launch_bounds__(kCsBlock) void k_cs_apply(DetConsts c, muz_classic_soa st, const int32_t* flag,
                                                       const int32_t* slot, const int32_t* s_action,
                                                       const float* s_weights, const float* s_value, muz_traj tr,
                                                       muz_traj_chance ch, int n, const int32_t* lane_game,
                                                       const uint32_t* legal) {
  __shared__ int8_t sboard[kCells * kCsBlock];
  const int g = blockIdx.x * kCsBlock + threadIdx.x;
  if (g >= n) return;
  const int f = flag[g];
  if (f == 0) return;
  BoardView b{sboard + threadIdx.x, kCsBlock};
  ClsLane s;
  cls_load(c, st, g, s, b);
  const bool teams = has(c.flags, R_TEAMS);
  const int T = tr.max_steps;
  const int gn = lane_game ? lane_game[g] : g;
  const int t = tr.idx[gn];
  const size_t rec = (size_t)gn * T + t;
  const int cp_before = s.cp;
  const int team_before = teams ? cp_before % 2 : -1;
  const int die = s.die;
  int act, rew_cls, disc_cls;
  float val, mask;
  if (f == 1) {
    const int sl = slot[g];
    act = s_action[sl];
    const int r = cls_step_masked(c, s, b, act, legal[g]);   // legal[g]: this state's mask (k_cs_flags)
    const bool nd = s.done != 0;
    const int next_team = teams ? s.cp % 2 : -1;
    rew_cls = (nd && r > 0) ? 2 : ((nd && r < 0) ? 0 : 1);
    disc_cls = nd ? 1 : (teams ? (team_before == next_team ? 2 : 0) : (cp_before == s.cp ? 2 : 0));
    val = s_value[sl];
    mask = 1.f;
    for (int a = 0; a < MUZ_CLASSIC_ACTIONS; ++a)
      tr.pol[rec * MUZ_CLASSIC_ACTIONS + a] = s_weights[(size_t)sl * MUZ_CLASSIC_ACTIONS + a];
  } else {
    s.cp = (s.cp + 1) % c.P;   // no_step (353-365); obs / policy records stay zero
    act = -1;
    rew_cls = 1;
    disc_cls = 1;
    val = 0.f;
    mask = 0.f;
  }
  cls_store(c, st, g, s, b);
  float p[6];
  cls_dice_probs(c, cls_soft_locked(c, s, b), p);   // dice_probabilities(next_env) (line 162)
  for (int i = 0; i < 6; ++i) ch.dice_dist[rec * 6 + i] = p[i];
  ch.dice[rec] = die;
  tr.act[rec] = act;
  tr.rew[rec] = rew_cls;
  tr.val[rec] = val;
  tr.mask[rec] = mask;
  tr.player[rec] = cp_before;
  tr.team[rec] = team_before;
  tr.discount[rec] = disc_cls;
  tr.idx[gn] = t + 1;
}

__device__ void cls_reset_lane(const DetConsts& c, const muz_classic_soa& st, int g) {
  const int S = st.stride;
  const bool fp = has(c.flags, R_FREE_PIN);
  for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = -1;
  for (int p = 0; p < c.P; ++p) {
    for (int k = 0; k < 4; ++k) st.pins[(p * 4 + k) * S + g] = (int8_t)((fp && k == 0) ? c.start[p] : -1);
    if (fp) st.board[c.start[p] * S + g] = (int8_t)p;
  }
  st.current_player[g] = (int8_t)c.starting_player;
  st.reward[g] = 0;
  st.done[g] = 0;
  st.die[g] = 0;
}

__global__ void k_cs_reset(DetConsts c, muz_classic_soa st, int n) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  cls_reset_lane(c, st, g);
}

__global__ void k_cs_init(DetConsts c, muz_classic_soa st, int32_t* lane_game, int32_t* next, int num_games, int W) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l == 0) next[0] = min(num_games, W);
  if (l >= W) return;
  lane_game[l] = l < num_games ? l : -1;
  cls_reset_lane(c, st, l);
}

// Streaming refill (see selfplay.hip k_ss_refill): lanes whose game ended take the next game numbers in
// lane order and are reset; lanes left without a game go idle.
__global__ __launch_bounds__(kScanThreads) void k_cs_refill(DetConsts c, muz_classic_soa st, int32_t* lane_game,
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
      cls_reset_lane(c, st, l);
    } else {
      lane_game[l] = -1;
    }
  }
  __syncthreads();
  if (t == kScanThreads - 1) next[0] = min(num_games, base + part[t]);
}

struct CsWs {
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
  int32_t* lane_game;
  int32_t* next_game;
};

static inline size_t cal256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t cs_carve(char* base, int n, int C, int S, CsWs* w) {
  const size_t n16 = (size_t)((n + 15) / 16 * 16);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += cal256(bytes);
    return p;
  };
  CsWs t;
  t.tree = take((size_t)stochastic_workspace_bytes(n, S));
  t.conv = (float*)take(n16 * kConvRowFloats * 4);
  t.obs = (float*)take(n16 * C * kCells * 4);
  t.legal = (uint32_t*)take((size_t)n * 4);
  t.legal_c = (uint32_t*)take((size_t)n * 4);
  t.flag = (int32_t*)take((size_t)n * 4);
  t.slot = (int32_t*)take((size_t)n * 4);
  t.list = (int32_t*)take((size_t)n * 4);
  t.root_logits = (float*)take(n16 * MUZ_CLASSIC_ACTIONS * 4);
  t.root_value = (float*)take(n16 * 4);
  t.root_emb = (float*)take(n16 * 256 * 4);
  t.action = (int32_t*)take(n16 * 4);
  t.weights = (float*)take(n16 * MUZ_CLASSIC_ACTIONS * 4);
  t.value = (float*)take(n16 * 4);
  t.counts = (int32_t*)take(64);
  t.lane_game = (int32_t*)take((size_t)n * 4);
  t.next_game = (int32_t*)take(64);
  if (w) *w = t;
  return off;
}

// Turn loop shared by the batch and the streaming driver (see selfplay.hip sp_turns).
static int cs_turns(const DetConsts& c, const muz_classic_net_w* w, const muz_stoch_cfg* cfg, muz_classic_soa st,
                    muz_traj tr, muz_traj_chance ch, int n, const CsWs& ws, const int32_t* lane_game, int num_games,
                    int max_turns, muz_sp_stats* stats, hipStream_t s) {
  const int T = tr.max_steps;
  int rc = MUZ_OK;
  SArgs sa = make_sargs(*cfg, w->num_actions);
  sa.key_game = lane_game;
  sa.key_turn = tr.idx;   // the game's own step count (== the turn for every game of a batch)
  TurnLedger led(s, stats != nullptr);
  if ((rc = led.begin())) return rc;
  int turns = 0;
  rc = MUZ_OK;
  for (int turn = 0; turn < max_turns; ++turn) {
    if (!led.proceed(turn)) break;
    if (lane_game)
      k_cs_refill<<<1, kScanThreads, 0, s>>>(c, st, ws.lane_game, tr.idx, T, ws.next_game, num_games, n);
    k_cs_flags<<<(n + kCsBlock - 1) / kCsBlock, kCsBlock, 0, s>>>(c, st, cfg->seed, tr.idx, T, lane_game, ws.legal,
                                                                   ws.flag, n);
    k_sp_compact<<<1, kScanThreads, 0, s>>>(ws.flag, n, ws.list, ws.slot, ws.counts);
    led.counts(turn, ws.counts);
    k_cs_encode<<<n, 64, 0, s>>>(c, st, ws.list, ws.counts, ws.legal, ws.legal_c, ws.obs, tr.obs, tr.idx, T, lane_game);
    if ((rc = muz_last_launch_error())) break;
    if ((rc = launch_root_inference(*w, ws.obs, n, ws.counts, ws.conv, ws.root_logits, ws.root_value, ws.root_emb,
                                    s)))
      break;
    sa.turn = turn;
    led.search_begin(turn);
    if ((rc = launch_stochastic_search(*w, sa, ws.root_logits, ws.root_value, ws.root_emb, ws.legal_c, nullptr, nullptr,
                                       ws.list, n, ws.counts, ws.tree, ws.action, ws.weights, ws.value, s)))
      break;
    led.search_end(turn);
    k_cs_apply<<<(n + kCsBlock - 1) / kCsBlock, kCsBlock, 0, s>>>(c, st, ws.flag, ws.slot, ws.action, ws.weights,
                                                                   ws.value, tr, ch, n, lane_game, ws.legal);
    if ((rc = muz_last_launch_error())) break;
    ++turns;
  }
  led.finish(turns, stats);
  return rc;
}


}  // namespace muz

using namespace muz;

extern "C" {

int64_t muz_classic_selfplay_workspace_bytes(int32_t n, int32_t obs_channels, const muz_stoch_cfg* cfg) {
  if (!cfg || n < 0 || cfg->num_simulations < 1) return -1;
  return (int64_t)cs_carve(nullptr, n, obs_channels, cfg->num_simulations, nullptr);
}

int muz_classic_selfplay(const muz_rules* rules, const muz_classic_net_w* w, const muz_stoch_cfg* cfg,
                         muz_classic_soa st, muz_traj tr, muz_traj_chance ch, int32_t n, void* workspace,
                         int64_t workspace_bytes, muz_sp_stats* stats, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  if (!cfg) return MUZ_E_INVALID;
  if ((rc = check_classic_net(w))) return rc;
  if (w->obs_channels != 2 * c.P + 3) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && workspace && tr.max_steps > 0 && tr.obs && tr.act && tr.rew &&
                 tr.val && tr.pol && tr.mask && tr.player && tr.team && tr.discount && tr.idx && ch.dice &&
                 ch.dice_dist);
  if (cfg->num_simulations < 1 || cfg->num_simulations > 100 || cfg->max_depth < 1 || cfg->max_depth > 64)
    return MUZ_E_UNSUPPORTED;
  if (stats) *stats = muz_sp_stats{};
  MUZ_HOST_CHECK(workspace_bytes >= (int64_t)cs_carve(nullptr, n, w->obs_channels, cfg->num_simulations, nullptr));
  if (n == 0) return MUZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int C = w->obs_channels;
  const int T = tr.max_steps;
  CsWs ws;
  cs_carve((char*)workspace, n, C, cfg->num_simulations, &ws);

  k_cs_reset<<<(n + 255) / 256, 256, 0, s>>>(c, st, n);
  const size_t nt = (size_t)n * T;
  MUZ_HIP_RET(hipMemsetAsync(tr.obs, 0, nt * C * kCells, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.act, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.rew, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.val, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.pol, 0, nt * MUZ_CLASSIC_ACTIONS * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.mask, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.player, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.team, 0xFF, nt * 4, s));   // jnp.full(..., -1)
  MUZ_HIP_RET(hipMemsetAsync(tr.discount, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.idx, 0, (size_t)n * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(ch.dice, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(ch.dice_dist, 0, nt * 6 * 4, s));

  return cs_turns(c, w, cfg, st, tr, ch, n, ws, nullptr, n, T, stats, s);
}

int muz_classic_selfplay_stream(const muz_rules* rules, const muz_classic_net_w* w, const muz_stoch_cfg* cfg,
                                muz_classic_soa st, muz_traj tr, muz_traj_chance ch, int32_t num_games, int32_t lanes,
                                void* workspace, int64_t workspace_bytes, muz_sp_stats* stats, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  if (!cfg) return MUZ_E_INVALID;
  if ((rc = check_classic_net(w))) return rc;
  if (w->obs_channels != 2 * c.P + 3) return MUZ_E_UNSUPPORTED;
  const int n = lanes;
  MUZ_HOST_CHECK(n >= 0 && num_games >= 0 && st.stride >= n && workspace && tr.max_steps > 0 && tr.obs && tr.act &&
                 tr.rew && tr.val && tr.pol && tr.mask && tr.player && tr.team && tr.discount && tr.idx && ch.dice &&
                 ch.dice_dist);
  if (cfg->num_simulations < 1 || cfg->num_simulations > 100 || cfg->max_depth < 1 || cfg->max_depth > 64)
    return MUZ_E_UNSUPPORTED;
  if (stats) *stats = muz_sp_stats{};
  MUZ_HOST_CHECK(workspace_bytes >= (int64_t)cs_carve(nullptr, n, w->obs_channels, cfg->num_simulations, nullptr));
  if (n == 0 || num_games == 0) return MUZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int C = w->obs_channels;
  const int T = tr.max_steps;
  CsWs ws;
  cs_carve((char*)workspace, n, C, cfg->num_simulations, &ws);
  const size_t nt = (size_t)num_games * T;
  MUZ_HIP_RET(hipMemsetAsync(tr.obs, 0, nt * C * kCells, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.act, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.rew, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.val, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.pol, 0, nt * MUZ_CLASSIC_ACTIONS * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.mask, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.player, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.team, 0xFF, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.discount, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(tr.idx, 0, (size_t)num_games * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(ch.dice, 0, nt * 4, s));
  MUZ_HIP_RET(hipMemsetAsync(ch.dice_dist, 0, nt * 6 * 4, s));
  k_cs_init<<<(n + 255) / 256, 256, 0, s>>>(c, st, ws.lane_game, ws.next_game, num_games, n);
  MUZ_HIP_RET(hipGetLastError());
  const long long gens = ((long long)num_games + n - 1) / n;
  const int max_turns = (int)std::min<long long>(gens * T + 1, 1 << 30);
  return cs_turns(c, w, cfg, st, tr, ch, n, ws, ws.lane_game, num_games, max_turns, stats, s);
}

}  // extern "C"
