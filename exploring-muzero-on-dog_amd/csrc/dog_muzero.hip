// DOG MuZero slice (include/muz.h "DOG MuZero slice"): the observation encoder, root_inference_fn and
// recurrent_inference_fn at A = 806.  The reference has only the RepresentationNetwork
// (MuZero_DOG/muzero_dog.py:25-83); encode_board (DOG/dog.py:1264-1272) and the dynamics / prediction networks
// (muzero_dog.py:85-99) are `pass` and are defined here as oracle/dog_muzero.py restates them.
#include "dog.hpp"
#include "dog_nets.hpp"
#include "host_consts.hpp"
#include "launch.hpp"

namespace muz {

// ---- encode_board (oracle/dog_muzero.py encode_board): one game per wave, lane c < 56 owns cell c ---------------
__global__ __launch_bounds__(256) void k_dog_encode(DetConsts c, muz_dog_soa st, float* __restrict__ obs, int n) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= n) return;
  const int S = st.stride;
  const int cp = st.current_player[g];
  const bool teams = has(c.flags, R_TEAMS);
  // the rolled board: track by -10 * cp, goals by -4 * cp (deterministic_madn.py:401-402's perspective)
  int owner = -1;
  if (lane < kCells) {
    const int src = lane < kTrack ? (lane + kDist * cp) % kTrack : kTrack + ((lane - kTrack) + 4 * cp) % 16;
    owner = st.board[(size_t)src * S + g];
  }
  // player p done: every goal cell of p occupied (dog.py is_player_done)
  auto done = [&](int p) {
    bool all = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) all &= st.board[(size_t)c.goal[p][k] * S + g] >= 0;
    return all;
  };
  const int sub = (teams && done(cp)) ? (cp + 2) % 4 : cp;
  float gl[28];
  int held[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int p = (cp + r) % 4;
    int home = 0, h = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) home += st.pins[(size_t)(p * 4 + k) * S + g] == -1 ? 1 : 0;
#pragma unroll
    for (int k = 0; k < kDogCards; ++k) h += st.hands[(size_t)(p * kDogCards + k) * S + g];
    gl[r] = (float)home;
    held[r] = h;
  }
#pragma unroll
  for (int k = 0; k < kDogCards; ++k) gl[4 + k] = (float)st.hands[(size_t)(sub * kDogCards + k) * S + g];
#pragma unroll
  for (int r = 0; r < 4; ++r) gl[18 + r] = (float)held[r];
  int deck = 0;
#pragma unroll
  for (int k = 0; k < kDogCards; ++k) deck += st.deck[(size_t)k * S + g];
  gl[22] = (float)st.phase[g];
  gl[23] = (float)st.hand_size[g];
  gl[24] = sub != cp ? 1.f : 0.f;
  gl[25] = (float)deck;
  gl[26] = (float)(((int)st.round_starter[g] - cp + 8) % 4);
  int ingoal = 0;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    if (m == 1 && !teams) break;
    const int p = (cp + 2 * m) % 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) ingoal += st.pins[(size_t)(p * 4 + k) * S + g] >= kTrack ? 1 : 0;
  }
  gl[27] = (float)ingoal;
  if (lane >= kCells) return;
  float* o = obs + (size_t)g * kDogC * kCells + lane;
  float pc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    pc[r] = owner == (cp + r) % 4 ? 1.f : 0.f;
    o[r * kCells] = pc[r];
  }
  o[4 * kCells] = teams ? pc[0] + pc[2] : pc[0];
  o[5 * kCells] = teams ? pc[1] + pc[3] : pc[1] + pc[2] + pc[3];
#pragma unroll
  for (int i = 0; i < 28; ++i) o[(6 + i) * kCells] = gl[i];
}

// ---- root_inference_fn: RepresentationNetwork (LayerNorm head) -> PredictionNetwork4 at A = 806 ----------------
__global__ __launch_bounds__(kThreads) void k_dog_root_dense(muz_dog_net_w Wt, const float* __restrict__ obs,
                                                         const float* __restrict__ convout, int n,
                                                         float* __restrict__ prior_logits, float* __restrict__ value,
                                                         float* __restrict__ embedding) {
  (void)Wt;
  if ((int)blockIdx.x * kRows >= n) return;
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  const Arena a = Arena::carve(smem);
  const AS4 muz_dog_net_w* W = kernarg0<muz_dog_net_w>();
  const int g0 = blockIdx.x * kRows;
  const int row = trow(), sub = tsub();
  const int gr = g0 + row;
  const bool valid = gr < n;
  Pf pf;
  repr16<NT256, true>(W->repr, obs, kDogC, convout, g0, n, a, pf, &W->pred.rb[0].d0, LAT, LAT);
  __syncthreads();
  ln16<LAT, LN_PLAIN>(a.T, LD, a.T, LD, W->repr_ln7);   // muzero_dog.py:80-81: LayerNorm instead of min-max
  __syncthreads();
  if (valid)
    for (int c = sub; c < LAT; c += kRowLanes) embedding[(size_t)gr * LAT + c] = a.T[row * LD + c];
  __syncthreads();
  pred16<NT256, false, false, false, NT256, true>(W->pred, kDogA, a.T, a, pf, nullptr, 0, 0);
  if (valid && sub == 0) value[gr] = a.v0[row];
  dog_logits16<NT256>(W, a, pf, [&](int r, int col, float v) {
    if (valid) prior_logits[(size_t)(g0 + r) * kDogA + col] = v;
  }, nullptr, 0, 0);
}

// ---- recurrent_inference_fn: DynamicsNetwork4 (one-hot 806) -> PredictionNetwork4 ------------------------------
__global__ __launch_bounds__(kThreads) void k_dog_recurrent(muz_dog_net_w Wt, const int32_t* __restrict__ action,
                                                        const float* __restrict__ emb, int n, float* reward,
                                                        float* discount, float* prior_logits, float* value,
                                                        float* next_emb) {
  (void)Wt;
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  const Arena a = Arena::carve(smem);
  const int g0 = blockIdx.x * kRows;
  const int row = trow(), sub = tsub();
  const int gr = g0 + row;
  const bool valid = gr < n;
  const AS4 muz_dog_net_w* W = kernarg0<muz_dog_net_w>();
  const int ar = valid ? action[gr] : 0;
  const DynIn din = dyn_load(W->dyn, kDogA, valid ? gp(emb) + (size_t)gr * LAT : nullptr, ar);
  Pf pf;
  pf_issue<NT256>(pf, &W->dyn.d3, LAT, LAT);
  dyn16<NT256>(W->dyn, kDogA, din, ar, a, pf, &W->pred.rb[0].d0, LAT, LAT);
  if (valid) {
    for (int c = sub; c < LAT; c += kRowLanes) next_emb[(size_t)gr * LAT + c] = a.T[row * LD + c];
    if (sub == 0) {
      reward[gr] = a.v1[row];
      discount[gr] = a.v2[row];
    }
  }
  // no barrier: pred16 reads a.T in its first pass and overwrites it only after its first SYNC
  pred16<NT256, false, false, false, NT256, true>(W->pred, kDogA, a.T, a, pf, nullptr, 0, 0);
  if (valid && sub == 0) value[gr] = a.v0[row];
  dog_logits16<NT256>(W, a, pf, [&](int r, int col, float v) {
    if (valid) prior_logits[(size_t)(g0 + r) * kDogA + col] = v;
  }, nullptr, 0, 0);
}

int check_dog_net(const muz_dog_net_w* w) {
  if (!w || !w->dyn.film || !w->repr_ln7.scale || !w->logits[3].w) return MUZ_E_INVALID;
  if (w->num_actions != kDogA || w->obs_channels != kDogC) return MUZ_E_UNSUPPORTED;
  if (w->pred.d2.w != w->logits[0].w) return MUZ_E_INVALID;
  return MUZ_OK;
}

int dog_muzero_consts(const muz_rules* rules, DetConsts* c) {
  int rc = make_det_consts(rules, c, true);
  if (rc) return rc;
  if (c->P != 4) return MUZ_E_UNSUPPORTED;   // the slice plays config (d): 4-player DOG
  if (rules->disable_swapping || rules->disable_hot_seven || rules->disable_joker) return MUZ_E_UNSUPPORTED;
  return MUZ_OK;
}

int launch_dog_encode(const DetConsts& c, const muz_dog_soa& st, float* obs, int n, hipStream_t s) {
  k_dog_encode<<<(n + 3) / 4, 256, 0, s>>>(c, st, obs, n);
  return muz_last_launch_error();
}

int launch_dog_root(const muz_dog_net_w& w, const float* obs, int n, float* conv, float* logits, float* value,
                    float* emb, hipStream_t s) {
  int rc = launch_repr_conv(w.repr, obs, kDogC, n, nullptr, conv, s);
  if (rc) return rc;
  rc = launch_dense0(w.repr.d0, n, nullptr, conv, s);
  if (rc) return rc;
  k_dog_root_dense<<<(n + kRows - 1) / kRows, kThreads, 0, s>>>(w, obs, conv, n, logits, value, emb);
  return muz_last_launch_error();
}

}  // namespace muz

using namespace muz;

extern "C" {

int muz_dog_net_prepare(const muz_dog_net_w* w, void* stream) {
  if (!w || !w->dyn.film || !w->dyn.d0.w || !w->dyn.d0.b || !w->dyn.d12.w || !w->dyn.d12.b) return MUZ_E_INVALID;
  if (w->num_actions != kDogA) return MUZ_E_UNSUPPORTED;
  return launch_film(w->dyn, w->num_actions, (hipStream_t)stream);
}

int muz_dog_encode(const muz_rules* rules, muz_dog_soa state, float* obs, int32_t n, void* stream) {
  DetConsts c;
  int rc = dog_muzero_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && state.stride >= n && obs);
  if (n == 0) return MUZ_OK;
  return launch_dog_encode(c, state, obs, n, (hipStream_t)stream);
}

int muz_dog_nets_root(const muz_dog_net_w* w, const float* obs, int32_t n, void* scratch, int64_t scratch_bytes,
                      float* prior_logits, float* value, float* embedding, void* stream) {
  int rc = check_dog_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && obs && scratch && prior_logits && value && embedding);
  MUZ_HOST_CHECK(scratch_bytes >= muz_nets_root_scratch_bytes(n));
  if (n == 0) return MUZ_OK;
  return launch_dog_root(*w, obs, n, (float*)scratch, prior_logits, value, embedding, (hipStream_t)stream);
}

int muz_dog_nets_recurrent(const muz_dog_net_w* w, const int32_t* action, const float* embedding, int32_t n,
                           float* reward, float* discount, float* prior_logits, float* value, float* next_embedding,
                           void* stream) {
  int rc = check_dog_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && action && embedding && reward && discount && prior_logits && value && next_embedding);
  if (n == 0) return MUZ_OK;
  k_dog_recurrent<<<(n + kRows - 1) / kRows, kThreads, 0, (hipStream_t)stream>>>(
      *w, action, embedding, n, reward, discount, prior_logits, value, next_embedding);
  return muz_last_launch_error();
}

}  // extern "C"
