// MuZero network kernels: root_inference_fn and recurrent_inference_fn
// (MuZero_det_MADN/muzero_deterministic_madn.py:621-661) as fused fp32 MFMA kernels.
#include <type_traits>

#include "launch.hpp"
#include "nn.hpp"

namespace muz {

// ---------------------------------------------------------------------------------------------------
// RepresentationNetwork2 spatial stream (lines 86-104): 3 x (Conv1D SAME -> LayerNorm -> ReLU) per game.
// One game per workgroup; conv1/conv2 are implicit GEMMs on MFMA: the zero-padded input [W+k-1][Cin]
// is read as a Toeplitz matrix A[w][dk*Cin+ci] = in[(w+dk)*Cin+ci], waves own 16-position row tiles.
constexpr int kConvRowsPad = 64;          // 56 positions padded to 4 MFMA row tiles
constexpr int kPreLd = 64 + 4;

// LayerNorm over channels for 56 positions, 4 lanes per position.
template <int N>
__device__ __forceinline__ void ln_positions(const float* pre, float* out, int out_row0, const AS4 muz_ln& P) {
  const int pos = threadIdx.x >> 2, q = threadIdx.x & 3;
  if (pos >= 56) return;
  constexpr int PER = N / 4;
  float v[PER], s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = pre[pos * kPreLd + q + 4 * i];
    s += v[i];
    s2 = fmaf(v[i], v[i], s2);
  }
  s += dpp<DPP_XOR1>(s);
  s += dpp<DPP_XOR2>(s);
  s2 += dpp<DPP_XOR1>(s2);
  s2 += dpp<DPP_XOR2>(s2);
  const float mean = s / (float)N, mean2 = s2 / (float)N;
  const float inv = ln_rstd(fmaxf(0.f, fmaf(-mean, mean, mean2)) + 1e-6f);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = q + 4 * i;
    out[(out_row0 + pos) * N + c] = fmaxf(fmaf(v[i] - mean, inv * gp(P.scale)[c], gp(P.bias)[c]), 0.f);
  }
}

// Conv_1 / Conv_2 as implicit GEMMs [64 positions (56 + pad)][K] x [K][64]: wave w owns output channels 16 w .. + 15
// for ALL four 16-position row tiles (the weights packed as 4 groups of one 16-column tile), so each wave streams a
// quarter of the kernel from L2 once per game.  (Round 3 split the rows instead: every wave streamed the whole
// [K][64] kernel for its 16 positions, 4x the L2 weight reads -- 328 KB per game for Conv_2.)
template <int KB>
__device__ __forceinline__ void conv_mfma(const AS4 muz_dense& L, const float* in, int cin, float* pre) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(L.w)) + (size_t)wv * KB * 64 + lane;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // weights of k-blocks kb + 1, kb + 2 in flight while kb is multiplied
  f32x4 w0 = wp[0], w1 = KB > 1 ? wp[64] : w0, w2;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 2 < KB) w2 = wp[(kb + 2) * 64];
    f32x4 a[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const f32x4*>(in + (t * 16 + r) * cin + kb * 16 + 4 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma4(w0[j], a[t][j], acc[t]);
    w0 = w1;
    w1 = w2;
  }
  // out^T layout: lane (r, g) holds channels 16 wv + 4 g .. + 3 of position t * 16 + r
  const AS1 f32x4* bias4 = gp(reinterpret_cast<const f32x4*>(L.b));
  const f32x4 bb = bias4[(16 * wv + 4 * g) >> 2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    *reinterpret_cast<f32x4*>(pre + (t * 16 + r) * kPreLd + 16 * wv + 4 * g) = acc[t] + bb;
}

__global__ __launch_bounds__(256) void k_repr_conv(muz_repr_w Rarg, const float* __restrict__ obs, int C, int n,
                                                   const int* __restrict__ n_dev, float* __restrict__ convout,
                                                   int32_t* host_counts) {
  if (host_counts && blockIdx.x == 0 && threadIdx.x == 0) {   // (n_dev set: the self-play turn's counts)
    __hip_atomic_store(&host_counts[0], n_dev[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host_counts[1], n_dev[1], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (n_dev) n = *n_dev;
  if ((int)blockIdx.x >= n) return;
  const AS4 muz_repr_w& R = *kernarg0<muz_repr_w>();   // == Rarg, read through the kernarg segment
  // LDS: pre + one buffer holding in0 | c1in until Conv_1 has read them, then c2in (34.8 KB: 4 workgroups per CU
  // instead of 3 with separate buffers)
  __shared__ __attribute__((aligned(16))) float pre[kConvRowsPad * kPreLd];
  __shared__ __attribute__((aligned(16))) float buf[68 * 64];
  float* in0 = buf;                 // [58][6]
  float* c1in = buf + 352;          // [66][32]
  float* c2in = buf;                // [68][64]
  static_assert(352 >= 58 * 6 && 352 + 66 * 32 <= 68 * 64, "conv LDS carve");
  const int g = blockIdx.x;
  const int tid = threadIdx.x;
  const float* o = obs + (size_t)g * C * 56;
  for (int i = tid; i < 58 * 6; i += 256) {
    const int w = i / 6 - 1, ch = i % 6;
    in0[i] = (w >= 0 && w < 56) ? o[ch * 56 + w] : 0.f;
  }
  for (int i = tid; i < 66 * 32; i += 256) c1in[i] = 0.f;
  __syncthreads();
  // Conv_0 (K = 3*6 = 18, N = 32) on VALU
  for (int i = tid; i < 56 * 32; i += 256) {
    const int w = i >> 5, co = i & 31;
    float s = 0.f;
#pragma unroll
    for (int dk = 0; dk < 3; ++dk)
#pragma unroll
      for (int ci = 0; ci < 6; ++ci) s = fmaf(in0[(w + dk) * 6 + ci], gp(R.conv0.w)[(dk * 6 + ci) * 32 + co], s);
    pre[w * kPreLd + co] = s + gp(R.conv0.b)[co];
  }
  __syncthreads();
  ln_positions<32>(pre, c1in, 1, R.ln0);   // pad 1 row on each side for k=3
  __syncthreads();
  conv_mfma<6>(R.conv1, c1in, 32, pre);     // K = 3*32 = 96
  __syncthreads();
  // c2in now reuses in0 | c1in: zero its pad rows (0, 1 and 58..67; the LayerNorm writes rows 2..57)
  for (int i = tid; i < 12 * 64; i += 256) c2in[(i < 128 ? 0 : 56 * 64) + i] = 0.f;
  ln_positions<64>(pre, c2in, 2, R.ln1);   // pad 2 rows for k=5
  __syncthreads();
  conv_mfma<20>(R.conv2, c2in, 64, pre);    // K = 5*64 = 320
  __syncthreads();
  ln_positions<64>(pre, c2in, 0, R.ln2);   // reuse c2in rows 0..55 as the flattened output
  __syncthreads();
  float* dst = convout + (size_t)g * 3584;
  for (int i = tid; i < 3584; i += 256) dst[i] = c2in[i];   // flatten (w, ch) -> w*64 + ch
}

// Rest of RepresentationNetwork2 + PredictionNetwork4 on 16-game tiles.  NW = muz_net_w (det) or
// muz_classic_net_w (classic): both carry obs_channels, num_actions, repr and pred.
template <class NW>
__global__ __launch_bounds__(kThreads) void k_root_dense(NW Wt, const float* __restrict__ obs,
                                                    const float* __restrict__ convout, int n,
                                                    const int* __restrict__ n_dev, float* prior_logits, float* value,
                                                    float* embedding) {
  if (n_dev) n = *n_dev;
  if ((int)blockIdx.x * kRows >= n) return;
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  const Arena a = Arena::carve(smem);
  const AS4 NW* W = kernarg0<NW>();   // == Wt, read through the kernarg segment
  const int A = Wt.num_actions;
  const int g0 = blockIdx.x * kRows;
  const int row = trow(), sub = tsub();
  const int gr = g0 + row;
  const bool valid = gr < n;
  Pf pf;
  repr16<NT256>(W->repr, obs, Wt.obs_channels, convout, g0, n, a, pf, &W->pred.rb[0].d0, LAT, LAT);
  __syncthreads();
  minmax16(a.T, LD);
  __syncthreads();
  if (valid)
    for (int c = sub; c < LAT; c += kRowLanes) embedding[(size_t)gr * LAT + c] = a.T[row * LD + c];
  __syncthreads();
  pred16<1, false, false, kSplitkLogits && std::is_same<NW, muz_net_w>::value>(W->pred, A, a.T, a, pf, nullptr, 0, 0);
  if (valid) {
    for (int c = sub; c < A; c += kRowLanes) prior_logits[(size_t)gr * A + c] = a.U[row * LD + c];
    if (sub == 0) value[gr] = a.v0[row];
  }
}

// recurrent_inference_fn on 16-row tiles.
__global__ __launch_bounds__(kThreads) void k_recurrent(muz_net_w Wt, const int32_t* __restrict__ action,
                                                   const float* __restrict__ emb, int n, float* reward,
                                                   float* discount, float* prior_logits, float* value,
                                                   float* next_emb) {
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  const Arena a = Arena::carve(smem);
  const int A = Wt.num_actions;
  const int g0 = blockIdx.x * kRows;
  const int row = trow(), sub = tsub();
  const int gr = g0 + row;
  const bool valid = gr < n;
  const AS4 muz_net_w* W = kernarg0<muz_net_w>();   // == Wt, read through the kernarg segment
  const int ar = valid ? action[gr] : 0;
  const DynIn din = dyn_load(W->dyn, A, valid ? gp(emb) + (size_t)gr * LAT : nullptr, ar);
  Pf pf;
  pf_issue<NT256>(pf, &W->dyn.d3, LAT, LAT);
  dyn16<NT256>(W->dyn, A, din, ar, a, pf, &W->pred.rb[0].d0, LAT, LAT);
  if (valid) {
    for (int c = sub; c < LAT; c += kRowLanes) next_emb[(size_t)gr * LAT + c] = a.T[row * LD + c];
    if (sub == 0) {
      reward[gr] = a.v1[row];
      discount[gr] = a.v2[row];
    }
  }
  // no barrier: pred16 reads a.T in its first pass and overwrites it only after its first SYNC
  pred16<1, false, false, kSplitkLogits>(W->pred, A, a.T, a, pf, nullptr, 0, 0);
  if (valid) {
    for (int c = sub; c < A; c += kRowLanes) prior_logits[(size_t)gr * A + c] = a.U[row * LD + c];
    if (sub == 0) value[gr] = a.v0[row];
  }
}

// dyn.film[a][0:256 | 256:512] = Dense_1 | Dense_2 (relu(Dense_0(one_hot(a))))  (Dyn4 lines 399-411):
// FiLM scale | shift depend on the action only.  Row A = zero one-hot (out-of-range action).
// One workgroup per action row, one thread per output column; d12 is read in its packed layout.
__global__ __launch_bounds__(512) void k_film(muz_dyn_w D, int A) {
  __shared__ float e[64];
  const int a = blockIdx.x, n = threadIdx.x;
  if (n < 64) e[n] = fmaxf((a < A ? D.d0.w[a * 64 + n] : 0.f) + D.d0.b[n], 0.f);
  __syncthreads();
  const int w = (n >> 4) / NT512, t = (n >> 4) % NT512;
  float acc = 0.f;
  for (int k = 0; k < 64; ++k) {
    const int kb = k >> 4, lane = ((k & 15) >> 2) * 16 + (n & 15), j = k & 3;
    acc = fmaf(e[k], D.d12.w[((((size_t)w * 4 + kb) * 64 + lane) * NT512 + t) * 4 + j], acc);
  }
  D.film[a * 512 + n] = acc + D.d12.b[n];
}

int check_net(const muz_net_w* w) {
  if (!w) return MUZ_E_INVALID;
  if (!w->dyn.film) return MUZ_E_INVALID;
  if (w->num_actions != MUZ_DET_ACTIONS) return MUZ_E_UNSUPPORTED;
  if (w->obs_channels < 7 || w->obs_channels > 38) return MUZ_E_UNSUPPORTED;
  return MUZ_OK;
}

int launch_repr_conv(const muz_repr_w& r, const float* obs, int C, int n, const int* n_dev, float* conv,
                     hipStream_t s, int32_t* host_counts) {
  if (host_counts && !n_dev) return MUZ_E_INVALID;
  k_repr_conv<<<n, 256, 0, s>>>(r, obs, C, n, n_dev, conv, host_counts);
  return muz_last_launch_error();
}

int launch_film(const muz_dyn_w& d, int A, hipStream_t s) {
  k_film<<<A + 1, 512, 0, s>>>(d, A);
  return muz_last_launch_error();
}

template <class NW>
static int launch_root_impl(const NW& w, const float* obs, int n, const int* n_dev, float* conv, float* logits,
                            float* value, float* emb, hipStream_t s, int32_t* host_counts = nullptr) {
  int rc = launch_repr_conv(w.repr, obs, w.obs_channels, n, n_dev, conv, s, host_counts);
  if (rc) return rc;
  k_root_dense<NW><<<(n + kRows - 1) / kRows, kThreads, 0, s>>>(w, obs, conv, n, n_dev, logits, value, emb);
  return muz_last_launch_error();
}

int launch_root_inference(const muz_net_w& w, const float* obs, int n, const int* n_dev, float* conv, float* logits,
                          float* value, float* emb, hipStream_t s, int32_t* host_counts) {
  return launch_root_impl(w, obs, n, n_dev, conv, logits, value, emb, s, host_counts);
}

int launch_root_inference(const muz_classic_net_w& w, const float* obs, int n, const int* n_dev, float* conv,
                          float* logits, float* value, float* emb, hipStream_t s) {
  return launch_root_impl(w, obs, n, n_dev, conv, logits, value, emb, s);
}

}  // namespace muz

using namespace muz;

extern "C" {

int32_t muz_tile_waves(void) { return kWaves; }

int muz_net_prepare(const muz_net_w* w, void* stream) {
  if (!w || !w->dyn.film || !w->dyn.d0.w || !w->dyn.d0.b || !w->dyn.d12.w || !w->dyn.d12.b) return MUZ_E_INVALID;
  if (w->num_actions != MUZ_DET_ACTIONS) return MUZ_E_UNSUPPORTED;
  k_film<<<w->num_actions + 1, 512, 0, (hipStream_t)stream>>>(w->dyn, w->num_actions);
  return muz_last_launch_error();
}

int64_t muz_nets_root_scratch_bytes(int32_t n) {
  const int64_t rows = ((int64_t)n + kRows - 1) / kRows * kRows;
  return rows * 3584 * (int64_t)sizeof(float);
}

int muz_nets_root(const muz_net_w* w, const float* obs, int32_t n, void* scratch, int64_t scratch_bytes,
                  float* prior_logits, float* value, float* embedding, void* stream) {
  int rc = check_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && obs && scratch && prior_logits && value && embedding);
  MUZ_HOST_CHECK(scratch_bytes >= muz_nets_root_scratch_bytes(n));
  if (n == 0) return MUZ_OK;
  return launch_root_inference(*w, obs, n, nullptr, (float*)scratch, prior_logits, value, embedding,
                               (hipStream_t)stream);
}

int muz_nets_recurrent(const muz_net_w* w, const int32_t* action, const float* embedding, int32_t n, float* reward,
                       float* discount, float* prior_logits, float* value, float* next_embedding, void* stream) {
  int rc = check_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && action && embedding && reward && discount && prior_logits && value && next_embedding);
  if (n == 0) return MUZ_OK;
  k_recurrent<<<(n + kRows - 1) / kRows, kThreads, 0, (hipStream_t)stream>>>(*w, action, embedding, n, reward, discount,
                                                                         prior_logits, value, next_embedding);
  return muz_last_launch_error();
}

}  // extern "C"
