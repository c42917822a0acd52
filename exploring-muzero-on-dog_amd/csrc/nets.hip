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
// Conv_1 / Conv_2 input rows (32 / 64 channels) padded by 8 floats: the MFMA A-fragment reads (ds_read_b128, 16 rows
// per fragment) then hit 16 different bank groups -- with unpadded rows (a multiple of 64 floats apart) every row of a
// fragment started in the same banks (round 6; the search kernel's tiles measured the same)
#ifndef MUZ_CONV_PAD
#define MUZ_CONV_PAD 8   // (A/B switch: 0 = the unpadded rows of round 5)
#endif
constexpr int kC1Ld = 32 + MUZ_CONV_PAD;
constexpr int kC2Ld = 64 + MUZ_CONV_PAD;

// LayerNorm over channels for 56 positions, 4 lanes per position.
template <int N, int LDO>
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
    out[(out_row0 + pos) * LDO + c] = fmaxf(fmaf(v[i] - mean, inv * gp(P.scale)[c], gp(P.bias)[c]), 0.f);
  }
}

// Conv_1 / Conv_2 as implicit GEMMs [64 positions (56 + pad)][K] x [K][64]: wave w owns output channels 16 w .. + 15
// for ALL four 16-position row tiles (the weights packed as 4 groups of one 16-column tile), so each wave streams a
// quarter of the kernel from L2 once per game.  (Round 3 split the rows instead: every wave streamed the whole
// [K][64] kernel for its 16 positions, 4x the L2 weight reads -- 328 KB per game for Conv_2.)  The Toeplitz read:
// A[w][dk * CIN + ci] = in[(w + dk) * LDI + ci], a k-block (16 consecutive k) never straddles two taps.
template <int KB, int CIN, int LDI>
__device__ __forceinline__ void conv_mfma(const AS4 muz_dense& L, const float* in, float* pre) {
  static_assert(CIN % 16 == 0, "a k-block within one tap");
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
    for (int t = 0; t < 4; ++t)
      a[t] = *reinterpret_cast<const f32x4*>(in + (t * 16 + r + (kb * 16) / CIN) * LDI + (kb * 16) % CIN + 4 * g);
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
  __shared__ __attribute__((aligned(16))) float buf[68 * kC2Ld];
  float* in0 = buf;                 // [58][6]
  float* c1in = buf + 352;          // [66][kC1Ld]
  float* c2in = buf;                // [68][kC2Ld]
  static_assert(352 >= 58 * 6 && 352 + 66 * kC1Ld <= 68 * kC2Ld, "conv LDS carve");
  const int g = blockIdx.x;
  const int tid = threadIdx.x;
  const float* o = obs + (size_t)g * C * 56;
  for (int i = tid; i < 58 * 6; i += 256) {
    const int w = i / 6 - 1, ch = i % 6;
    in0[i] = (w >= 0 && w < 56) ? o[ch * 56 + w] : 0.f;
  }
  for (int i = tid; i < 66 * kC1Ld; i += 256) c1in[i] = 0.f;
  __syncthreads();
  // Conv_0 (K = 3*6 = 18, N = 32) on VALU: a thread keeps one output channel, its 18 weights in registers
  {
    const int co = tid & 31;
    float wk[18];
#pragma unroll
    for (int k = 0; k < 18; ++k) wk[k] = gp(R.conv0.w)[k * 32 + co];
    const float bco = gp(R.conv0.b)[co];
    for (int w = tid >> 5; w < 56; w += 8) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 18; ++k) s = fmaf(in0[w * 6 + k], wk[k], s);   // in0[(w + dk) * 6 + ci], k = dk * 6 + ci
      pre[w * kPreLd + co] = s + bco;
    }
  }
  __syncthreads();
  ln_positions<32, kC1Ld>(pre, c1in, 1, R.ln0);   // pad 1 row on each side for k=3
  __syncthreads();
  conv_mfma<6, 32, kC1Ld>(R.conv1, c1in, pre);     // K = 3*32 = 96
  __syncthreads();
  // c2in now reuses in0 | c1in: zero its pad rows (0, 1 and 58..67; the LayerNorm writes rows 2..57)
  for (int i = tid; i < 12 * kC2Ld; i += 256) c2in[(i < 2 * kC2Ld ? 0 : 56 * kC2Ld) + i] = 0.f;
  ln_positions<64, kC2Ld>(pre, c2in, 2, R.ln1);   // pad 2 rows for k=5
  __syncthreads();
  conv_mfma<20, 64, kC2Ld>(R.conv2, c2in, pre);    // K = 5*64 = 320
  __syncthreads();
  ln_positions<64, 64>(pre, c2in, 0, R.ln2);   // reuse c2in as the flattened output [56][64] (dense rows)
  __syncthreads();
  float* dst = convout + (size_t)g * kConvRowFloats;
  for (int i = tid; i < kConvMapFloats; i += 256) dst[i] = c2in[i];   // flatten (w, ch) -> w*64 + ch
}

// Two games per workgroup (MUZ_CONV_PAIR 1: 4 waves, 2: 8 waves): their 112 positions are exactly 7 MFMA row tiles,
// where one game per workgroup pads its 56 positions to 64 (1/8 of Conv_1 / Conv_2's MFMAs on padding rows).  Lane r
// of row tile t computes position R = 16 t + r, i.e. position R % 56 of game R / 56, and reads that game's rows: each
// game keeps its own zero rows around its positions, so every output is the same sum in the same order as
// k_repr_conv's.  With 8 waves, waves w and w + 4 own the same 16 output channels, w tiles 0-3 and w + 4 tiles 4-6
// (one SIMD carries both: the same MFMAs per SIMD, twice the waves to hide the row phases' latency).
#ifndef MUZ_CONV_PAIR
#define MUZ_CONV_PAIR 3   // root conv kernel traces, profiles/r6p_root_*: one game 146.8 us, pairs on 4 waves 141.4, on 8 142.2;
                          // r6z_root_kernel_stats_*: pairs on 4 waves 139.0, register-resident LayerNorms (3) 125.9
#endif
constexpr int kPairThreads = MUZ_CONV_PAIR == 2 ? 512 : 256;
constexpr int kPairRows = 112, kPairTiles = 7;
constexpr int kG0 = 58, kG1 = 58, kG2 = 60;   // rows per game: Conv_0 / Conv_1 input (1 zero row each side), Conv_2 (2)

// LayerNorm of 112 positions (4 lanes each; 2 passes with 256 threads), output row (R / 56) * GR + PAD + R % 56
template <int N, int LDO, int GR, int PAD>
__device__ __forceinline__ void ln_pair(const float* pre, float* out, const AS4 muz_ln& P) {
  const int q = threadIdx.x & 3;
  constexpr int PER = N / 4;
#pragma unroll
  for (int pass = 0; pass < 512 / kPairThreads; ++pass) {
    const int pos = (threadIdx.x >> 2) + (kPairThreads / 4) * pass;
    if (pos >= kPairRows) break;
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
    const int gm = pos >= 56 ? 1 : 0, orow = gm * GR + PAD + pos - 56 * gm;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = q + 4 * i;
      out[orow * LDO + c] = fmaxf(fmaf(v[i] - mean, inv * gp(P.scale)[c], gp(P.bias)[c]), 0.f);
    }
  }
}

// conv_mfma over NT of the pair's 7 row tiles from tile T0 (wave wv's 16 output channels: wv % 4); GR = input rows
// per game
template <int KB, int CIN, int LDI, int GR, int T0, int NT>
__device__ __forceinline__ void conv_mfma_pair(const AS4 muz_dense& L, const float* in, float* pre) {
  static_assert(CIN % 16 == 0, "a k-block within one tap");
  const int lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) & 3;
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(L.w)) + (size_t)wv * KB * 64 + lane;
  int roff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int R = (T0 + t) * 16 + r, gm = R >= 56 ? 1 : 0;
    roff[t] = (gm * GR + R - 56 * gm) * LDI + 4 * g;
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 w0 = wp[0], w1 = KB > 1 ? wp[64] : w0, w2;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 2 < KB) w2 = wp[(kb + 2) * 64];
    f32x4 a[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      a[t] = *reinterpret_cast<const f32x4*>(in + roff[t] + ((kb * 16) / CIN) * LDI + (kb * 16) % CIN);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma4(w0[j], a[t][j], acc[t]);
    w0 = w1;
    w1 = w2;
  }
  const AS1 f32x4* bias4 = gp(reinterpret_cast<const f32x4*>(L.b));
  const f32x4 bb = bias4[(16 * wv + 4 * g) >> 2];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    *reinterpret_cast<f32x4*>(pre + ((T0 + t) * 16 + r) * kPreLd + 16 * wv + 4 * g) = acc[t] + bb;
}

template <int KB, int CIN, int LDI, int GR>
__device__ __forceinline__ void conv_pair(const AS4 muz_dense& L, const float* in, float* pre) {
  if (kPairThreads == 256)
    conv_mfma_pair<KB, CIN, LDI, GR, 0, kPairTiles>(L, in, pre);
  else if (threadIdx.x < 256)
    conv_mfma_pair<KB, CIN, LDI, GR, 0, 4>(L, in, pre);
  else
    conv_mfma_pair<KB, CIN, LDI, GR, 4, 3>(L, in, pre);
}

__global__ __launch_bounds__(kPairThreads) void k_repr_conv2(muz_repr_w Rarg, const float* __restrict__ obs, int C, int n,
                                                    const int* __restrict__ n_dev, float* __restrict__ convout,
                                                    int32_t* host_counts) {
  if (host_counts && blockIdx.x == 0 && threadIdx.x == 0) {   // (n_dev set: the self-play turn's counts)
    __hip_atomic_store(&host_counts[0], n_dev[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host_counts[1], n_dev[1], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (n_dev) n = *n_dev;
  const int g0 = 2 * (int)blockIdx.x;
  if (g0 >= n) return;
  const int ng = g0 + 1 < n ? 2 : 1;
  const AS4 muz_repr_w& R = *kernarg0<muz_repr_w>();   // == Rarg, read through the kernarg segment
  // LDS: pre + one buffer holding in0 | c1in until Conv_1 has read them, then c2in, then the flattened maps (65 KB)
  __shared__ __attribute__((aligned(16))) float pre[kPairRows * kPreLd];
  __shared__ __attribute__((aligned(16))) float buf[2 * kG2 * kC2Ld];
  float* in0 = buf;                 // [2][58][6]
  float* c1in = buf + 704;          // [2][58][kC1Ld]
  float* c2in = buf;                // [2][60][kC2Ld]
  static_assert(704 >= 2 * kG0 * 6 && 704 + 2 * kG1 * kC1Ld <= 2 * kG2 * kC2Ld && kPairRows * 64 <= 2 * kG2 * kC2Ld,
                "pair conv LDS carve");
  const int tid = threadIdx.x;
  for (int i = tid; i < 2 * kG0 * 6; i += kPairThreads) {
    const int gm = i / (kG0 * 6), j = i % (kG0 * 6), w = j / 6 - 1, ch = j % 6;
    in0[i] = (gm < ng && w >= 0 && w < 56) ? obs[((size_t)(g0 + gm) * C + ch) * 56 + w] : 0.f;
  }
  for (int i = tid; i < 2 * kG1 * kC1Ld; i += kPairThreads) c1in[i] = 0.f;
  __syncthreads();
  // Conv_0 (K = 3*6 = 18, N = 32) on VALU: a thread keeps one output channel, its 18 weights in registers
  {
    const int co = tid & 31;
    float wk[18];
#pragma unroll
    for (int k = 0; k < 18; ++k) wk[k] = gp(R.conv0.w)[k * 32 + co];
    const float bco = gp(R.conv0.b)[co];
    for (int p = tid >> 5; p < kPairRows; p += kPairThreads / 32) {
      const int gm = p >= 56 ? 1 : 0;
      const float* x = in0 + gm * kG0 * 6 + (p - 56 * gm) * 6;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 18; ++k) s = fmaf(x[k], wk[k], s);
      pre[p * kPreLd + co] = s + bco;
    }
  }
  __syncthreads();
  ln_pair<32, kC1Ld, kG1, 1>(pre, c1in, R.ln0);
  __syncthreads();
  conv_pair<6, 32, kC1Ld, kG1>(R.conv1, c1in, pre);
  __syncthreads();
  // c2in now reuses in0 | c1in: zero each game's pad rows (0, 1, 58, 59; the LayerNorm writes rows 2..57)
  for (int i = tid; i < 8 * kC2Ld; i += kPairThreads) {
    const int rr = i / kC2Ld, row = (rr >> 2) * kG2 + ((rr & 3) < 2 ? (rr & 3) : 56 + (rr & 3));
    c2in[row * kC2Ld + i % kC2Ld] = 0.f;
  }
  ln_pair<64, kC2Ld, kG2, 2>(pre, c2in, R.ln1);
  __syncthreads();
  conv_pair<20, 64, kC2Ld, kG2>(R.conv2, c2in, pre);
  __syncthreads();
  ln_pair<64, 64, 56, 0>(pre, c2in, R.ln2);   // reuse c2in as the flattened output [2][56][64] (dense rows)
  __syncthreads();
  for (int i = tid; i < ng * kConvMapFloats; i += kPairThreads) {
    const int gm = i >= kConvMapFloats ? 1 : 0;
    convout[(size_t)(g0 + gm) * kConvRowFloats + i - gm * kConvMapFloats] = c2in[i];
  }
}

// MUZ_CONV_PAIR 3: the pair kernel with Conv_1 / Conv_2's outputs kept in the MFMA accumulators.  Their LayerNorms
// run from registers: each wave sums its 16 channels of a position (4 values per lane, then the permlane swaps across
// the 4 lane groups), the 4 waves' partials meet in a 3.5 KB LDS table, and every lane normalises its own values and
// stores them -- into Conv_2's input rows, or (Conv_2) straight into the flattened maps in HBM.  No [112][68]
// pre-activation buffer and one LDS round trip less per convolution: 39 KB of LDS, so 4 pairs (8 games) per CU
// instead of 2.  The LayerNorm sums run in another order than ln_pair's (same formula and eps): not bit-identical to
// k_repr_conv / k_repr_conv2 (the root tests bound it; the search and self-play parity tests give the oracle the
// GPU's own root outputs).
constexpr int kC1Ld3 = 36, kC2Ld3 = 68, kP0Ld = 36;   // +4-float row pads: the 16-row fragments hit distinct banks
constexpr int kIn0F = 704, kPre0At = kIn0F, kC1At = kPre0At + kPairRows * kP0Ld, kStatAt = kC1At + 2 * kG1 * kC1Ld3;
constexpr int kConv3Floats = kStatAt + kPairRows * 8;
static_assert(2 * kG0 * 6 <= kIn0F && 2 * kG2 * kC2Ld3 <= kStatAt && kConv3Floats * 4 <= 40 * 1024, "conv3 LDS carve");

// LayerNorm over the 32 channels of 112 positions read from pre0 (4 lanes per position, 2 passes of 64)
template <int N, int LDI, int LDO, int GR, int PAD>
__device__ __forceinline__ void ln_pair_ld(const float* pre, float* out, const AS4 muz_ln& P) {
  const int q = threadIdx.x & 3;
  constexpr int PER = N / 4;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int pos = (threadIdx.x >> 2) + 64 * pass;
    if (pos >= kPairRows) break;
    float v[PER], s = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      v[i] = pre[pos * LDI + q + 4 * i];
      s += v[i];
      s2 = fmaf(v[i], v[i], s2);
    }
    s += dpp<DPP_XOR1>(s);
    s += dpp<DPP_XOR2>(s);
    s2 += dpp<DPP_XOR1>(s2);
    s2 += dpp<DPP_XOR2>(s2);
    const float mean = s / (float)N, mean2 = s2 / (float)N;
    const float inv = ln_rstd(fmaxf(0.f, fmaf(-mean, mean, mean2)) + 1e-6f);
    const int gm = pos >= 56 ? 1 : 0, orow = gm * GR + PAD + pos - 56 * gm;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = q + 4 * i;
      out[orow * LDO + c] = fmaxf(fmaf(v[i] - mean, inv * gp(P.scale)[c], gp(P.bias)[c]), 0.f);
    }
  }
}

// one convolution of the pair into the accumulators (+ bias): lane (r, g) of wave wv holds channels 16 wv + 4 g .. + 3
// of positions 16 t + r, t < 7; then the per-wave (sum, sum of squares) of each position into st[pos][wv]
template <int KB, int CIN, int LDI, int GR>
__device__ __forceinline__ void conv_acc_pair(const AS4 muz_dense& L, const float* in, f32x4 (&acc)[kPairTiles],
                                              float* st) {
  static_assert(CIN % 16 == 0, "a k-block within one tap");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(L.w)) + (size_t)wv * KB * 64 + lane;
  int roff[kPairTiles];
#pragma unroll
  for (int t = 0; t < kPairTiles; ++t) {
    const int R = t * 16 + r, gm = R >= 56 ? 1 : 0;
    roff[t] = (gm * GR + R - 56 * gm) * LDI + 4 * g;
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 w0 = wp[0], w1 = KB > 1 ? wp[64] : w0, w2;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 2 < KB) w2 = wp[(kb + 2) * 64];
    f32x4 a[kPairTiles];
#pragma unroll
    for (int t = 0; t < kPairTiles; ++t)
      a[t] = *reinterpret_cast<const f32x4*>(in + roff[t] + ((kb * 16) / CIN) * LDI + (kb * 16) % CIN);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < kPairTiles; ++t) acc[t] = mfma4(w0[j], a[t][j], acc[t]);
    w0 = w1;
    w1 = w2;
  }
  const f32x4 bb = gp(reinterpret_cast<const f32x4*>(L.b))[(16 * wv + 4 * g) >> 2];
#pragma unroll
  for (int t = 0; t < kPairTiles; ++t) {
    acc[t] += bb;
    float s = (acc[t][0] + acc[t][1]) + (acc[t][2] + acc[t][3]);
    float s2 = fmaf(acc[t][3], acc[t][3], fmaf(acc[t][2], acc[t][2], fmaf(acc[t][1], acc[t][1], acc[t][0] * acc[t][0])));
    LoHi<float> p = swap16(s);     // lane groups g, g ^ 1
    s = p.lo + p.hi;
    p = swap16(s2);
    s2 = p.lo + p.hi;
    p = swap32(s);                 // g < 2 with g >= 2
    s = p.lo + p.hi;
    p = swap32(s2);
    s2 = p.lo + p.hi;
    if (g == 0) *reinterpret_cast<float2*>(st + (t * 16 + r) * 8 + 2 * wv) = make_float2(s, s2);
  }
}

// the LayerNorm of the accumulators (after a barrier has published st): mean / rstd from the 4 waves' partials
// (in wave order), then relu(LN) of the lane's 4 channels of each position, handed to out(pos, channel0, value4)
template <class F>
__device__ __forceinline__ void ln_acc_pair(const f32x4 (&acc)[kPairTiles], const float* st, const AS4 muz_ln& P,
                                            F out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4, c0 = 16 * wv + 4 * g;
  const f32x4 ga = gp(reinterpret_cast<const f32x4*>(P.scale))[c0 >> 2];
  const f32x4 be = gp(reinterpret_cast<const f32x4*>(P.bias))[c0 >> 2];
#pragma unroll
  for (int t = 0; t < kPairTiles; ++t) {
    const int pos = t * 16 + r;
    const f32x4 a = *reinterpret_cast<const f32x4*>(st + pos * 8);
    const f32x4 b = *reinterpret_cast<const f32x4*>(st + pos * 8 + 4);
    const float s = ((a[0] + a[2]) + b[0]) + b[2], s2 = ((a[1] + a[3]) + b[1]) + b[3];
    const float mean = s / 64.f, mean2 = s2 / 64.f;
    const float inv = ln_rstd(fmaxf(0.f, fmaf(-mean, mean, mean2)) + 1e-6f);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaxf(fmaf(acc[t][j] - mean, inv * ga[j], be[j]), 0.f);
    out(pos, c0, o);
  }
}

__global__ __launch_bounds__(256) void k_repr_conv3(muz_repr_w Rarg, const float* __restrict__ obs, int C, int n,
                                                    const int* __restrict__ n_dev, float* __restrict__ convout,
                                                    int32_t* host_counts) {
  if (host_counts && blockIdx.x == 0 && threadIdx.x == 0) {   // (n_dev set: the self-play turn's counts)
    __hip_atomic_store(&host_counts[0], n_dev[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host_counts[1], n_dev[1], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (n_dev) n = *n_dev;
  const int g0 = 2 * (int)blockIdx.x;
  if (g0 >= n) return;
  const int ng = g0 + 1 < n ? 2 : 1;
  const AS4 muz_repr_w& R = *kernarg0<muz_repr_w>();   // == Rarg, read through the kernarg segment
  __shared__ __attribute__((aligned(16))) float sm[kConv3Floats];
  float* in0 = sm;                 // [2][58][6]
  float* pre0 = sm + kPre0At;      // [112][36] Conv_0 output
  float* c1in = sm + kC1At;        // [2][58][36]
  float* c2in = sm;                // [2][60][68] (over in0 | pre0 | c1in once Conv_1 has read them)
  float* st = sm + kStatAt;        // [112][4 waves][sum, sum of squares]
  const int tid = threadIdx.x;
  for (int i = tid; i < 2 * kG0 * 6; i += 256) {
    const int gm = i / (kG0 * 6), j = i % (kG0 * 6), w = j / 6 - 1, ch = j % 6;
    in0[i] = (gm < ng && w >= 0 && w < 56) ? obs[((size_t)(g0 + gm) * C + ch) * 56 + w] : 0.f;
  }
  for (int i = tid; i < 4 * kC1Ld3; i += 256) {   // Conv_1 input pad rows 0 and 57 of each game
    const int rr = i / kC1Ld3;
    c1in[((rr >> 1) * kG1 + (rr & 1) * 57) * kC1Ld3 + i % kC1Ld3] = 0.f;
  }
  __syncthreads();
  {  // Conv_0 (K = 3*6 = 18, N = 32) on VALU: a thread keeps one output channel, its 18 weights in registers
    const int co = tid & 31;
    float wk[18];
#pragma unroll
    for (int k = 0; k < 18; ++k) wk[k] = gp(R.conv0.w)[k * 32 + co];
    const float bco = gp(R.conv0.b)[co];
    for (int p = tid >> 5; p < kPairRows; p += 8) {
      const int gm = p >= 56 ? 1 : 0;
      const float* x = in0 + gm * kG0 * 6 + (p - 56 * gm) * 6;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 18; ++k) s = fmaf(x[k], wk[k], s);
      pre0[p * kP0Ld + co] = s + bco;
    }
  }
  __syncthreads();
  ln_pair_ld<32, kP0Ld, kC1Ld3, kG1, 1>(pre0, c1in, R.ln0);
  __syncthreads();
  f32x4 acc[kPairTiles];
  conv_acc_pair<6, 32, kC1Ld3, kG1>(R.conv1, c1in, acc, st);
  __syncthreads();   // st published; every Conv_1 read of c1in done
  for (int i = tid; i < 8 * kC2Ld3; i += 256) {   // Conv_2 input pad rows 0, 1, 58, 59 of each game
    const int rr = i / kC2Ld3, row = (rr >> 2) * kG2 + ((rr & 3) < 2 ? (rr & 3) : 56 + (rr & 3));
    c2in[row * kC2Ld3 + i % kC2Ld3] = 0.f;
  }
  ln_acc_pair(acc, st, R.ln1, [&](int pos, int c0, const f32x4& o) {
    const int gm = pos >= 56 ? 1 : 0;
    *reinterpret_cast<f32x4*>(c2in + (gm * kG2 + 2 + pos - 56 * gm) * kC2Ld3 + c0) = o;
  });
  __syncthreads();   // c2in complete; st read
  conv_acc_pair<20, 64, kC2Ld3, kG2>(R.conv2, c2in, acc, st);
  __syncthreads();
  ln_acc_pair(acc, st, R.ln2, [&](int pos, int c0, const f32x4& o) {   // flatten (w, ch) -> w*64 + ch
    const int gm = pos >= 56 ? 1 : 0;
    if (gm < ng)
      *reinterpret_cast<f32x4*>(convout + (size_t)(g0 + gm) * kConvRowFloats + (pos - 56 * gm) * 64 + c0) = o;
  });
}

// RepresentationNetwork2's Dense_0 (3584 -> 256, muzero_deterministic_madn.py:107) for every game as ONE GEMM over
// 64-row x 64-column output tiles.  k_root_dense used to run it on its 16-row tiles, each tile streaming the layer's
// 3.67 MB of weights from L2 for 16 rows (~80 us of a 4096-game root inference at the L2-served rate,
// profiles/r5zf_root_dense0.log); a 64 x 64 tile reads 0.92 MB of weights and 0.92 MB of rows -- half the L2 bytes per
// FLOP -- staged through LDS in chunks of 4 k-blocks (double buffered).  8 waves: wave w owns rows 16 (w & 3) .. + 15
// and the packed column group 2 cb + (w >> 2) (dense16's NT256 packing: two 16-column MFMA tiles).  The MFMA order is
// dense16's (k-blocks in order, for each its 4 k-steps; then the bias), so the output is the one dense16 computes.
// XCD-aware: workgroup i runs on XCD i % 8, and the 4 column blocks of a row block are consecutive slots of one XCD,
// so a row block's rows are read into one L2.
#ifndef MUZ_D0_NG
#define MUZ_D0_NG 2   // packed column groups (32 columns each) per workgroup: 2 (64 x 64 tiles) or 1 (64 x 32)
#endif
#ifndef MUZ_D0_KC
#define MUZ_D0_KC 4   // k-blocks (16 k each) per staged chunk
#endif
constexpr int kD0Rows = 64, kD0NG = MUZ_D0_NG, kD0KC = MUZ_D0_KC, kD0Ld = kD0KC * 16 + 8;
constexpr int kD0KB = kConvMapFloats / 16, kD0Chunks = kD0KB / kD0KC;
constexpr int kD0CB = 8 / kD0NG;          // column blocks per row block
constexpr int kD0AF4 = kD0Rows * kD0KC * 4;            // float4 of a chunk's rows
constexpr int kD0WF4 = kD0NG * kD0KC * 128;            // float4 of a chunk's weights (per group: [kb][lane][tile])
static_assert(kD0KB % kD0KC == 0 && (kD0NG == 1 || kD0NG == 2), "Dense_0 chunks");
static_assert(kD0AF4 % 512 == 0 && kD0WF4 % 512 == 0, "Dense_0 staging: whole float4 per thread");

__global__ __launch_bounds__(512) void k_dense0(muz_dense d0, int n, const int* __restrict__ n_dev, float* conv) {
  if (n_dev) n = *n_dev;
  const int id = blockIdx.x, slot = id >> 3;
  const int rb = (slot / kD0CB) * 8 + (id & 7), cb = slot % kD0CB;
  const int row0 = rb * kD0Rows;
  if (row0 >= n) return;
  __shared__ __attribute__((aligned(16))) float sA[2][kD0Rows * kD0Ld];
  __shared__ f32x4 sW[2][kD0WF4];   // [buffer][group][kb][tile][lane]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // wave: 16 rows (row tile rt) x 32 columns (NG 2: group wv >> 2, both tiles) or 16 (NG 1: tile wv >> 2)
  constexpr int TW = kD0NG;   // MFMA tiles per wave
  const int rt = wv & 3, part = wv >> 2, r = lane & 15, g = lane >> 4;
  constexpr int kGroupF4 = kD0KB * 64 * 2;   // float4 per packed column group
  const AS1 f32x4* Wg = gp(reinterpret_cast<const f32x4*>(d0.w)) + (size_t)(kD0NG * cb) * kGroupF4;
  constexpr int QA = kD0AF4 / 512, QW = kD0WF4 / 512;
  f32x4 ra[QA], rw[QW];
  // chunk c: rows row0 .. + 63 x k 16 KC c .. (4 KC float4 per row) and the groups' KC k-blocks (KC * 128 float4 each)
  auto gload = [&](int c) {
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int i = t + 512 * q;
      const int row = row0 + i / (4 * kD0KC);
      ra[q] = row < n ? *gp(reinterpret_cast<const f32x4*>(conv + (size_t)row * kConvRowFloats + c * 16 * kD0KC) +
                            i % (4 * kD0KC))
                      : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const int i = t + 512 * q;
      rw[q] = Wg[(size_t)(i / (kD0KC * 128)) * kGroupF4 + c * (kD0KC * 128) + i % (kD0KC * 128)];
    }
  };
  auto lstore = [&](int b) {
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int i = t + 512 * q;
      *reinterpret_cast<f32x4*>(&sA[b][(i / (4 * kD0KC)) * kD0Ld + 4 * (i % (4 * kD0KC))]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const int i = t + 512 * q;
      const int j = i % (kD0KC * 128), kb = j >> 7, ln = (j >> 1) & 63, tt = j & 1;   // global order [kb][lane][tile]
      sW[b][(i / (kD0KC * 128)) * (kD0KC * 128) + (kb * 2 + tt) * 64 + ln] = rw[q];
    }
  };
  f32x4 acc[TW];
#pragma unroll
  for (int tt = 0; tt < TW; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this workgroup's share of the k chunks (blockIdx.y of kD0KSplit)
  constexpr int kPer = kD0Chunks / kD0KSplit;
  static_assert(kD0Chunks % kD0KSplit == 0, "Dense_0 k split");
  const int cbeg = (int)blockIdx.y * kPer;
  gload(cbeg);
  lstore(0);
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < kPer; ++c) {
    const int b = c & 1;
    if (c + 1 < kPer) gload(cbeg + c + 1);
#pragma unroll
    for (int kb = 0; kb < kD0KC; ++kb) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&sA[b][(rt * 16 + r) * kD0Ld + kb * 16 + 4 * g]);
      f32x4 w[TW];
#pragma unroll
      for (int tt = 0; tt < TW; ++tt) {
        const int grp = kD0NG == 2 ? part : 0, tile = kD0NG == 2 ? tt : part;
        w[tt] = sW[b][grp * (kD0KC * 128) + (kb * 2 + tile) * 64 + lane];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tt = 0; tt < TW; ++tt) acc[tt] = mfma4(w[tt][j], a[j], acc[tt]);   // D = W^T A^T, dense16's order
    }
    if (c + 1 < kPer) lstore(b ^ 1);
    __syncthreads();
  }
  const int row = row0 + rt * 16 + r;
  if (row < n) {
    const AS1 f32x4* bias4 = gp(reinterpret_cast<const f32x4*>(d0.b));
#pragma unroll
    for (int tt = 0; tt < TW; ++tt) {
      const int col = kD0NG == 2 ? (2 * cb + part) * 32 + tt * 16 + 4 * g : cb * 32 + part * 16 + 4 * g;
      float* dst = conv + (size_t)row * kConvRowFloats + kConvMapFloats + 256 * blockIdx.y + col;
      // (split: partial planes without the bias, which the consumer adds after the planes)
      *reinterpret_cast<f32x4*>(dst) = kD0KSplit > 1 ? acc[tt] : acc[tt] + bias4[col >> 2];
    }
  }
}

int launch_dense0(const muz_dense& d0, int n, const int* n_dev, float* conv, hipStream_t s) {
  const int rbs = (n + kD0Rows - 1) / kD0Rows;
  const int wgs = (rbs + 7) / 8 * 8 * kD0CB;   // kD0CB column blocks per row block, row blocks dealt over the 8 XCDs
  k_dense0<<<dim3(wgs, kD0KSplit), 512, 0, s>>>(d0, n, n_dev, conv);
  return muz_last_launch_error();
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
  repr16<NT256, true>(W->repr, obs, Wt.obs_channels, convout, g0, n, a, pf, &W->pred.rb[0].d0, LAT, LAT);
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
  if (MUZ_CONV_PAIR == 3)
    k_repr_conv3<<<(n + 1) / 2, 256, 0, s>>>(r, obs, C, n, n_dev, conv, host_counts);
  else if (MUZ_CONV_PAIR)
    k_repr_conv2<<<(n + 1) / 2, kPairThreads, 0, s>>>(r, obs, C, n, n_dev, conv, host_counts);
  else
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
  rc = launch_dense0(w.repr.d0, n, n_dev, conv, s);
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
  return rows * kConvRowFloats * (int64_t)sizeof(float);
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
