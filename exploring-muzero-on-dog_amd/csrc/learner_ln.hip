// Fused Dense epilogue for the learner (train_with_reward.py / train_stochastic.py: Flax Dense -> LayerNorm
// -> ReLU, and the ResBlock tail relu(x + LayerNorm(Dense(.))).  The GEMM stays a library GEMM; these kernels
// replace the bias add, LayerNorm, ReLU and residual add of the forward pass (one kernel instead of 3-5) and
// the ReLU / LayerNorm / bias backward (two kernels instead of ~5), which is what a batch-128 training step
// is made of: hundreds of tiny launches.
//
// Forward, per row m of y [M][N] (one wave per row, N in {32, 64, 128, 256}):
//   z = y + bias;  Flax LayerNorm (eps 1e-6, fast variance E[z^2] - E[z]^2, as nn.hpp's ln16);
//   o = (z - mean) * (rstd * gamma) + beta;  out = o (PLAIN) | relu(o) (RELU) | relu(res + o) (RESID_RELU).
// Saved for the backward: z, mean, rstd and out (the ReLU mask).
// Split-K form (muz_ln_fwd_parts): y is `parts` planes of partial products (a long-K GEMM as a batched GEMM over K
// chunks), summed here in plane order before the bias.
// FiLM variant (the first op of a dynamics trunk, muzero_deterministic_madn.py:421-427: LayerNorm_0 of the latent,
// then x * (1 + scale) + shift): PLAIN LayerNorm without a bias, plus film = shift + out * scale1 (scale1 = 1 + scale);
// its backward takes d(film) and writes dscale = d(film) * out beside the LayerNorm backward of d(film) * scale1
// (one launch each way instead of LayerNorm + addcmul and two multiplies + LayerNorm backward).
// Backward: do = dout (PLAIN) or dout * (out > 0); dres = do (RESID_RELU);
//   xhat = (z - mean) * rstd, g = do * gamma,
//   dz = rstd * (g - mean_n(g) - xhat * mean_n(g * xhat))       (= dy, and its column sum is dbias),
//   dgamma = sum_m do * xhat, dbeta = sum_m do, dbias = sum_m dz
// with the column sums as per-block partials reduced in a fixed order (deterministic: graph-captured and
// eager steps stay bit-identical).
#include "launch.hpp"

namespace muz {

enum { LN_MODE_PLAIN = 0, LN_MODE_RELU = 1, LN_MODE_RESID_RELU = 2 };
constexpr int kLnRowsPerBlock = 4;    // backward: rows per workgroup (one per wave: these launches are latency-bound)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int N, bool FILM = false>
__global__ __launch_bounds__(256) void k_ln_fwd(const float* __restrict__ y, const float* __restrict__ bias,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                const float* __restrict__ res, int M, int mode, float* __restrict__ out,
                                                float* __restrict__ z, float* __restrict__ mean_out,
                                                float* __restrict__ rstd_out, const float* __restrict__ scale1 = nullptr,
                                                const float* __restrict__ shift = nullptr,
                                                float* __restrict__ film = nullptr, int parts = 1) {
  // no fma contraction: the row kernels and their fused boundary forms round identically
#pragma clang fp contract(off)
  constexpr int E = (N + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const size_t row = (size_t)m * N;
  float v[E];
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int c = lane + 64 * i;
    float yc = 0.f;
    if (c < N) {
      yc = y[row + c];
      if (!FILM && parts > 1) {   // plane order; the loads issued before the adds
        float pv[16];
        for (int q0 = 1; q0 < parts; q0 += 16) {
#pragma unroll
          for (int u = 0; u < 16; ++u) pv[u] = q0 + u < parts ? y[(size_t)(q0 + u) * M * N + row + c] : 0.f;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (q0 + u < parts) yc = yc + pv[u];
        }
      }
    }
    v[i] = c < N ? (FILM ? yc : yc + bias[c]) : 0.f;
    s += v[i];
    s2 += v[i] * v[i];
  }
  s = wave_sum(s);
  s2 = wave_sum(s2);
  const float mean = s / (float)N;
  const float rstd = 1.0f / sqrtf(fmaxf(0.f, s2 / (float)N - mean * mean) + 1e-6f);
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int c = lane + 64 * i;
    if (c >= N) continue;
    float o = (v[i] - mean) * (rstd * gamma[c]) + beta[c];
    if (mode == LN_MODE_RELU) o = fmaxf(o, 0.f);
    if (mode == LN_MODE_RESID_RELU) o = fmaxf(res[row + c] + o, 0.f);
    out[row + c] = o;
    z[row + c] = v[i];
    // rounded as torch's addcmul (a multiply, then an add; no fma), so the chain node and the per-step graph
    // see the same bits: min-max's extremum columns (and where their gradient goes) depend on the last ulp
    if constexpr (FILM) {
      float p = o * scale1[row + c];
      asm volatile("" : "+v"(p));   // keeps the multiply out of an fma with the add
      film[row + c] = shift[row + c] + p;
    }
  }
  if (lane == 0) {
    mean_out[m] = mean;
    rstd_out[m] = rstd;
  }
}

template <int N, bool FILM = false>
__global__ __launch_bounds__(256) void k_ln_bwd(const float* __restrict__ dout, const float* __restrict__ out,
                                                const float* __restrict__ z, const float* __restrict__ mean_in,
                                                const float* __restrict__ rstd_in, const float* __restrict__ gamma,
                                                int M, int mode, float* __restrict__ dz, float* __restrict__ dres,
                                                float* __restrict__ part, const float* __restrict__ scale1 = nullptr,
                                                float* __restrict__ dscale = nullptr, int ldd = N) {
  // no fma contraction: the row kernels and their fused boundary forms round identically
#pragma clang fp contract(off)
  constexpr int E = (N + 63) / 64;
  __shared__ float red[4][3][N];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pg[E], pb[E], pd[E];
#pragma unroll
  for (int i = 0; i < E; ++i) pg[i] = pb[i] = pd[i] = 0.f;
  for (int k = 0; k < kLnRowsPerBlock / 4; ++k) {
    const int m = blockIdx.x * kLnRowsPerBlock + wv * (kLnRowsPerBlock / 4) + k;
    if (m >= M) break;
    const size_t row = (size_t)m * N;
    const float mean = mean_in[m], rstd = rstd_in[m];
    float d[E], xh[E], g[E];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int c = lane + 64 * i;
      d[i] = xh[i] = g[i] = 0.f;
      if (c >= N) continue;
      float t = dout[(size_t)m * ldd + c];   // (dout rows ldd apart: a column slice of a wider gradient)
      if constexpr (FILM) {
        dscale[row + c] = t * out[row + c];
        t = t * scale1[row + c];
      }
      if (mode != LN_MODE_PLAIN && !(out[row + c] > 0.f)) t = 0.f;
      if (mode == LN_MODE_RESID_RELU) dres[row + c] = t;
      d[i] = t;
      xh[i] = (z[row + c] - mean) * rstd;
      g[i] = t * gamma[c];
      a += g[i];
      b += g[i] * xh[i];
    }
    a = wave_sum(a) / (float)N;
    b = wave_sum(b) / (float)N;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int c = lane + 64 * i;
      if (c >= N) continue;
      const float dzi = rstd * (g[i] - a - xh[i] * b);
      dz[row + c] = dzi;
      pg[i] += d[i] * xh[i];
      pb[i] += d[i];
      pd[i] += dzi;
    }
  }
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int c = lane + 64 * i;
    if (c >= N) continue;
    red[wv][0][c] = pg[i];
    red[wv][1][c] = pb[i];
    red[wv][2][c] = pd[i];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 3 * N; t += 256) {
    const int q = t / N, c = t % N;
    part[((size_t)blockIdx.x * 3 + q) * N + c] = ((red[0][q][c] + red[1][q][c]) + red[2][q][c]) + red[3][q][c];
  }
}

// column sums of the per-block partials: workgroup (q, 64-column chunk); thread (j, c) sums blocks j, j + 4,
// j + 8, ..., then the 4 partial sums are added in a fixed order (deterministic)
__global__ __launch_bounds__(256) void k_ln_colsum(const float* __restrict__ part, int nblk, int N,
                                                   float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                   float* __restrict__ dbias) {
  __shared__ float red[4][64];
  const int chunks = (N + 63) / 64;
  const int q = blockIdx.x / chunks, c = (blockIdx.x % chunks) * 64 + (threadIdx.x & 63), j = threadIdx.x >> 6;
  // 8 independent accumulators (blocks j + 4 * (8 i + u)), so the loads of a thread overlap; combined in order
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    int b = j;
    for (; b + 28 < nblk; b += 32)
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += part[((size_t)(b + 4 * u) * 3 + q) * N + c];
    for (; b < nblk; b += 4) acc[0] += part[((size_t)b * 3 + q) * N + c];
  }
  const float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[j][threadIdx.x & 63] = s;
  __syncthreads();
  if (j == 0 && c < N) {
    const int t = threadIdx.x & 63;
    (q == 0 ? dgamma : q == 1 ? dbeta : dbias)[c] = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
  }
}

// Min-max latent scaling at the end of a dynamics trunk (muzero_deterministic_madn.py:449-457,
// muzero_classic_madn.py:365-371): q = x + (y + bias), out = (q - min q) / (max q - min q + 1e-8) per row
// (one wave per row).  Saved: q, (lo, hi) and the first column of each extremum.
// Backward, with the incoming gradient d = (g + (a + b)) * scale + h (a, b: the carried gradient of the next
// application; h: a gradient that bypasses the 0.5 latent scaling, e.g. the det reward / discount heads which
// read the unscaled next latent, train_with_reward.py:49-105):
//   dq = d / den;  dq[c] += (-sum(d) / den + t) / n_lo for every c with q[c] == lo;  dq[c] += -t / n_hi for
//   every c with q[c] == hi,  t = sum(d (q - lo)) / den^2 -- the extremum's gradient split evenly over tied
//   columns, as JAX's reduce_min / reduce_max JVP does (jnp.min / jnp.max in the Flax modules).
__device__ __forceinline__ void wave_argext(float& v, int& i, bool is_max) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if ((is_max ? ov > v : ov < v) || (ov == v && oi < i)) v = ov, i = oi;
  }
}

template <int N>
__global__ __launch_bounds__(256) void k_minmax_fwd(const float* __restrict__ x, const float* __restrict__ y,
                                                    const float* __restrict__ bias, int M, float* __restrict__ out,
                                                    float* __restrict__ q, float* __restrict__ lohi,
                                                    int* __restrict__ idx) {
  // no fma contraction: the row kernels and their fused boundary forms round identically
#pragma clang fp contract(off)
  constexpr int E = N / 64;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const size_t row = (size_t)m * N;
  float v[E];
  float lo = INFINITY, hi = -INFINITY;
  int ilo = N, ihi = N;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = lane + 64 * e;
    v[e] = x ? x[row + c] + (y[row + c] + bias[c]) : y[row + c] + bias[c];
    q[row + c] = v[e];
    if (v[e] < lo) lo = v[e], ilo = c;
    if (v[e] > hi) hi = v[e], ihi = c;
  }
  wave_argext(lo, ilo, false);
  wave_argext(hi, ihi, true);
  const float den = (hi - lo) + 1e-8f;
#pragma unroll
  for (int e = 0; e < E; ++e) out[row + lane + 64 * e] = (v[e] - lo) / den;
  if (lane == 0) {
    lohi[2 * m] = lo, lohi[2 * m + 1] = hi;
    idx[2 * m] = ilo, idx[2 * m + 1] = ihi;
  }
}

template <int N>
__global__ __launch_bounds__(256) void k_minmax_bwd(const float* __restrict__ g, const float* __restrict__ a,
                                                    const float* __restrict__ b, const float* __restrict__ h,
                                                    float scale, int scaled, const float* __restrict__ q,
                                                    const float* __restrict__ lohi, int M, float* __restrict__ dq) {
  // no fma contraction: the row kernels and their fused boundary forms round identically
#pragma clang fp contract(off)
  constexpr int E = N / 64;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const size_t row = (size_t)m * N;
  const float lo = lohi[2 * m], hi = lohi[2 * m + 1];
  const float den = (hi - lo) + 1e-8f;
  float d[E], qv[E], sd = 0.f, st = 0.f;
  int nlo = 0, nhi = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const size_t k = row + lane + 64 * e;
    float t = g[k];
    if (a) t = t + (a[k] + b[k]);
    if (scaled) t = t * scale;
    if (h) t = t + h[k];
    d[e] = t;
    qv[e] = q[k];
    sd += t;
    st += t * (qv[e] - lo);
    nlo += __popcll(__ballot(qv[e] == lo));
    nhi += __popcll(__ballot(qv[e] == hi));
  }
  sd = wave_sum(sd);
  st = wave_sum(st) / (den * den);
  const float glo = (-sd / den + st) / (float)nlo, ghi = (-st) / (float)nhi;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float r = d[e] / den;
    if (qv[e] == lo) r = r + glo;
    if (qv[e] == hi) r = r + ghi;
    dq[row + lane + 64 * e] = r;
  }
}

// The boundary between two applications of a dynamics trunk as one launch each way (learner._TrunkChain):
// forward = k_minmax_fwd of application i followed by k_ln_fwd<256, FILM> of application i + 1 on the same row
// (its input is the min-max output, still in registers); backward = k_ln_bwd<256, FILM> of application i + 1
// followed by k_minmax_bwd of application i, whose carried gradient a is the LayerNorm input gradient just formed
// (never stored).  Same expressions in the same order as the separate kernels: bit-identical results.
__global__ __launch_bounds__(256) void k_minmax_film_fwd(const float* __restrict__ x, const float* __restrict__ y,
                                                         const float* __restrict__ bias, int M, float* __restrict__ out,
                                                         float* __restrict__ q, float* __restrict__ lohi,
                                                         int* __restrict__ idx, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ scale1,
                                                         const float* __restrict__ shift, float* __restrict__ ln_out,
                                                         float* __restrict__ ln_z, float* __restrict__ ln_mean,
                                                         float* __restrict__ ln_rstd, float* __restrict__ film) {
  // no fma contraction: the row kernels and their fused boundary forms round identically
#pragma clang fp contract(off)
  constexpr int N = 256, E = N / 64;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const size_t row = (size_t)m * N;
  float v[E];
  float lo = INFINITY, hi = -INFINITY;
  int ilo = N, ihi = N;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = lane + 64 * e;
    v[e] = x[row + c] + (y[row + c] + bias[c]);
    q[row + c] = v[e];
    if (v[e] < lo) lo = v[e], ilo = c;
    if (v[e] > hi) hi = v[e], ihi = c;
  }
  wave_argext(lo, ilo, false);
  wave_argext(hi, ihi, true);
  const float den = (hi - lo) + 1e-8f;
  float w[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    w[e] = (v[e] - lo) / den;
    out[row + lane + 64 * e] = w[e];
  }
  if (lane == 0) {
    lohi[2 * m] = lo, lohi[2 * m + 1] = hi;
    idx[2 * m] = ilo, idx[2 * m + 1] = ihi;
  }
  // the next application's LayerNorm_0 + FiLM of this row (k_ln_fwd<256, true>)
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    s += w[e];
    s2 += w[e] * w[e];
  }
  s = wave_sum(s);
  s2 = wave_sum(s2);
  const float mean = s / (float)N;
  const float rstd = 1.0f / sqrtf(fmaxf(0.f, s2 / (float)N - mean * mean) + 1e-6f);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = lane + 64 * e;
    const float o = (w[e] - mean) * (rstd * gamma[c]) + beta[c];
    ln_out[row + c] = o;
    ln_z[row + c] = w[e];
    float p = o * scale1[row + c];
    asm volatile("" : "+v"(p));
    film[row + c] = shift[row + c] + p;
  }
  if (lane == 0) {
    ln_mean[m] = mean;
    ln_rstd[m] = rstd;
  }
}

__global__ __launch_bounds__(256) void k_film_minmax_bwd(const float* __restrict__ dfilm, const float* __restrict__ out,
                                                         const float* __restrict__ z, const float* __restrict__ mean_in,
                                                         const float* __restrict__ rstd_in,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ scale1, int M,
                                                         float* __restrict__ dscale, float* __restrict__ part,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         const float* __restrict__ h, float scale, int scaled,
                                                         const float* __restrict__ q, const float* __restrict__ lohi,
                                                         float* __restrict__ dq) {
  // no fma contraction: the row kernels and their fused boundary forms round identically
#pragma clang fp contract(off)
  constexpr int N = 256, E = N / 64;
  __shared__ float red[4][3][N];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pg[E], pb[E], pd[E], dzr[E];
#pragma unroll
  for (int i = 0; i < E; ++i) pg[i] = pb[i] = pd[i] = dzr[i] = 0.f;
  const int m = blockIdx.x * kLnRowsPerBlock + wv;   // kLnRowsPerBlock == 4: one row per wave
  if (m < M) {
    const size_t row = (size_t)m * N;
    const float mean = mean_in[m], rstd = rstd_in[m];
    float d[E], xh[E], gg[E];
    float a = 0.f, bb = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int c = lane + 64 * i;
      float t = dfilm[row + c];
      dscale[row + c] = t * out[row + c];
      t = t * scale1[row + c];
      d[i] = t;
      xh[i] = (z[row + c] - mean) * rstd;
      gg[i] = t * gamma[c];
      a += gg[i];
      bb += gg[i] * xh[i];
    }
    a = wave_sum(a) / (float)N;
    bb = wave_sum(bb) / (float)N;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      dzr[i] = rstd * (gg[i] - a - xh[i] * bb);
      pg[i] += d[i] * xh[i];
      pb[i] += d[i];
      pd[i] += dzr[i];
    }
    // the previous application's min-max backward (k_minmax_bwd) with a = dzr
    const float lo = lohi[2 * m], hi = lohi[2 * m + 1];
    const float den = (hi - lo) + 1e-8f;
    float dd[E], qv[E], sd = 0.f, st = 0.f;
    int nlo = 0, nhi = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const size_t k = row + lane + 64 * e;
      float t = g[k];
      t = t + (dzr[e] + b[k]);
      if (scaled) t = t * scale;
      if (h) t = t + h[k];
      dd[e] = t;
      qv[e] = q[k];
      sd += t;
      st += t * (qv[e] - lo);
      nlo += __popcll(__ballot(qv[e] == lo));
      nhi += __popcll(__ballot(qv[e] == hi));
    }
    sd = wave_sum(sd);
    st = wave_sum(st) / (den * den);
    const float glo = (-sd / den + st) / (float)nlo, ghi = (-st) / (float)nhi;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float r = dd[e] / den;
      if (qv[e] == lo) r = r + glo;
      if (qv[e] == hi) r = r + ghi;
      dq[row + lane + 64 * e] = r;
    }
  }
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int c = lane + 64 * i;
    red[wv][0][c] = pg[i];
    red[wv][1][c] = pb[i];
    red[wv][2][c] = pd[i];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 3 * N; t += 256) {
    const int qq = t / N, c = t % N;
    part[((size_t)blockIdx.x * 3 + qq) * N + c] = ((red[0][qq][c] + red[1][qq][c]) + red[2][qq][c]) + red[3][qq][c];
  }
}

// 'SAME' Conv1D as one GEMM (learner.MuZeroNets._conv_cols): the im2col matrix of x [B][W][Cin] is
// cols [B][W][K * Cin], cols[b][w][d * Cin + c] = x[b][w + d - (K - 1) / 2][c] (0 outside the row), and its
// backward dx[b][w][c] = sum_d dcols[b][w - d + (K - 1) / 2][d * Cin + c] (d ascending: deterministic).
// x element (b, w, c) at x[b sb + w sw + c sc] (a strided view, e.g. the observation's first channels transposed)
__global__ __launch_bounds__(256) void k_im2col_fwd(const float* __restrict__ x, int B, int W, int Cin, int K,
                                                    int64_t sb, int64_t sw, int64_t sc, float* __restrict__ cols) {
  const int64_t n = (int64_t)B * W * K * Cin;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % Cin);
  const int d = (int)((i / Cin) % K);
  const int64_t bw = i / ((int64_t)K * Cin);
  const int w = (int)(bw % W), src = w + d - (K - 1) / 2;
  const int64_t b = bw / W;
  cols[i] = (src >= 0 && src < W) ? x[b * sb + src * sw + c * sc] : 0.f;
}

__global__ __launch_bounds__(256) void k_im2col_bwd(const float* __restrict__ dcols, int B, int W, int Cin, int K,
                                                    float* __restrict__ dx) {
  const int64_t n = (int64_t)B * W * Cin;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % Cin);
  const int64_t bw = i / Cin;
  const int w = (int)(bw % W);
  float s = 0.f;
  for (int d = 0; d < K; ++d) {
    const int dst = w - d + (K - 1) / 2;
    if (dst >= 0 && dst < W) s += dcols[((bw - w + dst) * K + d) * Cin + c];
  }
  dx[i] = s;
}

static bool ln_width_ok(int N) { return N == 32 || N == 64 || N == 128 || N == 256; }

}  // namespace muz

using namespace muz;

extern "C" {

int muz_ln_fwd_parts(const float* y, int32_t parts, const float* bias, const float* gamma, const float* beta,
                     const float* res, int32_t M, int32_t N, int32_t mode, float* out, float* z, float* mean, float* rstd,
                     void* stream) {
  if (!ln_width_ok(N) || mode < 0 || mode > 2) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && parts >= 1 && y && bias && gamma && beta && out && z && mean && rstd);
  MUZ_HOST_CHECK((mode == LN_MODE_RESID_RELU) == (res != nullptr));
  if (M == 0) return MUZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int grid = (M + 3) / 4;
#define MUZ_LN_FWD(n)                                                                                          \
  k_ln_fwd<n><<<grid, 256, 0, s>>>(y, bias, gamma, beta, res, M, mode, out, z, mean, rstd, nullptr, nullptr, \
                                   nullptr, parts)
  switch (N) {
    case 32: MUZ_LN_FWD(32); break;
    case 64: MUZ_LN_FWD(64); break;
    case 128: MUZ_LN_FWD(128); break;
    default: MUZ_LN_FWD(256); break;
  }
#undef MUZ_LN_FWD
  return muz_last_launch_error();
}

int muz_ln_fwd(const float* y, const float* bias, const float* gamma, const float* beta, const float* res, int32_t M,
               int32_t N, int32_t mode, float* out, float* z, float* mean, float* rstd, void* stream) {
  return muz_ln_fwd_parts(y, 1, bias, gamma, beta, res, M, N, mode, out, z, mean, rstd, stream);
}

int64_t muz_ln_bwd_scratch_floats(int32_t M, int32_t N) {
  if (M < 0 || !ln_width_ok(N)) return -1;
  return (int64_t)((M + kLnRowsPerBlock - 1) / kLnRowsPerBlock) * 3 * N;
}

int muz_ln_bwd_rows_ld(const float* dout, int32_t ldd, const float* out, const float* z, const float* mean,
                       const float* rstd, const float* gamma, int32_t M, int32_t N, int32_t mode, float* dz, float* dres,
                       float* scratch, void* stream) {
  if (!ln_width_ok(N) || mode < 0 || mode > 2) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && ldd >= N && dout && out && z && mean && rstd && gamma && dz && scratch);
  MUZ_HOST_CHECK((mode == LN_MODE_RESID_RELU) == (dres != nullptr));
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (M + kLnRowsPerBlock - 1) / kLnRowsPerBlock;
  if (M > 0) {
#define MUZ_LN_BWD(n)                                                                                        \
  k_ln_bwd<n><<<nblk, 256, 0, s>>>(dout, out, z, mean, rstd, gamma, M, mode, dz, dres, scratch, nullptr, nullptr, \
                                   ldd)
    switch (N) {
      case 32: MUZ_LN_BWD(32); break;
      case 64: MUZ_LN_BWD(64); break;
      case 128: MUZ_LN_BWD(128); break;
      default: MUZ_LN_BWD(256); break;
    }
#undef MUZ_LN_BWD
    return muz_last_launch_error();
  }
  return MUZ_OK;
}

int muz_ln_bwd_rows(const float* dout, const float* out, const float* z, const float* mean, const float* rstd,
                    const float* gamma, int32_t M, int32_t N, int32_t mode, float* dz, float* dres, float* scratch,
                    void* stream) {
  return muz_ln_bwd_rows_ld(dout, N, out, z, mean, rstd, gamma, M, N, mode, dz, dres, scratch, stream);
}

int muz_ln_colsum(const float* scratch, int64_t nblk, int32_t N, float* dgamma, float* dbeta, float* dbias,
                  void* stream) {
  if (!ln_width_ok(N)) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(nblk >= 0 && nblk <= INT32_MAX && scratch && dgamma && dbeta && dbias);
  k_ln_colsum<<<3 * ((N + 63) / 64), 256, 0, (hipStream_t)stream>>>(scratch, (int)nblk, N, dgamma, dbeta, dbias);
  return muz_last_launch_error();
}

int muz_ln_bwd(const float* dout, const float* out, const float* z, const float* mean, const float* rstd,
               const float* gamma, int32_t M, int32_t N, int32_t mode, float* dz, float* dres, float* scratch,
               float* dgamma, float* dbeta, float* dbias, void* stream) {
  MUZ_HOST_CHECK(dgamma && dbeta && dbias);
  const int rc = muz_ln_bwd_rows(dout, out, z, mean, rstd, gamma, M, N, mode, dz, dres, scratch, stream);
  if (rc) return rc;
  return muz_ln_colsum(scratch, muz_ln_bwd_scratch_floats(M, N) / (3 * N), N, dgamma, dbeta, dbias, stream);
}

int muz_ln_film_fwd(const float* x, const float* gamma, const float* beta, const float* scale1, const float* shift,
                    int32_t M, int32_t N, float* out, float* z, float* mean, float* rstd, float* film, void* stream) {
  if (N != 256) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && x && gamma && beta && scale1 && shift && out && z && mean && rstd && film);
  if (M == 0) return MUZ_OK;
  k_ln_fwd<256, true><<<(M + 3) / 4, 256, 0, (hipStream_t)stream>>>(x, nullptr, gamma, beta, nullptr, M, LN_MODE_PLAIN,
                                                                    out, z, mean, rstd, scale1, shift, film);
  return muz_last_launch_error();
}

int muz_ln_film_bwd_rows(const float* dfilm, const float* out, const float* z, const float* mean, const float* rstd,
                         const float* gamma, const float* scale1, int32_t M, int32_t N, float* dz, float* dscale,
                         float* scratch, void* stream) {
  if (N != 256) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && dfilm && out && z && mean && rstd && gamma && scale1 && dz && dscale && scratch);
  if (M == 0) return MUZ_OK;
  k_ln_bwd<256, true><<<(M + kLnRowsPerBlock - 1) / kLnRowsPerBlock, 256, 0, (hipStream_t)stream>>>(
      dfilm, out, z, mean, rstd, gamma, M, LN_MODE_PLAIN, dz, nullptr, scratch, scale1, dscale);
  return muz_last_launch_error();
}

int muz_minmax_fwd(const float* x, const float* y, const float* bias, int32_t M, int32_t N, float* out, float* q,
                   float* lohi, int32_t* idx, void* stream) {
  if (N != 256) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && y && bias && out && q && lohi && idx);
  if (M == 0) return MUZ_OK;
  k_minmax_fwd<256><<<(M + 3) / 4, 256, 0, (hipStream_t)stream>>>(x, y, bias, M, out, q, lohi, idx);
  return muz_last_launch_error();
}

int muz_minmax_bwd(const float* g, const float* a, const float* b, const float* h, float scale, int32_t scaled,
                   const float* q, const float* lohi, int32_t M, int32_t N, float* dq, void* stream) {
  if (N != 256) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && g && q && lohi && dq && (a == nullptr) == (b == nullptr));
  if (M == 0) return MUZ_OK;
  k_minmax_bwd<256><<<(M + 3) / 4, 256, 0, (hipStream_t)stream>>>(g, a, b, h, scale, scaled, q, lohi, M, dq);
  return muz_last_launch_error();
}

int muz_minmax_film_fwd(const float* x, const float* y, const float* bias, int32_t M, int32_t N, float* out, float* q,
                        float* lohi, int32_t* idx, const float* gamma, const float* beta, const float* scale1,
                        const float* shift, float* ln_out, float* ln_z, float* ln_mean, float* ln_rstd, float* film,
                        void* stream) {
  if (N != 256) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && x && y && bias && out && q && lohi && idx && gamma && beta && scale1 && shift && ln_out &&
                 ln_z && ln_mean && ln_rstd && film);
  if (M == 0) return MUZ_OK;
  k_minmax_film_fwd<<<(M + 3) / 4, 256, 0, (hipStream_t)stream>>>(x, y, bias, M, out, q, lohi, idx, gamma, beta, scale1,
                                                                  shift, ln_out, ln_z, ln_mean, ln_rstd, film);
  return muz_last_launch_error();
}

int muz_film_minmax_bwd(const float* dfilm, const float* out, const float* z, const float* mean, const float* rstd,
                        const float* gamma, const float* scale1, int32_t M, int32_t N, float* dscale, float* scratch,
                        const float* g, const float* b, const float* h, float scale, int32_t scaled, const float* q,
                        const float* lohi, float* dq, void* stream) {
  if (N != 256) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && dfilm && out && z && mean && rstd && gamma && scale1 && dscale && scratch && g && b && q &&
                 lohi && dq);
  if (M == 0) return MUZ_OK;
  k_film_minmax_bwd<<<(M + kLnRowsPerBlock - 1) / kLnRowsPerBlock, 256, 0, (hipStream_t)stream>>>(
      dfilm, out, z, mean, rstd, gamma, scale1, M, dscale, scratch, g, b, h, scale, scaled, q, lohi, dq);
  return muz_last_launch_error();
}

int muz_im2col_fwd_strided(const float* x, int32_t B, int32_t W, int32_t Cin, int32_t K, int64_t sb, int64_t sw,
                           int64_t sc, float* cols, void* stream) {
  MUZ_HOST_CHECK(B >= 0 && W > 0 && Cin > 0 && K > 0 && x && cols);
  const int64_t n = (int64_t)B * W * K * Cin;
  if (n == 0) return MUZ_OK;
  k_im2col_fwd<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, B, W, Cin, K, sb, sw, sc, cols);
  return muz_last_launch_error();
}

int muz_im2col_fwd(const float* x, int32_t B, int32_t W, int32_t Cin, int32_t K, float* cols, void* stream) {
  return muz_im2col_fwd_strided(x, B, W, Cin, K, (int64_t)W * Cin, Cin, 1, cols, stream);
}

int muz_im2col_bwd(const float* dcols, int32_t B, int32_t W, int32_t Cin, int32_t K, float* dx, void* stream) {
  MUZ_HOST_CHECK(B >= 0 && W > 0 && Cin > 0 && K > 0 && dcols && dx);
  const int64_t n = (int64_t)B * W * Cin;
  if (n == 0) return MUZ_OK;
  k_im2col_bwd<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(dcols, B, W, Cin, K, dx);
  return muz_last_launch_error();
}

}  // extern "C"
