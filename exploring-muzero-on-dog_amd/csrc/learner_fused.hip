// One launch per learner layer instead of two: the Dense GEMM fused with its LayerNorm epilogue (forward) and
// the LayerNorm backward fused with the input-gradient GEMM (backward).  Every Dense -> LayerNorm [-> ReLU]
// [-> + residual -> ReLU] of Repr2 / DynamicsNetwork4 / Pred4 (muzero_deterministic_madn.py,
// muzero_classic_madn.py; trained by train_with_reward.py:24-164 / train_stochastic.py:34-199) goes through
// these two kernels; at batch 128 x unroll 10 each launch is latency-bound (a few microseconds), so halving the
// launch count is what shortens the step.
//
// Tiles: one workgroup per 16 rows, N / 32 waves (wave w owns output columns 32 w .. + 31 as two 16-column
// MFMA tiles).  v_mfma_f32_16x16x4_f32 computes the transposed tile (the weights are the A operand), so lane l
// ends with 4 consecutive columns 4 (l / 16) .. + 3 of row l % 16.
//
// Forward (x [M][K] -> out [M][N]):  the 16 x K input tile is staged in LDS (row stride K16 + 4: the
//   conflict-free b128 read of lane (i, g) at row i, columns 16 b + 4 g .. + 3); the weights stream from
//   global / L2 (column reads, 4 k-blocks in flight); y + bias lands in LDS and the row epilogue is k_ln_fwd's
//   arithmetic (Flax LayerNorm, fast variance E[z^2] - E[z]^2, eps 1e-6) with 4 W threads per row, 8 columns
//   each.  Saved: out, z = y + bias, mean, rstd (what muz_ln_bwd_rows reads).
// Backward (dout [M][N] -> dz, dres, dx [M][K]):  k_ln_bwd's row arithmetic into an LDS dz tile (and dz to
//   global for the grouped weight gradient), per-tile column partials (dgamma, dbeta, dbias) in
//   muz_ln_bwd_rows' scratch layout [tiles][3][N], then dx = dz W^T (+ acc), one 16-column tile of K per wave
//   and the K tiles spread over a second grid dimension; the A operand W[k][16 b + 4 g .. + 3] is one 16-byte
//   load per lane.
#include "launch.hpp"

namespace muz {

typedef float f32x4_u __attribute__((ext_vector_type(4)));

enum { FLN_PLAIN = 0, FLN_RELU = 1, FLN_RESID_RELU = 2 };
constexpr int kFRows = 16;

__host__ __device__ constexpr int fused_k16(int K) { return (K + 15) / 16 * 16; }
__host__ __device__ constexpr int fused_ld(int K) { return fused_k16(K) + 4; }

__device__ __forceinline__ f32x4_u mfma_u(float a, float b, f32x4_u c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// sum over the T consecutive lanes that share a row (T a power of two <= 64, rows aligned to T)
template <int T>
__device__ __forceinline__ float row_sum_t(float v) {
#pragma unroll
  for (int o = T / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- forward -------------------------------------------------------------------------------------------
// Weights as the A operand: lane (i, g) needs W[16 b + 4 g + j][n0 + i] for j = 0..3.  With TR the caller
// passes W^T zero-padded to [N][ldw] (ldw >= K16, a multiple of 4: learner.WeightTranspose keeps one per
// layer, refreshed once per step), so that is one 16-byte load per lane and tile; without it, four 4-byte
// column loads.
template <bool TR>
struct FwdW {
  f32x4_u w0, w1;
};

template <bool TR>
__device__ __forceinline__ void fwd_wload(FwdW<TR>& B, const float* __restrict__ W, int ldw, int K, int N, int n0,
                                          int blk) {
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int kb = 16 * blk + 4 * g;
  if constexpr (TR) {
    B.w0 = *reinterpret_cast<const f32x4_u*>(W + (size_t)(n0 + i) * ldw + kb);
    B.w1 = *reinterpret_cast<const f32x4_u*>(W + (size_t)(n0 + 16 + i) * ldw + kb);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* wr = W + (size_t)(kb + j) * N + n0 + i;
      B.w0[j] = kb + j < K ? wr[0] : 0.f;
      B.w1[j] = kb + j < K ? wr[16] : 0.f;
    }
  }
}

// acc[t][j & 1]: four independent accumulation chains per wave (a dependent MFMA waits for its predecessor)
template <bool TR>
__device__ __forceinline__ void fwd_mma(const FwdW<TR>& B, const float* xs, int ld, int blk, f32x4_u (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const f32x4_u x = *reinterpret_cast<const f32x4_u*>(xs + i * ld + 16 * blk + 4 * g);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc[0][j & 1] = mfma_u(B.w0[j], x[j], acc[0][j & 1]);
    acc[1][j & 1] = mfma_u(B.w1[j], x[j], acc[1][j & 1]);
  }
}

// KB > 0: the layer's k-block count as a compile-time constant, so the weight ring below is straight-line code
// (static buffer indices, exact s_waitcnt counts: with a runtime trip count the compiler waited for every
// load at every block).  KB = 0: any K, one block at a time.
template <int N, bool TR, int KB>
__global__ __launch_bounds__(2 * N) void k_dense_ln_fwd(const float* __restrict__ x, int M, int K,
                                                        const float* __restrict__ W, int ldw,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, const float* __restrict__ res,
                                                        int mode, float* __restrict__ out, float* __restrict__ z,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int NW = N / 32, NTH = 64 * NW, TPR = NTH / kFRows;   // waves, threads, threads per row
  constexpr int LDY = N + 4;
  constexpr int D = KB > 0 ? (KB < 8 ? KB : 8) : 1;              // k-blocks of weights in flight
  extern __shared__ float smem[];
  const int ld = fused_ld(K), K16 = fused_k16(K);
  float* xs = smem;                      // [16][ld]
  float* ys = smem + kFRows * ld;        // [16][LDY]
  const int r0 = blockIdx.x * kFRows, tid = threadIdx.x;
  const int n0 = 32 * (tid >> 6);
  // the first weight blocks fly while the input tile is staged
  FwdW<TR> buf[D];
  if constexpr (KB > 0) {
#pragma unroll
    for (int p = 0; p < D - 1; ++p) fwd_wload<TR>(buf[p], W, ldw, K, N, n0, p);
  }
  if ((K & 3) == 0) {
    const int q = K16 / 4;
    for (int e = tid; e < kFRows * q; e += NTH) {
      const int r = e / q, k = 4 * (e - r * q);
      f32x4_u v = {0.f, 0.f, 0.f, 0.f};
      if (r0 + r < M && k < K) v = *reinterpret_cast<const f32x4_u*>(x + (size_t)(r0 + r) * K + k);
      *reinterpret_cast<f32x4_u*>(xs + r * ld + k) = v;
    }
  } else {
    for (int e = tid; e < kFRows * K16; e += NTH) {
      const int r = e / K16, k = e - r * K16;
      xs[r * ld + k] = (r0 + r < M && k < K) ? x[(size_t)(r0 + r) * K + k] : 0.f;
    }
  }
  __syncthreads();
  f32x4_u acc4[2][2] = {};
  if constexpr (KB > 0) {
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      if (b + D - 1 < KB) fwd_wload<TR>(buf[(b + D - 1) % D], W, ldw, K, N, n0, b + D - 1);
      // pin the issue point: the scheduler otherwise sinks each load next to its first MFMA
      __builtin_amdgcn_sched_barrier(0);
      fwd_mma<TR>(buf[b % D], xs, ld, b, acc4);
    }
  } else {
    for (int b = 0; b < K16 / 16; ++b) {
      fwd_wload<TR>(buf[0], W, ldw, K, N, n0, b);
      fwd_mma<TR>(buf[0], xs, ld, b, acc4);
    }
  }
  const f32x4_u acc[2] = {acc4[0][0] + acc4[0][1], acc4[1][0] + acc4[1][1]};
  const int lane = tid & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = n0 + 16 * t + 4 * g;
    const f32x4_u bb = *reinterpret_cast<const f32x4_u*>(bias + c);
    *reinterpret_cast<f32x4_u*>(ys + i * LDY + c) = acc[t] + bb;
  }
  // row epilogue: thread (row, sub) owns columns 8 sub .. + 7 (its gamma / beta / residual loads are issued
  // before the barrier)
  const int row = tid / TPR, sub = tid % TPR, m = r0 + row;
  const int c0 = 8 * sub;
  const size_t o = (size_t)m * N + c0;
  const f32x4_u ga = *reinterpret_cast<const f32x4_u*>(gamma + c0), gb = *reinterpret_cast<const f32x4_u*>(gamma + c0 + 4);
  const f32x4_u ba = *reinterpret_cast<const f32x4_u*>(beta + c0), bb2 = *reinterpret_cast<const f32x4_u*>(beta + c0 + 4);
  f32x4_u ra = {0.f, 0.f, 0.f, 0.f}, rb = ra;
  if (mode == FLN_RESID_RELU && m < M) {
    ra = *reinterpret_cast<const f32x4_u*>(res + o);
    rb = *reinterpret_cast<const f32x4_u*>(res + o + 4);
  }
  __syncthreads();
  const f32x4_u va = *reinterpret_cast<const f32x4_u*>(ys + row * LDY + c0);
  const f32x4_u vb = *reinterpret_cast<const f32x4_u*>(ys + row * LDY + c0 + 4);
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    s += va[e] + vb[e];
    s2 += va[e] * va[e] + vb[e] * vb[e];
  }
  s = row_sum_t<TPR>(s);
  s2 = row_sum_t<TPR>(s2);
  if (m >= M) return;
  const float mean = s / (float)N;
  const float rstd = 1.0f / sqrtf(fmaxf(0.f, s2 / (float)N - mean * mean) + 1e-6f);
  f32x4_u oa, ob;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float t0 = (va[e] - mean) * (rstd * ga[e]) + ba[e];
    float t1 = (vb[e] - mean) * (rstd * gb[e]) + bb2[e];
    if (mode == FLN_RELU) t0 = fmaxf(t0, 0.f), t1 = fmaxf(t1, 0.f);
    if (mode == FLN_RESID_RELU) t0 = fmaxf(ra[e] + t0, 0.f), t1 = fmaxf(rb[e] + t1, 0.f);
    oa[e] = t0;
    ob[e] = t1;
  }
  *reinterpret_cast<f32x4_u*>(out + o) = oa;
  *reinterpret_cast<f32x4_u*>(out + o + 4) = ob;
  *reinterpret_cast<f32x4_u*>(z + o) = va;
  *reinterpret_cast<f32x4_u*>(z + o + 4) = vb;
  if (sub == 0) {
    mean_out[m] = mean;
    rstd_out[m] = rstd;
  }
}

// W [K][N] -> W^T [N][ldt] (columns >= K left as they are: the caller zero-fills once), 32 x 32 tiles through LDS
struct TransposeTable {
  const float* src[48];
  float* dst[48];
  int K[48], N[48], ldt[48], tiles_n[48], wg0[49];
  int count;
};

__global__ __launch_bounds__(256) void k_transpose_grouped(TransposeTable t) {
  __shared__ float tile[32][33];
  const int wg = blockIdx.x;
  int p = 0;
  while (p + 1 < t.count && t.wg0[p + 1] <= wg) ++p;
  const int local = wg - t.wg0[p];
  const int k0 = (local / t.tiles_n[p]) * 32, n0 = (local % t.tiles_n[p]) * 32;
  const int K = t.K[p], N = t.N[p];
  const int cx = threadIdx.x & 31, cy = threadIdx.x >> 5;   // 8 rows per pass
#pragma unroll
  for (int r = cy; r < 32; r += 8)
    if (k0 + r < K && n0 + cx < N) tile[r][cx] = t.src[p][(size_t)(k0 + r) * N + n0 + cx];
  __syncthreads();
#pragma unroll
  for (int r = cy; r < 32; r += 8)
    if (n0 + r < N && k0 + cx < K) t.dst[p][(size_t)(n0 + r) * t.ldt[p] + k0 + cx] = tile[cx][r];
}

// ---- backward ------------------------------------------------------------------------------------------
// Grid (row tile, k-block): every workgroup of a row tile redoes the (cheap) LayerNorm half for its 16 rows --
// the input gradient needs whole dz rows -- and computes 16 * N / 32 of dx's K columns (one 16-column tile per
// wave), so a layer's MFMA work spreads over ceil(K / (16 * waves)) CUs per row tile; k-block 0 alone writes
// dz, dres and the column partials.
template <int N>
__global__ __launch_bounds__(2 * N) void k_dense_ln_bwd(const float* __restrict__ dout,
                                                        const float* __restrict__ out, const float* __restrict__ z,
                                                        const float* __restrict__ mean_in,
                                                        const float* __restrict__ rstd_in,
                                                        const float* __restrict__ gamma, int M, int mode,
                                                        const float* __restrict__ W, int K,
                                                        const float* __restrict__ acc_in, float* __restrict__ dz,
                                                        float* __restrict__ dres, float* __restrict__ dx,
                                                        float* __restrict__ part, int ldd) {
  constexpr int NW = N / 32, NTH = 64 * NW, TPR = NTH / kFRows;
  constexpr int LDZ = N + 4;
  __shared__ float dzs[kFRows][LDZ];
  __shared__ float pgs[kFRows][N];       // per-row do * xhat and do, for the column partials
  __shared__ float pbs[kFRows][N];
  const int tid = threadIdx.x, r0 = blockIdx.x * kFRows;
  const bool lead = blockIdx.y == 0;     // writes dz / dres / partials
  const int row = tid / TPR, sub = tid % TPR, m = r0 + row, c0 = 8 * sub;
  // dx's weight blocks W[k][16 b + 4 g .. + 3] of the wave's k tile; the first D - 1 are issued here so they
  // fly during the LayerNorm half (rows past K read row K - 1 and are never stored: no branch around the
  // load, so the compiler keeps exact s_waitcnt counts)
  constexpr int KB = N / 16;
  constexpr int D = KB < 4 ? KB : 4;
  const int lane = tid & 63, wv = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int ktile = wv + NW * blockIdx.y;
  const float* wrow = W ? W + (size_t)min(16 * ktile + li, K - 1) * N + 4 * lg : nullptr;
  f32x4_u wbuf[D];
  if (dx) {
#pragma unroll
    for (int p = 0; p < D - 1; ++p) wbuf[p] = *reinterpret_cast<const f32x4_u*>(wrow + 16 * p);
  }
  float d[8], xh[8], gg[8];
  float a = 0.f, b = 0.f;
  if (m < M) {
    const size_t o = (size_t)m * N + c0;
    const float mean = mean_in[m], rstd = rstd_in[m];
    float ov[8], zv[8];
    const float* dr = dout + (size_t)m * ldd + c0;   // (rows ldd apart: a column slice of a wider gradient)
    *reinterpret_cast<f32x4_u*>(d) = *reinterpret_cast<const f32x4_u*>(dr);
    *reinterpret_cast<f32x4_u*>(d + 4) = *reinterpret_cast<const f32x4_u*>(dr + 4);
    *reinterpret_cast<f32x4_u*>(ov) = *reinterpret_cast<const f32x4_u*>(out + o);
    *reinterpret_cast<f32x4_u*>(ov + 4) = *reinterpret_cast<const f32x4_u*>(out + o + 4);
    *reinterpret_cast<f32x4_u*>(zv) = *reinterpret_cast<const f32x4_u*>(z + o);
    *reinterpret_cast<f32x4_u*>(zv + 4) = *reinterpret_cast<const f32x4_u*>(z + o + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (mode != FLN_PLAIN && !(ov[e] > 0.f)) d[e] = 0.f;
      xh[e] = (zv[e] - mean) * rstd;
      gg[e] = d[e] * gamma[c0 + e];
      a += gg[e];
      b += gg[e] * xh[e];
    }
    if (mode == FLN_RESID_RELU && lead) {
      *reinterpret_cast<f32x4_u*>(dres + o) = *reinterpret_cast<const f32x4_u*>(d);
      *reinterpret_cast<f32x4_u*>(dres + o + 4) = *reinterpret_cast<const f32x4_u*>(d + 4);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = xh[e] = gg[e] = 0.f;
  }
  a = row_sum_t<TPR>(a) / (float)N;
  b = row_sum_t<TPR>(b) / (float)N;
  float dzv[8];
  const float rstd = m < M ? rstd_in[m] : 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    dzv[e] = m < M ? rstd * (gg[e] - a - xh[e] * b) : 0.f;
    dzs[row][c0 + e] = dzv[e];
    if (lead) {
      pgs[row][c0 + e] = d[e] * xh[e];
      pbs[row][c0 + e] = d[e];
    }
  }
  if (m < M && lead) {
    const size_t o = (size_t)m * N + c0;
    *reinterpret_cast<f32x4_u*>(dz + o) = *reinterpret_cast<const f32x4_u*>(dzv);
    *reinterpret_cast<f32x4_u*>(dz + o + 4) = *reinterpret_cast<const f32x4_u*>(dzv + 4);
  }
  __syncthreads();
  if (lead) {   // column partials of this tile (rows in order), muz_ln_bwd_rows' layout: [tile][dgamma, dbeta, dbias][N]
    for (int c = tid; c < N; c += NTH) {
      float sg = 0.f, sb = 0.f, sd = 0.f;
#pragma unroll
      for (int r = 0; r < kFRows; ++r) {
        sg += pgs[r][c];
        sb += pbs[r][c];
        sd += dzs[r][c];
      }
      float* p = part + (size_t)blockIdx.x * 3 * N + c;
      p[0] = sg;
      p[N] = sb;
      p[2 * N] = sd;
    }
  }
  if (!dx || 16 * ktile >= K) return;
  // dx[16][16 ktile .. + 15] = dz[16][N] W^T (+ acc)
  f32x4_u acc2[2] = {};
#pragma unroll
  for (int bk = 0; bk < KB; ++bk) {
    if (bk + D - 1 < KB) wbuf[(bk + D - 1) % D] = *reinterpret_cast<const f32x4_u*>(wrow + 16 * (bk + D - 1));
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch D - 1 blocks ahead of its MFMAs
    const f32x4_u bx = *reinterpret_cast<const f32x4_u*>(&dzs[li][16 * bk + 4 * lg]);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[j & 1] = mfma_u(wbuf[bk % D][j], bx[j], acc2[j & 1]);
  }
  const int mr = r0 + li, kc = 16 * ktile + 4 * lg;
  if (mr >= M || kc >= K) return;
  const size_t o = (size_t)mr * K + kc;
  f32x4_u v = acc2[0] + acc2[1];
  if ((K & 3) == 0) {
    if (acc_in) v += *reinterpret_cast<const f32x4_u*>(acc_in + o);
    *reinterpret_cast<f32x4_u*>(dx + o) = v;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (kc + e < K) dx[o + e] = acc_in ? acc_in[o + e] + v[e] : v[e];
  }
}

static bool fused_width_ok(int N) { return N == 32 || N == 64 || N == 128 || N == 256; }

}  // namespace muz

using namespace muz;

extern "C" {

int muz_dense_ln_fwd(const float* x, int32_t M, int32_t K, const float* W, const float* WT, int32_t ldt,
                     const float* bias, const float* gamma, const float* beta, const float* res, int32_t N,
                     int32_t mode, float* out, float* z, float* mean, float* rstd, void* stream) {
  if (!fused_width_ok(N) || mode < 0 || mode > 2 || K > 512) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && K > 0 && x && (W || WT) && bias && gamma && beta && out && z && mean && rstd);
  MUZ_HOST_CHECK(!WT || (ldt >= fused_k16(K) && ldt % 4 == 0));
  MUZ_HOST_CHECK((mode == FLN_RESID_RELU) == (res != nullptr));
  if (M == 0) return MUZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int grid = (M + kFRows - 1) / kFRows;
  const size_t lds = (size_t)kFRows * (fused_ld(K) + N + 4) * sizeof(float);
#define MUZ_DLF(n, tr, kb, w, l)                                                                          \
  k_dense_ln_fwd<n, tr, kb><<<grid, 2 * n, lds, s>>>(x, M, K, w, l, bias, gamma, beta, res, mode, out, z, mean, rstd)
  // compile-time k-block counts of the learner's layers (K = 16 KB): 1 / 2 (embeddings, Conv_0), 4, 6 (Conv_1),
  // 16 (the 256-wide trunks), 20 (Conv_2, Dense_3)
#define MUZ_DLF_N(n)                                     \
  if (!WT) {                                             \
    MUZ_DLF(n, false, 0, W, N);                          \
  } else {                                               \
    switch (fused_k16(K) / 16) {                         \
      case 1: MUZ_DLF(n, true, 1, WT, ldt); break;       \
      case 2: MUZ_DLF(n, true, 2, WT, ldt); break;       \
      case 4: MUZ_DLF(n, true, 4, WT, ldt); break;       \
      case 6: MUZ_DLF(n, true, 6, WT, ldt); break;       \
      case 16: MUZ_DLF(n, true, 16, WT, ldt); break;     \
      case 20: MUZ_DLF(n, true, 20, WT, ldt); break;     \
      default: MUZ_DLF(n, true, 0, WT, ldt); break;      \
    }                                                    \
  }
  switch (N) {
    case 32: MUZ_DLF_N(32); break;
    case 64: MUZ_DLF_N(64); break;
    case 128: MUZ_DLF_N(128); break;
    default: MUZ_DLF_N(256); break;
  }
#undef MUZ_DLF_N
#undef MUZ_DLF
  return muz_last_launch_error();
}

int muz_transpose_grouped(const muz_transpose_problem* probs, int32_t count, void* stream) {
  MUZ_HOST_CHECK(count >= 0 && (count == 0 || probs));
  for (int s0 = 0; s0 < count; s0 += 48) {
    TransposeTable t{};
    int wgs = 0;
    for (int i = s0; i < count && t.count < 48; ++i) {
      const muz_transpose_problem& q = probs[i];
      MUZ_HOST_CHECK(q.src && q.dst && q.K > 0 && q.N > 0 && q.ldt >= q.K);
      const int c = t.count++;
      t.src[c] = q.src, t.dst[c] = q.dst, t.K[c] = q.K, t.N[c] = q.N, t.ldt[c] = q.ldt;
      t.tiles_n[c] = (q.N + 31) / 32;
      t.wg0[c] = wgs;
      wgs += ((q.K + 31) / 32) * t.tiles_n[c];
    }
    t.wg0[t.count] = wgs;
    if (!wgs) continue;
    k_transpose_grouped<<<wgs, 256, 0, (hipStream_t)stream>>>(t);
    const int rc = muz_last_launch_error();
    if (rc) return rc;
  }
  return MUZ_OK;
}

int64_t muz_dense_ln_bwd_scratch_floats(int32_t M, int32_t N) {
  if (M < 0 || !fused_width_ok(N)) return -1;
  return (int64_t)((M + kFRows - 1) / kFRows) * 3 * N;
}

int muz_dense_ln_bwd_ld(const float* dout, int32_t ldd, const float* out, const float* z, const float* mean,
                        const float* rstd, const float* gamma, int32_t M, int32_t N, int32_t mode, const float* W,
                        int32_t K, const float* acc, float* dz, float* dres, float* dx, float* scratch, void* stream) {
  if (!fused_width_ok(N) || mode < 0 || mode > 2) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(M >= 0 && dout && out && z && mean && rstd && gamma && dz && scratch);
  MUZ_HOST_CHECK(ldd >= N && ldd % 4 == 0 && ((uintptr_t)dout & 15u) == 0);   // (16-byte row loads)
  MUZ_HOST_CHECK((mode == FLN_RESID_RELU) == (dres != nullptr));
  MUZ_HOST_CHECK(!dx || (W && K > 0));
  MUZ_HOST_CHECK(!acc || dx);
  if (M == 0) return MUZ_OK;
  const int NW = N / 32, kblocks = dx ? ((K + 15) / 16 + NW - 1) / NW : 1;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((M + kFRows - 1) / kFRows, kblocks);
#define MUZ_DLB(n) \
  k_dense_ln_bwd<n><<<grid, 2 * n, 0, s>>>(dout, out, z, mean, rstd, gamma, M, mode, W, K, acc, dz, dres, dx, scratch, \
                                           ldd)
  switch (N) {
    case 32: MUZ_DLB(32); break;
    case 64: MUZ_DLB(64); break;
    case 128: MUZ_DLB(128); break;
    default: MUZ_DLB(256); break;
  }
#undef MUZ_DLB
  return muz_last_launch_error();
}

int muz_dense_ln_bwd(const float* dout, const float* out, const float* z, const float* mean, const float* rstd,
                     const float* gamma, int32_t M, int32_t N, int32_t mode, const float* W, int32_t K,
                     const float* acc, float* dz, float* dres, float* dx, float* scratch, void* stream) {
  return muz_dense_ln_bwd_ld(dout, N, out, z, mean, rstd, gamma, M, N, mode, W, K, acc, dz, dres, dx, scratch, stream);
}

}  // extern "C"
