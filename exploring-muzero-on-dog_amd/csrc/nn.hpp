// Fused fp32 MLP building blocks for 16-row tiles on CDNA4 MFMA (v_mfma_f32_16x16x4_f32).
//
// A workgroup of 8 waves (two per SIMD, so one wave's weight loads hide under the other's MFMAs)
// owns a tile of 16 rows (games).  Activations live in LDS ([16][ld] fp32 rows); a dense layer
// out = A[16][K] @ W[K][N] + b splits its N columns over the 8 waves (NT 16-column tiles each).  Per 16-deep k-block a lane reads ONE float4 of A from
// LDS (row lane&15, k = kb*16 + 4*(lane>>4) + j, j = 0..3) and NT float4 of pre-packed weights
// straight from global memory (L2/MALL resident, streamed once per tile), then issues 4*NT
// MFMAs, with the weights of the next two k-blocks in flight.  The f32-input MFMA is an exact
// k-ordered fma chain, so only the reduction order differs from the fp32 reference.  Row-wise ops
// (LayerNorm, min-max) use 32 lanes (half a wave) per row.
#pragma once
#include "common.hpp"

namespace muz {

constexpr int kRows = 16;
constexpr int kRowLanes = 32;                 // lanes per row in row-wise phases
constexpr int kThreads = kRows * kRowLanes;   // 512
constexpr int kWaves = kThreads / 64;         // 8
constexpr int LAT = 256;

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[t] += A[16 rows][K] @ Wgroup[K][NT*16]  (KB = K/16 k-blocks; Wg = packed weights of this group).
// b0 / b1 hold k-blocks 0 and 1 on entry.  Weights for k-blocks kb+1 and kb+2 are in flight while kb is
// multiplied (3-deep register ring, written as a 3-way unrolled loop so every index is static).
template <int NT, bool AG>
__device__ __forceinline__ void mfma_ring_impl(const float* __restrict__ Wg, int KB, const float* A, int lda,
                                               f32x4 (&acc)[NT], f32x4 (&b0)[NT], f32x4 (&b1)[NT]) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(Wg)) + lane * NT;
  const int wstep = 64 * NT;   // f32x4 per k-block
  const float* ap = A + r * lda + 4 * g;
  auto lda4 = [&](int kb) -> f32x4 {
    if constexpr (AG) return *gp(reinterpret_cast<const f32x4*>(ap + kb * 16));
    else return *reinterpret_cast<const f32x4*>(ap + kb * 16);
  };
  f32x4 b2[NT];
  // step kb: issue k-block kb+2 into `nxt` (the buffer consumed at step kb-1), multiply `cur` (= kb)
  auto step = [&](int kb, const f32x4 (&cur)[NT], f32x4 (&nxt)[NT]) {
    if (kb + 2 < KB) {
#pragma unroll
      for (int t = 0; t < NT; ++t) nxt[t] = wp[(kb + 2) * wstep + t];
    }
    const f32x4 a = lda4(kb);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[j], cur[t][j], acc[t]);
  };
  int kb = 0;
  for (; kb + 3 <= KB; kb += 3) {
    step(kb, b0, b2);
    step(kb + 1, b1, b0);
    step(kb + 2, b2, b1);
  }
  if (kb < KB) step(kb, b0, b2);
  if (kb + 1 < KB) step(kb + 1, b1, b0);
}

template <int NT>
__device__ __forceinline__ void mfma_ring(const float* __restrict__ Wg, int KB, const float* A, int lda,
                                          f32x4 (&acc)[NT], f32x4 (&b0)[NT], f32x4 (&b1)[NT], bool a_global) {
  if (a_global)
    mfma_ring_impl<NT, true>(Wg, KB, A, lda, acc, b0, b1);
  else
    mfma_ring_impl<NT, false>(Wg, KB, A, lda, acc, b0, b1);
}

template <int NT>
__device__ __forceinline__ void mfma_rows16(const float* __restrict__ Wg, int KB, const float* A, int lda,
                                            f32x4 (&acc)[NT]) {
  const int lane = threadIdx.x & 63;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(Wg)) + lane * NT;
  f32x4 b0[NT], b1[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    b0[t] = wp[t];
    b1[t] = KB > 1 ? wp[64 * NT + t] : b0[t];
  }
  mfma_ring_impl<NT, false>(Wg, KB, A, lda, acc, b0, b1);
}

// ---- cross-layer weight prefetch ----------------------------------------------------------------
// Every dense layer issues the first two k-blocks of the NEXT layer's weights for this wave before its
// epilogue, so the loads fly across the epilogue, the barrier and the LayerNorm pass in between.
constexpr int kPfMax = 4;
struct Pf {
  f32x4 v0[kPfMax], v1[kPfMax];
};

__device__ __forceinline__ const float* wave_group(const AS4 muz_dense& L, int KB, int NT) {
  return L.w + (size_t)(threadIdx.x >> 6) * KB * 64 * NT * 4;
}

template <int NT>
__device__ __forceinline__ void pf_issue(Pf& pf, const AS4 muz_dense* L, int K, int N) {
  static_assert(NT <= kPfMax, "prefetch buffer too small");
  if (!L) return;
  const int KB = (K + 15) >> 4;
  if ((threadIdx.x >> 6) * NT * 16 >= N) return;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(wave_group(*L, KB, NT))) + (threadIdx.x & 63) * NT;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    pf.v0[t] = wp[t];
    if (KB > 1) pf.v1[t] = wp[64 * NT + t];
  }
}

// Dense layer over the tile: out[16][N] = A @ W + b, waves split N (NT tiles of 16 columns each).
// `pf` holds this layer's first k-blocks on entry and the next layer's (Ln: K=Kn, N=Nn, NTN tiles)
// on exit.  A may live in LDS or global memory.  Caller synchronises before/after.
template <int NT, int NTN>
__device__ __forceinline__ void dense16(const AS4 muz_dense& L, int K, int N, const float* A, int lda, float* out,
                                        int ldo, Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn,
                                        bool a_global = false) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int KB = (K + 15) >> 4;
  const int col0 = wv * NT * 16;
  if (col0 >= N) {
    pf_issue<NTN>(pf, Ln, Kn, Nn);
    return;
  }
  f32x4 acc[NT], b0[NT], b1[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    b0[t] = pf.v0[t];
    b1[t] = pf.v1[t];
  }
  mfma_ring<NT>(wave_group(L, KB, NT), KB, A, lda, acc, b0, b1, a_global);
  pf_issue<NTN>(pf, Ln, Kn, Nn);
  const int r = lane & 15, g = lane >> 4;
  const AS1 float* bias = gp(L.b);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = col0 + t * 16 + r;
    if (col < N) {
      const float bb = bias[col];
#pragma unroll
      for (int i = 0; i < 4; ++i) out[(4 * g + i) * ldo + col] = acc[t][i] + bb;
    }
  }
}

// ---- row-wise ops: thread t -> row t/32, lane-in-row t%32 (half a wave per row) ---------------------
__device__ __forceinline__ int trow() { return threadIdx.x >> 5; }
__device__ __forceinline__ int tsub() { return threadIdx.x & 31; }
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m, 32);
  return v;
}
__device__ __forceinline__ float row_max(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 32));
  return v;
}
__device__ __forceinline__ float row_min(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v = fminf(v, __shfl_xor(v, m, 32));
  return v;
}
__device__ __forceinline__ int row_isum(int v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m, 32);
  return v;
}
__device__ __forceinline__ int row_imax(int v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, 32));
  return v;
}

enum LnMode { LN_PLAIN = 0, LN_RELU = 1, LN_RESID_RELU = 2 };

// Flax LayerNorm (eps 1e-6, fast variance) of in[16][N] -> out.
//   LN_PLAIN: out = y;  LN_RELU: out = relu(y);  LN_RESID_RELU: out = relu(out + y)  (ResBlock tail)
template <int N, int MODE>
__device__ __forceinline__ void ln16(const float* in, int ldi, float* out, int ldo, const AS4 muz_ln& P) {
  constexpr int PER = N / kRowLanes;
  const int row = trow(), sub = tsub();
  const AS1 float* scale = gp(P.scale);
  const AS1 float* shift = gp(P.bias);
  float sc[PER], sh[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {   // parameter loads first, so they overlap the statistics
    sc[i] = scale[sub + kRowLanes * i];
    sh[i] = shift[sub + kRowLanes * i];
  }
  float v[PER];
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = in[row * ldi + sub + kRowLanes * i];
    s += v[i];
    s2 += v[i] * v[i];
  }
  s = row_sum(s);
  s2 = row_sum(s2);
  const float mean = s / (float)N;
  const float mean2 = s2 / (float)N;
  const float var = fmaxf(0.f, mean2 - mean * mean);
  const float inv = 1.0f / sqrtf(var + 1e-6f);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = sub + kRowLanes * i;
    float y = (v[i] - mean) * (inv * sc[i]) + sh[i];
    if (MODE == LN_RELU) y = fmaxf(y, 0.f);
    if (MODE == LN_RESID_RELU) y = fmaxf(out[row * ldo + c] + y, 0.f);
    out[row * ldo + c] = y;
  }
}

// x <- (x - min) / (max - min + 1e-8) per row of 256 (Repr2 139-140, Dyn4 435-437).
__device__ __forceinline__ void minmax16(float* buf, int ld) {
  constexpr int PER = LAT / kRowLanes;
  const int row = trow(), sub = tsub();
  float v[PER];
  float lo = INFINITY, hi = -INFINITY;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = buf[row * ld + sub + kRowLanes * i];
    lo = fminf(lo, v[i]);
    hi = fmaxf(hi, v[i]);
  }
  lo = row_min(lo);
  hi = row_max(hi);
  const float den = hi - lo + 1e-8f;
#pragma unroll
  for (int i = 0; i < PER; ++i) buf[row * ld + sub + kRowLanes * i] = (v[i] - lo) / den;
}

__device__ __forceinline__ void relu16(float* buf, int ld, int col0, int n) {
  const int row = trow(), sub = tsub();
  for (int c = sub; c < n; c += kRowLanes) buf[row * ld + col0 + c] = fmaxf(buf[row * ld + col0 + c], 0.f);
}

// ---- LDS arena of a 16-row tile ---------------------------------------------------------------------
constexpr int LD = LAT + 4;      // 260: row stride of 256-wide buffers (keeps b128 reads 16B aligned)
constexpr int LDW = 512 + 4;     // wide buffer (FiLM scale|shift 512, pred heads 384, concat 320)
constexpr int LDE = 64 + 4;      // small buffer (action embed, global features)
constexpr int kArenaFloats = 4 * kRows * LD + kRows * LDW + kRows * LDE + 4 * kRows;

struct Arena {
  float* L;   // latent input (parent embedding)           [16][LD]
  float* X;   // working activation                        [16][LD]
  float* T;   // scratch / next latent                     [16][LD]
  float* U;   // scratch / pred heads                      [16][LD]
  float* W;   // wide scratch                              [16][LDW]
  float* E;   // small scratch                             [16][LDE]
  float* v0;  // per-row scalars: value                    [16]
  float* v1;  // reward                                    [16]
  float* v2;  // discount                                  [16]
  float* v3;  // spare                                     [16]
  __device__ static Arena carve(float* base) {
    Arena a;
    a.L = base;
    a.X = a.L + kRows * LD;
    a.T = a.X + kRows * LD;
    a.U = a.T + kRows * LD;
    a.W = a.U + kRows * LD;
    a.E = a.W + kRows * LDW;
    a.v0 = a.E + kRows * LDE;
    a.v1 = a.v0 + kRows;
    a.v2 = a.v1 + kRows;
    a.v3 = a.v2 + kRows;
    return a;
  }
};

// ResBlock (muzero_deterministic_madn.py:12-24): X <- relu(X + LN1(D1(relu(LN0(D0(X))))))
// pf: rb.d0 on entry, (Ln: Kn x Nn, NTN tiles) on exit.
template <int NTN>
__device__ __forceinline__ void resblock16(const AS4 muz_resblock& R, float* X, float* T, float* U, Pf& pf,
                                           const AS4 muz_dense* Ln, int Kn, int Nn) {
  dense16<2, 2>(R.d0, LAT, LAT, X, LD, T, LD, pf, &R.d1, LAT, LAT);
  __syncthreads();
  ln16<LAT, LN_RELU>(T, LD, T, LD, R.ln0);
  __syncthreads();
  dense16<2, NTN>(R.d1, LAT, LAT, T, LD, U, LD, pf, Ln, Kn, Nn);
  __syncthreads();
  ln16<LAT, LN_RESID_RELU>(U, LD, X, LD, R.ln1);
  __syncthreads();
}

// small dot head: out[row] = b + sum_k in[row][k] * w[k][col] for one column (32 lanes per row)
__device__ __forceinline__ float head_dot16(const float* in, int ld, int K, const float* w_, int ncol, int col,
                                            float b) {
  const int row = trow(), sub = tsub();
  const AS1 float* w = gp(w_);
  float s = 0.f;
  for (int k = sub; k < K; k += kRowLanes) s += in[row * ld + k] * w[k * ncol + col];
  return row_sum(s) + b;
}

// PredictionNetwork4 (muzero_deterministic_madn.py:549-583) on the latent in `lat` ([16][LD]).
// Leaves policy logits in a.U[:, 0:A] and tanh value in a.v0.  Clobbers X, T, U, W.
// pf: rb[0].d0 on entry, (Ln, NTN tiles) on exit.
template <int NTN>
__device__ __forceinline__ void pred16(const AS4 muz_pred_w& P, int A, const float* lat, const Arena& a, Pf& pf,
                                       const AS4 muz_dense* Ln, int Kn, int Nn) {
  ln16<LAT, LN_PLAIN>(lat, LD, a.X, LD, P.ln0);
  __syncthreads();
  resblock16<2>(P.rb[0], a.X, a.T, a.U, pf, &P.rb[1].d0, LAT, LAT);
  resblock16<3>(P.rb[1], a.X, a.T, a.U, pf, &P.d03, LAT, 384);
  dense16<3, 1>(P.d03, LAT, 384, a.X, LD, a.W, LDW, pf, &P.d1, LAT, 128);   // [policy Dense_0 | value Dense_3]
  __syncthreads();
  ln16<LAT, LN_RELU>(a.W, LDW, a.W, LDW, P.ln1);
  ln16<128, LN_RELU>(a.W + 256, LDW, a.W + 256, LDW, P.ln3);
  __syncthreads();
  dense16<1, 1>(P.d1, LAT, 128, a.W, LDW, a.T, LD, pf, &P.d4, 128, 64);     // policy Dense_1
  dense16<1, 1>(P.d4, 128, 64, a.W + 256, LDW, a.X, LD, pf, &P.d2, 128, A);  // value Dense_4 (X is free)
  __syncthreads();
  ln16<128, LN_RELU>(a.T, LD, a.T, LD, P.ln2);
  relu16(a.X, LD, 0, 64);
  __syncthreads();
  dense16<1, NTN>(P.d2, 128, A, a.T, LD, a.U, LD, pf, Ln, Kn, Nn);         // policy logits
  {
    const float v = head_dot16(a.X, LD, 64, P.d5.w, 1, 0, gp(P.d5.b)[0]);
    if (tsub() == 0) a.v0[trow()] = tanhf(v);
  }
  __syncthreads();
}

__device__ __forceinline__ float softmax3_support(float l0, float l1, float l2) {
  // sum(softmax(l) * [-1, 0, 1])  (recurrent_inference_fn 648-653)
  const float m = fmaxf(fmaxf(l0, l1), l2);
  const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = expf(l2 - m);
  const float z = e0 + e1 + e2;
  return (e0 / z) * -1.0f + (e1 / z) * 0.0f + (e2 / z) * 1.0f;
}

// DynamicsNetwork4 (muzero_deterministic_madn.py:391-457): latent a.L, action per row in act[16].
// Leaves the next latent in a.T, reward / discount expectations in a.v1 / a.v2.  Clobbers X, U, W, E.
// pf: d12 on entry, (Ln, NTN tiles) on exit.
template <int NTN>
__device__ __forceinline__ void dyn16(const AS4 muz_dyn_w& D, int A, const int* act, const Arena& a, Pf& pf,
                                      const AS4 muz_dense* Ln, int Kn, int Nn) {
  const int row = trow(), sub = tsub();
  const int ar = act[row];
  const bool oh = ar >= 0 && ar < A;   // jax.nn.one_hot: out-of-range -> zero row
  // action embedding: relu(one_hot @ W0 + b0) == relu(W0[a] + b0)
  const AS1 float* w0 = gp(D.d0.w);
  const AS1 float* b0 = gp(D.d0.b);
  for (int c = sub; c < 64; c += kRowLanes)
    a.E[row * LDE + c] = fmaxf((oh ? w0[ar * 64 + c] : 0.f) + b0[c], 0.f);
  ln16<LAT, LN_PLAIN>(a.L, LD, a.X, LD, D.ln0);
  __syncthreads();
  dense16<4, 2>(D.d12, 64, 512, a.E, LDE, a.W, LDW, pf, &D.d3, LAT, LAT);     // [scale | shift]
  __syncthreads();
  for (int c = sub; c < LAT; c += kRowLanes)
    a.X[row * LD + c] = a.X[row * LD + c] * (1.0f + a.W[row * LDW + c]) + a.W[row * LDW + 256 + c];
  __syncthreads();
  dense16<2, 2>(D.d3, LAT, LAT, a.X, LD, a.T, LD, pf, &D.d4, LAT, LAT);
  __syncthreads();
  ln16<LAT, LN_RELU>(a.T, LD, a.T, LD, D.ln1);
  __syncthreads();
  dense16<2, 2>(D.d4, LAT, LAT, a.T, LD, a.X, LD, pf, &D.rb[0].d0, LAT, LAT);
  __syncthreads();
  ln16<LAT, LN_RELU>(a.X, LD, a.X, LD, D.ln2);
  __syncthreads();
  resblock16<2>(D.rb[0], a.X, a.T, a.U, pf, &D.rb[1].d0, LAT, LAT);
  resblock16<2>(D.rb[1], a.X, a.T, a.U, pf, &D.d5, LAT, LAT);
  dense16<2, 1>(D.d5, LAT, LAT, a.X, LD, a.T, LD, pf, &D.d67, LAT, 128);
  __syncthreads();
  for (int c = sub; c < LAT; c += kRowLanes) a.T[row * LD + c] = a.L[row * LD + c] + a.T[row * LD + c];
  __syncthreads();
  minmax16(a.T, LD);
  __syncthreads();
  dense16<1, NTN>(D.d67, LAT, 128, a.T, LD, a.W, LDW, pf, Ln, Kn, Nn);   // [reward | discount] hidden
  __syncthreads();
  const AS1 float* w67 = gp(D.d67_onehot);
  for (int c = sub; c < 128; c += kRowLanes)
    a.W[row * LDW + c] = fmaxf(a.W[row * LDW + c] + (oh ? w67[ar * 128 + c] : 0.f), 0.f);
  __syncthreads();
  float rl[3], dl[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    rl[j] = head_dot16(a.W, LDW, 64, D.reward_head.w, 3, j, gp(D.reward_head.b)[j]);
    dl[j] = head_dot16(a.W + 64, LDW, 64, D.discount_head.w, 3, j, gp(D.discount_head.b)[j]);
  }
  if (sub == 0) {
    a.v1[row] = softmax3_support(rl[0], rl[1], rl[2]);
    a.v2[row] = softmax3_support(dl[0], dl[1], dl[2]);
  }
  __syncthreads();
}

}  // namespace muz
