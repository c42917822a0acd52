// DynamicsNetwork4's action-only FiLM sub-graph (muzero_deterministic_madn.py:404-418: one_hot(action) ->
// Dense_0 -> relu -> Dense_1 (scale) | Dense_2 (shift)) for all K unrolled steps of a learner batch as ONE launch
// each way.  As library GEMMs and torch ops it was ~11 launches forward (arange / compare / copy for the one-hot,
// three GEMMs, three bias adds, the relu, 1 + scale) and ~5 backward -- each ~5 us at the learner's 1280 rows.
//
// Forward (M rows): e = relu(b0 + W0[a]) -- the one-hot product is a row gather, exactly (every other term of
// one_hot @ W0 adds an exact zero) -- then scale = e W1 + b1, shift = e W2 + b2 (k-ordered fma chains), scale1 =
// 1 + scale for the trunk chain, and the float one-hot rows the reward / discount heads read.  Two workgroups per 16
// rows (128 output columns each).
// Backward: de = (dscale W1^T + dshift W2^T) * [e > 0]; W1 | W2 staged transposed through LDS.  The weight / bias gradients (e^T dscale, e^T dshift, one_hot^T de and the column sums) stay with the
// learner's grouped gradient launches.
#include "launch.hpp"

namespace muz {

constexpr int kFilmRows = 16, kFilmE = 64, kFilmN = 256, kFilmThreads = 256;

// grid (rows / 16, 2): blockIdx.y picks 128 of the 256 output columns; thread t owns column 128 y + (t & 127) of
// rows 8 (t >> 7) .. + 7 of the tile, for both products (e rows read as float4 over j from LDS)
// row r of the M = B x K learner rows (step-major: r = k B + b) reads action[b * lda + k] -- the batch's [B][lda]
// action rows directly, no transposed copy (B = M, lda = 1: a plain vector)
__global__ __launch_bounds__(kFilmThreads) void k_film_fwd(const int32_t* __restrict__ action, int B, int lda, int M,
                                                            int A,
                                                            const float* __restrict__ W0, const float* __restrict__ b0,
                                                            const float* __restrict__ W1, const float* __restrict__ b1,
                                                            const float* __restrict__ W2, const float* __restrict__ b2,
                                                            float* onehot, float* e_out, float* scale, float* shift,
                                                            float* scale1) {
  __shared__ __attribute__((aligned(16))) float es[kFilmRows][kFilmE];
  const int t = threadIdx.x, r0 = blockIdx.x * kFilmRows;
  const bool first = blockIdx.y == 0;
  for (int i = t; i < kFilmRows * kFilmE; i += kFilmThreads) {
    const int r = i / kFilmE, j = i % kFilmE, row = r0 + r;
    float v = 0.f;
    if (row < M) {
      const int a = action[(size_t)(row % B) * lda + row / B];
      v = (a >= 0 && a < A) ? W0[(size_t)a * kFilmE + j] + b0[j] : b0[j];
      v = fmaxf(v, 0.f);
      if (first) e_out[(size_t)row * kFilmE + j] = v;
    }
    es[r][j] = v;
  }
  if (onehot && first) {
    for (int i = t; i < kFilmRows * A; i += kFilmThreads) {
      const int r = i / A, c = i % A, row = r0 + r;
      if (row < M) onehot[(size_t)row * A + c] = action[(size_t)(row % B) * lda + row / B] == c ? 1.f : 0.f;
    }
  }
  __syncthreads();
  const int c = blockIdx.y * 128 + (t & 127), rb = 8 * (t >> 7);
  float s1[8], s2[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) s1[r] = s2[r] = 0.f;
#pragma unroll 4
  for (int j = 0; j < kFilmE; j += 4) {
    float w1[4], w2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      w1[q] = W1[(size_t)(j + q) * kFilmN + c];
      w2[q] = W2[(size_t)(j + q) * kFilmN + c];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float4 x = *reinterpret_cast<const float4*>(&es[rb + r][j]);
      const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s1[r] = fmaf(xv[q], w1[q], s1[r]);
        s2[r] = fmaf(xv[q], w2[q], s2[r]);
      }
    }
  }
  const float bb1 = b1[c], bb2 = b2[c];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int row = r0 + rb + r;
    if (row >= M) break;
    const float sc = s1[r] + bb1;
    scale[(size_t)row * kFilmN + c] = sc;
    shift[(size_t)row * kFilmN + c] = s2[r] + bb2;
    if (scale1) scale1[(size_t)row * kFilmN + c] = 1.0f + sc;
  }
}

// thread t: row t / 16 of the tile, outputs 4 (t % 16) .. + 3.  W1 then W2 are staged transposed into LDS whole
// (two passes of 256 columns: coalesced global reads, every load of a pass in flight together), wt[c][j] with row
// stride 68 (16-byte aligned float4 reads over j); d rows read as float4 over c.
constexpr int kFilmWtLd = kFilmE + 4;
__global__ __launch_bounds__(kFilmThreads) void k_film_bwd(const float* __restrict__ dscale,
                                                            const float* __restrict__ dshift,
                                                            const float* __restrict__ e, const float* __restrict__ W1,
                                                            const float* __restrict__ W2, int M, float* de) {
  extern __shared__ __attribute__((aligned(16))) float film_smem[];
  float (*ds)[2 * kFilmN + 4] = reinterpret_cast<float (*)[2 * kFilmN + 4]>(film_smem);
  float (*wt)[kFilmWtLd] = reinterpret_cast<float (*)[kFilmWtLd]>(film_smem + kFilmRows * (2 * kFilmN + 4));
  const int t = threadIdx.x, r0 = blockIdx.x * kFilmRows;
  for (int i = t; i < kFilmRows * 2 * kFilmN; i += kFilmThreads) {
    const int r = i / (2 * kFilmN), c = i % (2 * kFilmN), row = r0 + r;
    float v = 0.f;
    if (row < M) v = c < kFilmN ? dscale[(size_t)row * kFilmN + c] : dshift[(size_t)row * kFilmN + c - kFilmN];
    ds[r][c] = v;
  }
  const int r = t / 16, j0 = 4 * (t % 16);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (half) __syncthreads();   // pass 0's readers are done
    const float* W = half ? W2 : W1;
#pragma unroll 8
    for (int i = t; i < kFilmN * kFilmE; i += kFilmThreads) {
      const int j = i / kFilmN, c = i % kFilmN;   // coalesced along the weight row
      wt[c][j] = W[i];
    }
    __syncthreads();
#pragma unroll 4
    for (int c = 0; c < kFilmN; c += 4) {
      const float4 d4 = *reinterpret_cast<const float4*>(&ds[r][half * kFilmN + c]);
      const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 w4 = *reinterpret_cast<const float4*>(&wt[c + k][j0]);
        acc[0] = fmaf(dv[k], w4.x, acc[0]);
        acc[1] = fmaf(dv[k], w4.y, acc[1]);
        acc[2] = fmaf(dv[k], w4.z, acc[2]);
        acc[3] = fmaf(dv[k], w4.w, acc[3]);
      }
    }
  }
  const int row = r0 + r;
  if (row < M) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const size_t o = (size_t)row * kFilmE + j0 + q;
      de[o] = e[o] > 0.f ? acc[q] : 0.f;
    }
  }
}
constexpr size_t kFilmBwdLds = sizeof(float) * ((size_t)kFilmRows * (2 * kFilmN + 4) + (size_t)kFilmN * kFilmWtLd);

}  // namespace muz

using namespace muz;

extern "C" {

int muz_film_fwd_strided(const int32_t* action, int32_t B, int32_t K, int32_t lda, int32_t A, const float* W0,
                         const float* b0, const float* W1, const float* b1, const float* W2, const float* b2,
                         float* onehot, float* e, float* scale, float* shift, float* scale1, void* stream) {
  MUZ_HOST_CHECK(B >= 0 && K >= 0 && lda >= K && A > 0 && action && W0 && b0 && W1 && b1 && W2 && b2 && e && scale &&
                 shift);
  const int M = B * K;
  if (M == 0) return MUZ_OK;
  k_film_fwd<<<dim3((M + kFilmRows - 1) / kFilmRows, 2), kFilmThreads, 0, (hipStream_t)stream>>>(
      action, B, lda, M, A, W0, b0, W1, b1, W2, b2, onehot, e, scale, shift, scale1);
  return muz_last_launch_error();
}

int muz_film_fwd(const int32_t* action, int32_t M, int32_t A, const float* W0, const float* b0, const float* W1,
                 const float* b1, const float* W2, const float* b2, float* onehot, float* e, float* scale,
                 float* shift, float* scale1, void* stream) {
  MUZ_HOST_CHECK(M >= 0);
  return muz_film_fwd_strided(action, M, 1, 1, A, W0, b0, W1, b1, W2, b2, onehot, e, scale, shift, scale1, stream);
}

int muz_film_bwd(const float* dscale, const float* dshift, const float* e, const float* W1, const float* W2,
                 int32_t M, float* de, void* stream) {
  MUZ_HOST_CHECK(M >= 0 && dscale && dshift && e && W1 && W2 && de);
  if (M == 0) return MUZ_OK;
  static bool attr = false;
  if (!attr) {   // > 64 KB of dynamic LDS
    MUZ_HIP_RET(hipFuncSetAttribute((const void*)k_film_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFilmBwdLds));
    attr = true;
  }
  k_film_bwd<<<(M + kFilmRows - 1) / kFilmRows, kFilmThreads, kFilmBwdLds, (hipStream_t)stream>>>(dscale, dshift, e, W1,
                                                                                                  W2, M, de);
  return muz_last_launch_error();
}

}  // extern "C"
