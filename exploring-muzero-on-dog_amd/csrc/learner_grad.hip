// Grouped weight-gradient GEMMs and column sums of one learner backward (train_with_reward.py:148-164 /
// train_stochastic.py:183-199 through learner.py).
//
// A batch-128, unroll-10 train step has ~45 weight matrices; their gradients dW = X^T dZ (reduction over the
// layer's rows: 128 for the root, 1280-1408 for the unrolled trunk / prediction, 7168 for the convolutions) and
// the bias / LayerNorm column sums were ~130 separate library launches of a few microseconds each.  The learner
// now records every (X, dZ, dW) and every column sum during backward and runs them here in three launches:
//
// k_wgrad_grouped: one workgroup (8 waves) per (64 x 64 output tile, 2048-row segment) of any problem; wave w
//   computes the 32 x 32 quadrant w % 4 over half of the segment's rows (half w / 4 takes rows 8 s + 4 h .. + 3
//   of every 8-row step s) with 2 x 2 v_mfma_f32_16x16x4_f32 accumulators (A = X^T: lane l reads X[m + l/16][k + l%16], B = dZ: lane l reads
//   dZ[m + l/16][n + l%16], so each operand load is a 64-byte row segment).  Loads are issued 8 steps ahead of
//   their MFMAs (one memory latency per 64 rows instead of per 8); the 64 x 64 tile halves the L2 re-reads of
//   X and dZ against 32 x 32 tiles.  The two halves add their partials through LDS in a fixed order; a problem with
//   one segment writes dW directly, longer ones write per-segment partials to scratch, which k_seg_sum adds in
//   segment order (deterministic: graph-captured and eager steps stay bit-identical).
// k_seg_sum: one thread per output element, p_0 + p_1 + ... in segment order (the sum k_colsum_grouped's kind 1
//   formed for these partials, bit for bit, with one thread per element instead of a 1024-thread workgroup per 64
//   columns: the round-5 512-row segments measured wgrad 107 -> 69 us but the partial sums 16 -> 118 us that way,
//   profiles/r5q_wgrad_seg.log).
// k_colsum_grouped: one workgroup per (problem, output, 64-column chunk); kind 0 reduces muz_ln_bwd_rows'
//   per-block partials [nblk][3][N] into dgamma / dbeta / dbias (k_ln_colsum's order), kind 1 sums the rows of
//   a matrix (a dZ into a bias gradient, or a weight gradient's segment partials).
#include "launch.hpp"

namespace muz {

typedef float f32x4_g __attribute__((ext_vector_type(4)));

constexpr int kWgMax = 48;    // problems per launch (kernel-argument table)
#ifndef MUZ_WGRAD_SEG
#define MUZ_WGRAD_SEG 256   // det / DOG learner step, profiles/r6p_steps.log: 2048 1.543 / 1.782 ms, 512 1.522 / 1.731, 256 1.512 / 1.729
#endif
constexpr int kWgSeg = MUZ_WGRAD_SEG;  // rows per workgroup (a multiple of 64)
static_assert(kWgSeg % 64 == 0, "segments are whole 64-row steps");

__host__ __device__ constexpr int wgrad_segs(int M) { return M <= kWgSeg ? 1 : (M + kWgSeg - 1) / kWgSeg; }

struct WgradTable {
  const float* x[kWgMax];
  const float* dz[kWgMax];
  float* out[kWgMax];   // dW, or the [segs][K][N] partials
  int M[kWgMax], K[kWgMax], N[kWgMax], ldx[kWgMax], lddz[kWgMax], tiles_n[kWgMax], segs[kWgMax], wg0[kWgMax + 1];
  int count;
};

__global__ __launch_bounds__(512) void k_wgrad_grouped(WgradTable t) {
  __shared__ f32x4_g red[4][2][2][64];
  const int wg = blockIdx.x;
  int p = 0;
  while (p + 1 < t.count && t.wg0[p + 1] <= wg) ++p;
  const int local = wg - t.wg0[p], segs = t.segs[p];
  const int seg = local % segs, tile = local / segs;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int qd = wv & 3, h = wv >> 2;     // 32 x 32 quadrant of the 64 x 64 tile, row half
  const int k0 = (tile / t.tiles_n[p]) * 64 + 32 * (qd >> 1), n0 = (tile % t.tiles_n[p]) * 64 + 32 * (qd & 1);
  const int K = t.K[p], N = t.N[p], ldx = t.ldx[p], lddz = t.lddz[p];
  const int mbeg = seg * kWgSeg, mend = min(t.M[p], mbeg + kWgSeg);
  const float* __restrict__ X = t.x[p];
  const float* __restrict__ DZ = t.dz[p];
  const int li = lane & 15, lq = lane >> 4;
  const bool ka = k0 + li < K, kb = k0 + 16 + li < K, na = n0 + li < N, nb = n0 + 16 + li < N;
  f32x4_g acc[2][2] = {};
  // (loop bounds are wave-uniform -- MFMAs run with every lane active); half h takes rows 8 s + 4 h .. + 3
  int m = mbeg;
  for (; m + 64 <= mend; m += 64) {
    float a0[8], a1[8], b0[8], b1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = m + 8 * j + 4 * h + lq;
      const float* xr = X + (size_t)r * ldx + k0 + li;
      const float* dr = DZ + (size_t)r * lddz + n0 + li;
      a0[j] = ka ? xr[0] : 0.f;
      a1[j] = kb ? xr[16] : 0.f;
      b0[j] = na ? dr[0] : 0.f;
      b1[j] = nb ? dr[16] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], b0[j], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], b1[j], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], b0[j], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], b1[j], acc[1][1], 0, 0, 0);
    }
  }
  for (; m < mend; m += 8) {   // tail: rows past the segment read as zero
    const int r = m + 4 * h + lq;
    const bool mv = r < mend;
    const float* xr = X + (size_t)r * ldx + k0 + li;
    const float* dr = DZ + (size_t)r * lddz + n0 + li;
    const float a0 = (mv && ka) ? xr[0] : 0.f, a1 = (mv && kb) ? xr[16] : 0.f;
    const float b0 = (mv && na) ? dr[0] : 0.f, b1 = (mv && nb) ? dr[16] : 0.f;
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
  }
  if (h == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[qd][i][j][lane] = acc[i][j];
  }
  __syncthreads();
  if (h != 0) return;
  float* o = t.out[p] + (size_t)seg * K * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const f32x4_g s = acc[i][j] + red[qd][i][j][lane];
      const int n = n0 + 16 * j + li;
      if (n >= N) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int k = k0 + 16 * i + 4 * lq + v;
        if (k < K) o[(size_t)k * N + n] = s[v];
      }
    }
}

struct SegSumTable {
  const float* part[kWgMax];
  float* out[kWgMax];
  int segs[kWgMax], kn[kWgMax], wg0[kWgMax + 1];
  int count;
};

__global__ __launch_bounds__(256) void k_seg_sum(SegSumTable t) {
  const int wg = blockIdx.x;
  int p = 0;
  while (p + 1 < t.count && t.wg0[p + 1] <= wg) ++p;
  const int kn = t.kn[p], e = (wg - t.wg0[p]) * 256 + threadIdx.x;
  if (e >= kn) return;
  const float* __restrict__ src = t.part[p] + e;
  const int segs = t.segs[p];
  float acc = 0.f;
  // 8 partials in flight, then added in segment order (a load-add chain would wait one memory latency per segment)
  for (int q0 = 0; q0 < segs; q0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = q0 + u < segs ? src[(size_t)(q0 + u) * kn] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (q0 + u < segs) acc += v[u];
  }
  t.out[p][e] = acc;
}

struct ColsumTable {
  const float* src[kWgMax];
  float* out[kWgMax][3];
  int kind[kWgMax], rows[kWgMax], N[kWgMax], ld[kWgMax], wg0[kWgMax + 1];
  int count;
};

// workgroup -> (problem, output q, 64-column chunk); thread (j, c) sums rows j, j + 16, ... with 8 independent
// accumulators (8 loads in flight), then the 16 partial sums are added in a fixed order
constexpr int kCsGroups = 16;
__global__ __launch_bounds__(64 * kCsGroups) void k_colsum_grouped(ColsumTable t) {
  __shared__ float red[kCsGroups][64];
  const int wg = blockIdx.x;
  int p = 0;
  while (p + 1 < t.count && t.wg0[p + 1] <= wg) ++p;
  const int local = wg - t.wg0[p];
  const int N = t.N[p], chunks = (N + 63) / 64, nrows = t.rows[p];
  const int q = local / chunks, c = (local % chunks) * 64 + (threadIdx.x & 63), j = threadIdx.x >> 6;
  const bool ln = t.kind[p] == 0;
  const float* __restrict__ src = t.src[p];
  // element (row b, column c) of this output's matrix
  const size_t rstride = ln ? (size_t)3 * N : (size_t)t.ld[p];
  const size_t base = ln ? (size_t)q * N + c : (size_t)c;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    int b = j;
    for (; b + 7 * kCsGroups < nrows; b += 8 * kCsGroups)
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += src[(size_t)(b + kCsGroups * u) * rstride + base];
    for (; b < nrows; b += kCsGroups) acc[0] += src[(size_t)b * rstride + base];
  }
  red[j][threadIdx.x & 63] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (j == 0 && c < N) {
    const int tt = threadIdx.x & 63;
    float s = red[0][tt];
#pragma unroll
    for (int g = 1; g < kCsGroups; ++g) s += red[g][tt];
    float* o = t.out[p][q];
    if (o) o[c] = s;
  }
}

}  // namespace muz

using namespace muz;

extern "C" {

int32_t muz_wgrad_segment_rows(void) { return kWgSeg; }

int64_t muz_wgrad_scratch_floats(const muz_wgrad_problem* probs, int32_t count) {
  if (count < 0 || (count > 0 && !probs)) return -1;
  int64_t n = 0;
  for (int i = 0; i < count; ++i) {
    const int segs = wgrad_segs(probs[i].M);
    if (segs > 1) n += (int64_t)segs * probs[i].K * probs[i].N;
  }
  return n;
}

int muz_wgrad_grouped(const muz_wgrad_problem* probs, int32_t count, float* scratch, int64_t scratch_floats,
                      void* stream) {
  MUZ_HOST_CHECK(count >= 0 && (count == 0 || probs));
  const int64_t need = muz_wgrad_scratch_floats(probs, count);
  MUZ_HOST_CHECK(need >= 0 && scratch_floats >= need && (need == 0 || scratch));
  // the segment partials are summed by k_seg_sum, one launch per chunk of problems
  int64_t off = 0;
  for (int s = 0; s < count; s += kWgMax) {
    WgradTable t{};
    SegSumTable r{};
    t.count = 0;
    int wgs = 0, nred = 0, rwgs = 0;
    for (int i = s; i < count && t.count < kWgMax; ++i) {
      const muz_wgrad_problem& q = probs[i];
      MUZ_HOST_CHECK((q.M == 0 || (q.x && q.dz)) && q.out && q.M >= 0 && q.K > 0 && q.N > 0 && q.ldx >= q.K &&
                     q.lddz >= q.N);
      const int c = t.count++;
      const int segs = wgrad_segs(q.M);
      t.x[c] = q.x, t.dz[c] = q.dz;
      t.M[c] = q.M, t.K[c] = q.K, t.N[c] = q.N, t.ldx[c] = q.ldx, t.lddz[c] = q.lddz;
      t.tiles_n[c] = (q.N + 63) / 64;
      t.segs[c] = segs;
      t.wg0[c] = wgs;
      wgs += ((q.K + 63) / 64) * t.tiles_n[c] * segs;
      if (segs == 1) {
        t.out[c] = q.out;
      } else {
        float* part = scratch + off;
        off += (int64_t)segs * q.K * q.N;
        t.out[c] = part;
        r.part[nred] = part, r.out[nred] = q.out, r.segs[nred] = segs, r.kn[nred] = q.K * q.N;
        r.wg0[nred++] = rwgs;
        rwgs += (q.K * q.N + 255) / 256;
      }
    }
    t.wg0[t.count] = wgs;
    if (wgs == 0) continue;
    k_wgrad_grouped<<<wgs, 512, 0, (hipStream_t)stream>>>(t);
    int rc = muz_last_launch_error();
    if (rc) return rc;
    if (nred) {
      r.count = nred;
      r.wg0[nred] = rwgs;
      k_seg_sum<<<rwgs, 256, 0, (hipStream_t)stream>>>(r);
      rc = muz_last_launch_error();
      if (rc) return rc;
    }
  }
  return MUZ_OK;
}

int muz_colsum_grouped(const muz_colsum_problem* probs, int32_t count, void* stream) {
  MUZ_HOST_CHECK(count >= 0 && (count == 0 || probs));
  for (int s = 0; s < count; s += kWgMax) {
    ColsumTable t{};
    t.count = 0;
    int wgs = 0;
    for (int i = s; i < count && t.count < kWgMax; ++i) {
      const muz_colsum_problem& q = probs[i];
      MUZ_HOST_CHECK((q.rows == 0 || q.src) && q.N > 0 && q.rows >= 0 && (q.kind == 0 || (q.kind == 1 && q.ld >= q.N && q.out0)));
      const int c = t.count++;
      t.src[c] = q.src;
      t.out[c][0] = q.out0, t.out[c][1] = q.out1, t.out[c][2] = q.out2;
      t.kind[c] = q.kind, t.rows[c] = q.rows, t.N[c] = q.N, t.ld[c] = q.ld;
      t.wg0[c] = wgs;
      wgs += (q.kind == 0 ? 3 : 1) * ((q.N + 63) / 64);
    }
    t.wg0[t.count] = wgs;
    if (wgs == 0) continue;
    k_colsum_grouped<<<wgs, 64 * kCsGroups, 0, (hipStream_t)stream>>>(t);
    const int rc = muz_last_launch_error();
    if (rc) return rc;
  }
  return MUZ_OK;
}

}  // extern "C"
