// The learner's losses and their gradients w.r.t. the network outputs in ONE launch: value MSE, policy
// cross-entropy and the class-balanced cross-entropies of loss_fn (train_with_reward.py:24-141: reward,
// discount) / loss_fn_stochastic (train_stochastic.py:34-180: chance, discount, reward), all K + 1 unroll
// steps at once.  As torch ops the same arithmetic was ~120 launches of ~4.5 us (forward + autograd) per step.
//
// One workgroup per unroll step k (256 threads, thread = sample row), so the per-step sums are block
// reductions in a fixed order (deterministic):
//   phase 1: step k's mask / rare counts of the CE terms -> the balanced-loss normalisers n_rare, n_common;
//   phase 2: per row, the losses and their gradients (softmax - target, scaled by the row's weight), with every
//            load of a row issued before its arithmetic;
//   phase 3: the step's sums -> partials[k]; the last workgroup to finish (a ticket counter, reset by that
//            workgroup for the next launch / graph replay) adds the K + 1 partials in step order into the parts.
// (Round 3's first version ran all steps in one workgroup: 70 us of serial memory latency.)
#include "launch.hpp"

namespace muz {

constexpr int kLossThreads = 256;
constexpr int kLossWaves = kLossThreads / 64;
constexpr int kLossMaxK = 64;

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

constexpr int kLossMaxA = 32;     // policy width of the per-thread rows (det 24, classic 4)
constexpr int kLossMaxWideA = 1024;   // wider policies (DOG 806): one wave per row
constexpr int kLossMaxCls = 8;    // classes of a CE term

// rare predicate of term t for (sample b, step k)
__device__ __forceinline__ bool loss_rare(const muz_loss_term& t, int b, int k) {
  if (t.labels) {
    const int lab = t.labels[(size_t)b * t.ld + k];
    return t.rare_not_one ? lab != 1 : lab == 1;
  }
  const float* p = t.probs + ((size_t)b * t.ld + k) * t.ncls;
  float v[kLossMaxCls];
#pragma unroll
  for (int a = 0; a < kLossMaxCls; ++a) v[a] = a < t.ncls ? p[a] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < kLossMaxCls; ++a) {
    const float d = v[a] - (1.0f / 6.0f);
    s += a < t.ncls ? d * d : 0.f;
  }
  return s > 1e-6f;
}

// cross-entropy of one row against a label / distribution; writes coef * (softmax * sum(target) - target).
// The row and its target are loaded into registers first (all loads in flight at once: the kernel is a
// single workgroup, so it is bound by memory latency, not by arithmetic).
template <int NMAX>
__device__ __forceinline__ float loss_ce_row(const float* __restrict__ l, float* __restrict__ dl, int n,
                                             int label, const float* __restrict__ tgt, float coef) {
  float x[NMAX], t[NMAX];
#pragma unroll
  for (int a = 0; a < NMAX; ++a) {
    x[a] = a < n ? l[a] : -INFINITY;
    t[a] = a < n ? (tgt ? tgt[a] : (a == label ? 1.f : 0.f)) : 0.f;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int a = 0; a < NMAX; ++a) mx = fmaxf(mx, x[a]);
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < NMAX; ++a) s += a < n ? expf(x[a] - mx) : 0.f;
  const float lse = mx + logf(s);
  float ce = 0.f, st = 0.f;
#pragma unroll
  for (int a = 0; a < NMAX; ++a) {
    if (a < n) {
      ce -= t[a] * (x[a] - lse);
      st += t[a];
    }
  }
#pragma unroll
  for (int a = 0; a < NMAX; ++a)
    if (a < n) dl[a] = coef * (expf(x[a] - lse) * st - t[a]);
  return ce;
}

// loss_ce_row for a row of n <= kLossMaxWideA logits held by one wave (lane a, a + 64, ...); returns the row's
// cross-entropy in every lane (wave sums in a fixed butterfly order)
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ float loss_ce_row_wide(const float* __restrict__ l, float* __restrict__ dl, int n,
                                                  const float* __restrict__ tgt, float coef, int lane) {
  constexpr int J = kLossMaxWideA / 64;
  float x[J], t[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int a = lane + 64 * j;
    x[j] = a < n ? l[a] : -INFINITY;
    t[j] = a < n ? tgt[a] : 0.f;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < J; ++j) mx = fmaxf(mx, x[j]);
  mx = wave_max_f(mx);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) s += lane + 64 * j < n ? expf(x[j] - mx) : 0.f;
  s = wave_sum_f(s);
  const float lse = mx + logf(s);
  float ce = 0.f, st = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (lane + 64 * j < n) {
      ce -= t[j] * (x[j] - lse);
      st += t[j];
    }
  }
  ce = wave_sum_f(ce);
  st = wave_sum_f(st);
#pragma unroll
  for (int j = 0; j < J; ++j)
    if (lane + 64 * j < n) dl[lane + 64 * j] = coef * (expf(x[j] - lse) * st - t[j]);
  return ce;
}

// a load that sees other workgroups' stores after their fence (relaxed atomic: not served from a stale L1 line)
__device__ __forceinline__ float ld_coherent(const float* p) {
  return __builtin_bit_cast(float, __atomic_load_n(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED));
}

// fixed-order block sum of NV values (every thread passes its own; the result is valid in every thread)
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float (*red)[NV]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const float s = wave_sum_f(v[q]);
    if (lane == 0) red[wv][q] = s;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    float s = red[0][q];
#pragma unroll
    for (int w = 1; w < kLossWaves; ++w) s += red[w][q];
    v[q] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kLossThreads) void k_loss_heads(muz_loss_args g) {
  __shared__ float red4[kLossWaves][4];
  __shared__ float red5[kLossWaves][5];
  __shared__ int last;
  const int k = blockIdx.x, tid = threadIdx.x;
  const int K = g.K, B = g.B, nt = g.nterms;
  // phase 1: S(m), S(m r_j) of step k (the CE terms cover the first K steps)
  float cnt[4] = {0.f, 0.f, 0.f, 0.f};
  if (k < K) {
    for (int b = tid; b < B; b += kLossThreads) {
      const float m = g.masks[(size_t)b * g.T + k];
      cnt[0] += m;
#pragma unroll
      for (int j = 0; j < 3; ++j)      // (static term indices: the term fields stay in scalar registers)
        if (j < nt) cnt[1 + j] += loss_rare(g.term[j], b, k) ? m : 0.f;
    }
  }
  block_sum<4>(cnt, red4);
  // phase 2: per row, losses (weighted) and gradients
  const float invB = 1.0f / (float)B;
  float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b = tid; b < B; b += kLossThreads) {
    const size_t row = (size_t)k * B + b;
    const float m = g.masks[(size_t)b * g.T + k];
    const float val = g.value[row], tv = g.target_values[(size_t)b * g.T + k];
    int lab[3] = {-1, -1, -1};
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < nt && k < K && g.term[j].labels) lab[j] = g.term[j].labels[(size_t)b * g.term[j].ld + k];
    const float d = val - tv;
    v[0] += m * d * d;
    g.dvalue[row] = g.scale_value * invB * m * 2.0f * d;
    if (g.A <= kLossMaxA)
      v[1] += m * loss_ce_row<kLossMaxA>(g.logits + row * g.A, g.dlogits + row * g.A, g.A, -1,
                                        g.policies + ((size_t)b * g.T + k) * g.A, g.scale_policy * invB * m);
    if (k < K) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (j >= nt) break;
        const muz_loss_term& t = g.term[j];
        const float nr = fmaxf(cnt[1 + j], 1.f);
        const float nc = fmaxf(cnt[0] - (g.norm ? nr : cnt[1 + j]), 1.f);
        const bool r = t.labels ? (t.rare_not_one ? lab[j] != 1 : lab[j] == 1) : loss_rare(t, b, k);
        const float w = m * (r ? t.w_rare / nr : t.w_common / nc);
        const float* tg = t.labels ? nullptr : t.probs + ((size_t)b * t.ld + k) * t.ncls;
        v[2 + j] += w * loss_ce_row<kLossMaxCls>(t.logits + row * t.ncls, t.dlogits + row * t.ncls, t.ncls, lab[j],
                                                 tg, t.scale * w);
      }
    }
  }
  if (g.A > kLossMaxA) {   // the policy cross-entropy of wide rows: one wave per row, the wave's rows summed in order
    const int lane = tid & 63, wv = tid >> 6;
    float acc = 0.f;
    for (int b = wv; b < B; b += kLossWaves) {
      const size_t row = (size_t)k * B + b;
      const float m = g.masks[(size_t)b * g.T + k];
      const float ce = m * loss_ce_row_wide(g.logits + row * g.A, g.dlogits + row * g.A, g.A,
                                            g.policies + ((size_t)b * g.T + k) * g.A, g.scale_policy * invB * m, lane);
      acc += ce;
    }
    v[1] = lane == 0 ? acc : 0.f;
  }
  block_sum<5>(v, red5);
  // phase 3: this step's sums; the last workgroup adds all steps in order
  if (tid == 0) {
#pragma unroll
    for (int q = 0; q < 5; ++q) g.partials[5 * k + q] = v[q];
    __threadfence();
    last = atomicAdd(g.ticket, 1) == K;
  }
  __syncthreads();
  if (!last || tid != 0) return;
  __threadfence();
  float lv = 0.f, lp = 0.f, lt[3] = {0.f, 0.f, 0.f}, total = 0.f;
  for (int kk = 0; kk <= K; ++kk) {
    const float* pk = g.partials + 5 * kk;
    const float a = ld_coherent(pk) * invB, p = ld_coherent(pk + 1) * invB;
    lv += a;
    lp += p;
    total += g.scale_value * a + g.scale_policy * p;
    if (kk < K) {
#pragma unroll
      for (int j = 0; j < 3; ++j) lt[j] += ld_coherent(pk + 2 + j);
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (j < nt) total += g.term[j].scale * lt[j];
  float* o = g.parts;
  *g.total = total;
  o[0] = total, o[1] = lv, o[2] = lp, o[3] = lt[0], o[4] = lt[1], o[5] = lt[2];
  *g.ticket = 0;     // ready for the next launch (or graph replay)
}

}  // namespace muz

using namespace muz;

extern "C" int muz_loss_heads(const muz_loss_args* args, void* stream) {
  MUZ_HOST_CHECK(args);
  const muz_loss_args& a = *args;
  MUZ_HOST_CHECK(a.K >= 0 && a.B > 0 && a.A > 0 && a.T >= a.K + 1 && a.nterms >= 0 && a.nterms <= 3);
  MUZ_HOST_CHECK(a.masks && a.target_values && a.policies && a.value && a.logits && a.dvalue && a.dlogits && a.parts && a.total);
  if (a.K > kLossMaxK || a.A > kLossMaxWideA) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(a.partials && a.ticket);
  for (int j = 0; j < a.nterms; ++j) {
    const muz_loss_term& t = a.term[j];
    if (t.ncls > kLossMaxCls) return MUZ_E_UNSUPPORTED;
    MUZ_HOST_CHECK(t.logits && t.dlogits && t.ncls > 0 && t.ld >= a.K && (t.labels != nullptr) != (t.probs != nullptr));
  }
  k_loss_heads<<<a.K + 1, kLossThreads, 0, (hipStream_t)stream>>>(a);
  return muz_last_launch_error();
}
