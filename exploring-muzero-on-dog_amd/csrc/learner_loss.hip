// The learner's losses and their gradients w.r.t. the network outputs in ONE launch: value MSE, policy
// cross-entropy and the class-balanced cross-entropies of loss_fn (train_with_reward.py:24-141: reward,
// discount) / loss_fn_stochastic (train_stochastic.py:34-180: chance, discount, reward), all K + 1 unroll
// steps at once.  As torch ops the same arithmetic was ~120 launches of ~4.5 us (forward + autograd) per step.
//
// One workgroup of 16 waves.  A wave takes a 64-row chunk of one unroll step (lane = sample), so every
// per-step sum is a wave reduction plus a fixed-order sum over the step's chunks (deterministic):
//   phase 1: per-step mask / rare counts of the CE terms -> the balanced-loss normalisers n_rare, n_common;
//   phase 2: per row, the losses and their gradients (softmax - target, scaled by the row's weight);
//   phase 3: per-step sums -> parts and total.
#include "launch.hpp"

namespace muz {

constexpr int kLossThreads = 1024;
constexpr int kLossWaves = kLossThreads / 64;
constexpr int kLossMaxChunks = 1024;
constexpr int kLossMaxK = 64;

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

constexpr int kLossMaxA = 32;     // policy width
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

__global__ __launch_bounds__(kLossThreads) void k_loss_heads(muz_loss_args g) {
  __shared__ float part[kLossMaxChunks][5];
  __shared__ float cnt[kLossMaxK][4];
  __shared__ float sk[kLossMaxK + 1][5];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, tid = threadIdx.x;
  const int K = g.K, B = g.B, nch = (B + 63) / 64, nt = g.nterms;
  // phase 1: S(m), S(m r_j) per (step, chunk) of the first K steps
  for (int i = wv; i < K * nch; i += kLossWaves) {
    const int k = i / nch, b = (i % nch) * 64 + lane;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (b < B) {
      const float m = g.masks[(size_t)b * g.T + k];
      v[0] = m;
#pragma unroll
      for (int j = 0; j < 3; ++j)      // (static term indices: the term fields stay in scalar registers)
        if (j < nt) v[1 + j] = loss_rare(g.term[j], b, k) ? m : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float s = wave_sum_f(v[q]);
      if (lane == 0) part[i][q] = s;
    }
  }
  __syncthreads();
  if (tid < K * 4) {
    const int k = tid / 4, q = tid % 4;
    float s = 0.f;
    for (int c = 0; c < nch; ++c) s += part[k * nch + c][q];
    cnt[k][q] = s;
  }
  __syncthreads();
  // phase 2: per row, losses (weighted) and gradients
  const float invB = 1.0f / (float)B;
  for (int i = wv; i < (K + 1) * nch; i += kLossWaves) {
    const int k = i / nch, b = (i % nch) * 64 + lane;
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (b < B) {
      const size_t row = (size_t)k * B + b;
      const float m = g.masks[(size_t)b * g.T + k];
      const float d = g.value[row] - g.target_values[(size_t)b * g.T + k];
      v[0] = m * d * d;
      g.dvalue[row] = g.scale_value * invB * m * 2.0f * d;
      v[1] = m * loss_ce_row<kLossMaxA>(g.logits + row * g.A, g.dlogits + row * g.A, g.A, -1,
                             g.policies + ((size_t)b * g.T + k) * g.A, g.scale_policy * invB * m);
      if (k < K) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (j >= nt) break;
          const muz_loss_term& t = g.term[j];
          const float nr = fmaxf(cnt[k][1 + j], 1.f);
          const float nc = fmaxf(cnt[k][0] - (g.norm ? nr : cnt[k][1 + j]), 1.f);
          const bool r = loss_rare(t, b, k);
          const float w = m * (r ? t.w_rare / nr : t.w_common / nc);
          const int lab = t.labels ? t.labels[(size_t)b * t.ld + k] : -1;
          const float* tg = t.labels ? nullptr : t.probs + ((size_t)b * t.ld + k) * t.ncls;
          v[2 + j] = w * loss_ce_row<kLossMaxCls>(t.logits + row * t.ncls, t.dlogits + row * t.ncls, t.ncls, lab, tg, t.scale * w);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const float s = wave_sum_f(v[q]);
      if (lane == 0) part[i][q] = s;
    }
  }
  __syncthreads();
  // phase 3: per-step sums, then the parts in step order
  if (tid < (K + 1) * 5) {
    const int k = tid / 5, q = tid % 5;
    float s = 0.f;
    for (int c = 0; c < nch; ++c) s += part[k * nch + c][q];
    sk[k][q] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float lv = 0.f, lp = 0.f, lt[3] = {0.f, 0.f, 0.f}, total = 0.f;
    for (int k = 0; k <= K; ++k) {
      const float v = sk[k][0] * invB, p = sk[k][1] * invB;
      lv += v;
      lp += p;
      total += g.scale_value * v + g.scale_policy * p;
    }
    for (int j = 0; j < nt; ++j) {
      for (int k = 0; k < K; ++k) lt[j] += sk[k][2 + j];
      total += g.term[j].scale * lt[j];
    }
    float* o = g.parts;
    *g.total = total;
    o[0] = total, o[1] = lv, o[2] = lp, o[3] = lt[0], o[4] = lt[1], o[5] = lt[2];
  }
}

}  // namespace muz

using namespace muz;

extern "C" int muz_loss_heads(const muz_loss_args* args, void* stream) {
  MUZ_HOST_CHECK(args);
  const muz_loss_args& a = *args;
  MUZ_HOST_CHECK(a.K >= 0 && a.B > 0 && a.A > 0 && a.T >= a.K + 1 && a.nterms >= 0 && a.nterms <= 3);
  MUZ_HOST_CHECK(a.masks && a.target_values && a.policies && a.value && a.logits && a.dvalue && a.dlogits && a.parts && a.total);
  if (a.K > kLossMaxK || (a.K + 1) * ((a.B + 63) / 64) > kLossMaxChunks || a.A > kLossMaxA) return MUZ_E_UNSUPPORTED;
  for (int j = 0; j < a.nterms; ++j) {
    const muz_loss_term& t = a.term[j];
    if (t.ncls > kLossMaxCls) return MUZ_E_UNSUPPORTED;
    MUZ_HOST_CHECK(t.logits && t.dlogits && t.ncls > 0 && t.ld >= a.K && (t.labels != nullptr) != (t.probs != nullptr));
  }
  k_loss_heads<<<1, kLossThreads, 0, (hipStream_t)stream>>>(a);
  return muz_last_launch_error();
}
