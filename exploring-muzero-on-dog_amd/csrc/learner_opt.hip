// The learner's optimizer step over every parameter tensor in a few launches:
// optax.chain(clip_by_global_norm(max_norm), adamw(piecewise-constant lr, b1, b2, eps, weight_decay))
// (train_with_reward.py:361-372, train_stochastic.py:415-426).  The torch._foreach_* form of the same
// update (learner.AdamW on the CPU) was ~40 multi-tensor launches plus a dozen scalar kernels per step,
// ~0.6 ms of a 4.6 ms graph-captured det step; this is two passes over the parameters (HBM-bound:
// 4 B of gradient read by the norm pass, 24 B read+written per element by the update pass).
//
// Pass 1 (k_adam_sqnorm): one workgroup per 4096-element chunk of a tensor writes the chunk's sum of
//   squared gradients to partial[chunk]; workgroup 0 also latches the step counter (stepbuf = count,
//   count += 1) so pass 2 never reads a value it races with.
// Pass 2 (k_adam_update): every workgroup reduces ALL partials in the same fixed order (same global norm
//   in every workgroup, bit-identical run to run), then updates its chunk:
//     g = grad / denom * mult  (denom, mult = 1, 1 if ||g|| < max_norm else ||g||, max_norm)
//     mu = b1 mu + (1 - b1) g;  nu = b2 nu + (1 - b2) g^2
//     p -= lr * (mu / c1 / (sqrt(nu / c2) + eps) + wd p),  c_i = 1 - b_i^(step), lr = lr(step - 1)
//   with the scalars in float64 on the device as learner.AdamW computes them.
// muz_adamw_step: the tensors travel in the kernel arguments, kAdamMaxTensors per launch (nothing to upload, so
// the step is capturable in a HIP graph as it stands).  muz_adamw_step_table: one launch per pass over a
// caller-owned device table (muz_adamw_table_write, eager and blocking); the caller keeps that table unchanged
// for as long as a graph that captured the step may replay (learner.AdamW keeps one table per pointer set).
#include "launch.hpp"

#include <math.h>

#include <vector>

namespace muz {

constexpr int kAdamThreads = 256;
constexpr int kAdamPerThread = 16;
constexpr int kAdamChunk = kAdamThreads * kAdamPerThread;
constexpr int kAdamMaxTensors = 80;   // 80: the det learner's 156 tensors in 2 launches per pass (kernargs ~3.6 KB)
constexpr int kAdamMaxBounds = 4;

struct AdamTable {
  int n;                              // tensors in this launch
  int chunk0;                         // global index of the launch's first chunk
  int cstart[kAdamMaxTensors + 1];    // chunk prefix within the launch
  int64_t numel[kAdamMaxTensors];
  float* p[kAdamMaxTensors];
  const float* g[kAdamMaxTensors];    // nullptr: a parameter without gradient (treated as zero)
  float* m[kAdamMaxTensors];
  float* v[kAdamMaxTensors];
};

struct AdamHyper {
  double b1, b2, lr0, spi;
  double bound[kAdamMaxBounds], factor[kAdamMaxBounds];
  float max_norm, eps, wd;
  int nb, nchunks;
};

__device__ __forceinline__ float adam_block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const float s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__device__ __forceinline__ int adam_tensor_of(const AdamTable& t, int b) {
  int ti = 0;
  while (ti + 1 < t.n && t.cstart[ti + 1] <= b) ++ti;
  return ti;
}

__global__ __launch_bounds__(kAdamThreads) void k_adam_sqnorm(AdamTable t, float* __restrict__ partial,
                                                              double* __restrict__ count, double* __restrict__ stepbuf) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int ti = adam_tensor_of(t, b);
  const float* g = t.g[ti];
  const int64_t base = (int64_t)(b - t.cstart[ti]) * kAdamChunk;
  const int64_t n = t.numel[ti];
  float s = 0.f;
  if (g) {
#pragma unroll
    for (int k = 0; k < kAdamPerThread; ++k) {
      const int64_t i = base + k * kAdamThreads + threadIdx.x;
      if (i < n) {
        const float x = g[i];
        s += x * x;
      }
    }
  }
  s = adam_block_sum(s, red);
  if (threadIdx.x == 0) {
    partial[t.chunk0 + b] = s;
    if (t.chunk0 == 0 && b == 0) {
      const double c = *count;
      *stepbuf = c;
      *count = c + 1.0;
    }
  }
}

__global__ __launch_bounds__(kAdamThreads) void k_adam_update(AdamTable t, const float* __restrict__ partial,
                                                              const double* __restrict__ stepbuf, AdamHyper h,
                                                              float* __restrict__ gnorm_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < h.nchunks; i += kAdamThreads) s += partial[i];
  const float gnorm = sqrtf(adam_block_sum(s, red));
  const bool trigger = gnorm < h.max_norm;
  const float denom = trigger ? 1.f : gnorm;
  const float mult = trigger ? 1.f : h.max_norm;
  const double prev = *stepbuf;
  double lr = h.lr0;
  for (int j = 0; j < h.nb; ++j)
    if (prev >= h.bound[j] * h.spi) lr *= h.factor[j];
  const float lrf = (float)lr;
  const float c1 = (float)(1.0 - pow(h.b1, prev + 1.0));
  const float c2 = (float)(1.0 - pow(h.b2, prev + 1.0));
  const float b1 = (float)h.b1, b2 = (float)h.b2;
  const float a1 = (float)(1.0 - h.b1), a2 = (float)(1.0 - h.b2);
  if (t.chunk0 == 0 && blockIdx.x == 0 && threadIdx.x == 0) *gnorm_out = gnorm;

  const int b = blockIdx.x;
  const int ti = adam_tensor_of(t, b);
  const float* g = t.g[ti];
  float* p = t.p[ti];
  float* m = t.m[ti];
  float* v = t.v[ti];
  const int64_t base = (int64_t)(b - t.cstart[ti]) * kAdamChunk;
  const int64_t n = t.numel[ti];
#pragma unroll 4
  for (int k = 0; k < kAdamPerThread; ++k) {
    const int64_t i = base + k * kAdamThreads + threadIdx.x;
    if (i >= n) break;
    float gr = g ? g[i] : 0.f;
    gr = gr / denom;
    gr = gr * mult;
    const float mu = m[i] * b1 + a1 * gr;
    const float nu = v[i] * b2 + a2 * (gr * gr);
    const float pv = p[i];
    float u = (mu / c1) / (sqrtf(nu / c2) + h.eps);
    u = u + h.wd * pv;
    u = u * lrf;
    m[i] = mu;
    v[i] = nu;
    p[i] = pv - u;
  }
}

static int64_t adam_chunks(int64_t numel) { return (numel + kAdamChunk - 1) / kAdamChunk; }

// ---- one launch per pass: the tensor table in device memory (inside the caller's scratch) ----------------------
// The kernel-argument table holds 80 tensors, so the det learner's 156 took two launches per pass; with the table in
// the scratch buffer (uploaded by an eager call, read unchanged by a graph capture of the same step) each pass is one
// launch.  Same per-chunk arithmetic and the same fixed reduction order as the kernels above (bit-identical).
struct AdamDesc {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t numel;
};

__device__ __forceinline__ int adam_tensor_of_dev(const int* __restrict__ cstart, int n, int b) {
  int lo = 0, hi = n - 1;   // largest ti with cstart[ti] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cstart[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kAdamThreads) void k_adam_sqnorm_t(const AdamDesc* __restrict__ desc,
                                                                const int* __restrict__ cstart, int n,
                                                                float* __restrict__ partial, double* __restrict__ count,
                                                                double* __restrict__ stepbuf) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int ti = adam_tensor_of_dev(cstart, n, b);
  const float* g = desc[ti].g;
  const int64_t base = (int64_t)(b - cstart[ti]) * kAdamChunk;
  const int64_t num = desc[ti].numel;
  float s = 0.f;
  if (g) {
#pragma unroll
    for (int k = 0; k < kAdamPerThread; ++k) {
      const int64_t i = base + k * kAdamThreads + threadIdx.x;
      if (i < num) {
        const float x = g[i];
        s += x * x;
      }
    }
  }
  s = adam_block_sum(s, red);
  if (threadIdx.x == 0) {
    partial[b] = s;
    if (b == 0) {
      const double c = *count;
      *stepbuf = c;
      *count = c + 1.0;
    }
  }
}

__global__ __launch_bounds__(kAdamThreads) void k_adam_update_t(const AdamDesc* __restrict__ desc,
                                                                const int* __restrict__ cstart, int n,
                                                                const float* __restrict__ partial,
                                                                const double* __restrict__ stepbuf, AdamHyper h,
                                                                float* __restrict__ gnorm_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < h.nchunks; i += kAdamThreads) s += partial[i];
  const float gnorm = sqrtf(adam_block_sum(s, red));
  const bool trigger = gnorm < h.max_norm;
  const float denom = trigger ? 1.f : gnorm;
  const float mult = trigger ? 1.f : h.max_norm;
  const double prev = *stepbuf;
  double lr = h.lr0;
  for (int j = 0; j < h.nb; ++j)
    if (prev >= h.bound[j] * h.spi) lr *= h.factor[j];
  const float lrf = (float)lr;
  const float c1 = (float)(1.0 - pow(h.b1, prev + 1.0));
  const float c2 = (float)(1.0 - pow(h.b2, prev + 1.0));
  const float b1 = (float)h.b1, b2 = (float)h.b2;
  const float a1 = (float)(1.0 - h.b1), a2 = (float)(1.0 - h.b2);
  if (blockIdx.x == 0 && threadIdx.x == 0) *gnorm_out = gnorm;

  const int b = blockIdx.x;
  const int ti = adam_tensor_of_dev(cstart, n, b);
  const AdamDesc d = desc[ti];
  const int64_t base = (int64_t)(b - cstart[ti]) * kAdamChunk;
#pragma unroll 4
  for (int k = 0; k < kAdamPerThread; ++k) {
    const int64_t i = base + k * kAdamThreads + threadIdx.x;
    if (i >= d.numel) break;
    float gr = d.g ? d.g[i] : 0.f;
    gr = gr / denom;
    gr = gr * mult;
    const float mu = d.m[i] * b1 + a1 * gr;
    const float nu = d.v[i] * b2 + a2 * (gr * gr);
    const float pv = d.p[i];
    float u = (mu / c1) / (sqrtf(nu / c2) + h.eps);
    u = u + h.wd * pv;
    u = u * lrf;
    d.m[i] = mu;
    d.v[i] = nu;
    d.p[i] = pv - u;
  }
}

// scratch layout: [stepbuf f64][partials f32 x nchunks]
// table layout (muz_adamw_table_*): [AdamDesc x ntensors][cstart i32 x (ntensors + 1)]
static size_t adam_table_bytes(int ntensors) { return sizeof(AdamDesc) * ntensors + 4 * (size_t)(ntensors + 1); }

static int adam_hyper(AdamHyper& h, float max_norm, double b1, double b2, float eps, float weight_decay, double lr0,
                      double steps_per_iteration, const double* boundaries, int32_t nb) {
  if (nb < 0 || nb > kAdamMaxBounds || (nb && !boundaries)) return MUZ_E_INVALID;
  h = AdamHyper{};
  h.b1 = b1, h.b2 = b2, h.lr0 = lr0, h.spi = steps_per_iteration;
  for (int j = 0; j < nb; ++j) h.bound[j] = boundaries[2 * j], h.factor[j] = boundaries[2 * j + 1];
  h.max_norm = max_norm, h.eps = eps, h.wd = weight_decay, h.nb = nb;
  return MUZ_OK;
}

// chunks over all tensors (-1: a negative size or more than 2^30 chunks)
static int64_t adam_total_chunks(const int64_t* numel, int32_t ntensors) {
  int64_t total = 0;
  for (int i = 0; i < ntensors; ++i) {
    if (numel[i] < 0) return -1;
    total += adam_chunks(numel[i]);
  }
  return total > (1 << 30) ? -1 : total;
}

}  // namespace muz

using namespace muz;

extern "C" {

int64_t muz_adamw_scratch_bytes(int32_t ntensors, const int64_t* numel) {
  if (ntensors < 0 || (ntensors && !numel)) return -1;
  const int64_t c = adam_total_chunks(numel, ntensors);
  return c < 0 ? -1 : 8 + 4 * c;
}

int64_t muz_adamw_table_bytes(int32_t ntensors) {
  return ntensors < 0 ? -1 : (int64_t)adam_table_bytes(ntensors);
}

int muz_adamw_table_write(void* table, float* const* params, const float* const* grads, float* const* mu,
                          float* const* nu, const int64_t* numel, int32_t ntensors, void* stream) {
  if (ntensors < 0 || !table || (ntensors && (!params || !grads || !mu || !nu || !numel))) return MUZ_E_INVALID;
  if (adam_total_chunks(numel, ntensors) < 0) return MUZ_E_INVALID;
  std::vector<char> tab(adam_table_bytes(ntensors), 0);
  AdamDesc* dd = reinterpret_cast<AdamDesc*>(tab.data());
  int* cs = reinterpret_cast<int*>(tab.data() + sizeof(AdamDesc) * ntensors);
  int nz = 0, c = 0;
  for (int i = 0; i < ntensors; ++i) {
    if (!numel[i]) continue;
    if (!params[i] || !mu[i] || !nu[i]) return MUZ_E_INVALID;
    dd[nz] = AdamDesc{params[i], grads[i], mu[i], nu[i], numel[i]};
    cs[nz++] = c;
    c += (int)adam_chunks(numel[i]);
  }
  cs[nz] = c;
  hipStream_t s = (hipStream_t)stream;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  MUZ_HIP_RET(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) return MUZ_E_INVALID;   // a table is written eagerly, never captured
  // stream-ordered after earlier steps that read the table, and complete before the host vector goes away
  MUZ_HIP_RET(hipMemcpyAsync(table, tab.data(), tab.size(), hipMemcpyHostToDevice, s));
  MUZ_HIP_RET(hipStreamSynchronize(s));
  return MUZ_OK;
}

int muz_adamw_step_table(const void* table, const int64_t* numel, int32_t ntensors, double* count, void* scratch,
                         float* gnorm, float max_norm, double b1, double b2, float eps, float weight_decay, double lr0,
                         double steps_per_iteration, const double* boundaries, int32_t nb, void* stream) {
  if (ntensors < 0 || !table || !count || !scratch || !gnorm || (ntensors && !numel)) return MUZ_E_INVALID;
  AdamHyper h;
  if (int rc = adam_hyper(h, max_norm, b1, b2, eps, weight_decay, lr0, steps_per_iteration, boundaries, nb))
    return rc;
  const int64_t total = adam_total_chunks(numel, ntensors);
  if (total < 0) return MUZ_E_INVALID;
  if (total == 0) return MUZ_OK;
  h.nchunks = (int)total;
  int nz = 0;
  for (int i = 0; i < ntensors; ++i) nz += numel[i] != 0;
  double* stepbuf = (double*)scratch;
  float* partial = (float*)((char*)scratch + 8);
  hipStream_t s = (hipStream_t)stream;
  const AdamDesc* ddev = reinterpret_cast<const AdamDesc*>(table);
  const int* cdev = reinterpret_cast<const int*>((const char*)table + sizeof(AdamDesc) * ntensors);
  k_adam_sqnorm_t<<<(int)total, kAdamThreads, 0, s>>>(ddev, cdev, nz, partial, count, stepbuf);
  if (int rc = muz_last_launch_error()) return rc;
  k_adam_update_t<<<(int)total, kAdamThreads, 0, s>>>(ddev, cdev, nz, partial, stepbuf, h, gnorm);
  return muz_last_launch_error();
}

int muz_adamw_step(float* const* params, const float* const* grads, float* const* mu, float* const* nu,
                   const int64_t* numel, int32_t ntensors, double* count, void* scratch, float* gnorm,
                   float max_norm, double b1, double b2, float eps, float weight_decay, double lr0,
                   double steps_per_iteration, const double* boundaries, int32_t nb, void* stream) {
  if (ntensors < 0) return MUZ_E_INVALID;
  if (!count || !scratch || !gnorm || (ntensors && (!params || !grads || !mu || !nu || !numel))) return MUZ_E_INVALID;
  AdamHyper h;
  if (int rc = adam_hyper(h, max_norm, b1, b2, eps, weight_decay, lr0, steps_per_iteration, boundaries, nb))
    return rc;
  for (int i = 0; i < ntensors; ++i)
    if (numel[i] < 0 || (numel[i] && (!params[i] || !mu[i] || !nu[i]))) return MUZ_E_INVALID;
  const int64_t total = adam_total_chunks(numel, ntensors);
  if (total < 0) return MUZ_E_INVALID;
  if (total == 0) return MUZ_OK;
  h.nchunks = (int)total;
  double* stepbuf = (double*)scratch;
  float* partial = (float*)((char*)scratch + 8);
  hipStream_t s = (hipStream_t)stream;

  // the tensors travel in the kernel arguments (copied at launch and at capture: nothing the host or a later
  // call could change under a replayed graph); muz_adamw_step_table is the one-launch-per-pass form
  std::vector<AdamTable> tabs;
  int chunk = 0;
  for (int i = 0; i < ntensors; ++i) {
    if (!numel[i]) continue;
    if (tabs.empty() || tabs.back().n == kAdamMaxTensors) {
      tabs.push_back(AdamTable{});
      tabs.back().chunk0 = chunk;
    }
    AdamTable& t = tabs.back();
    t.numel[t.n] = numel[i];
    t.p[t.n] = params[i], t.g[t.n] = grads[i], t.m[t.n] = mu[i], t.v[t.n] = nu[i];
    chunk += (int)adam_chunks(numel[i]);
    t.cstart[++t.n] = chunk - t.chunk0;
  }
  for (size_t k = 0; k < tabs.size(); ++k) {
    k_adam_sqnorm<<<tabs[k].cstart[tabs[k].n], kAdamThreads, 0, s>>>(tabs[k], partial, count, stepbuf);
    if (int rc = muz_last_launch_error()) return rc;
  }
  for (size_t k = 0; k < tabs.size(); ++k) {
    k_adam_update<<<tabs[k].cstart[tabs[k].n], kAdamThreads, 0, s>>>(tabs[k], partial, stepbuf, h, gnorm);
    if (int rc = muz_last_launch_error()) return rc;
  }
  return MUZ_OK;
}

}  // extern "C"
