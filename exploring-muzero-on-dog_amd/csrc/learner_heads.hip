// The learner's output heads as ONE launch each way (csrc/learner_heads.hip; learner._OutHeads):
//   PredictionNetwork4's policy logits Dense_2 and value head Dense_4 -> relu -> Dense_5 -> tanh
//   (muzero_deterministic_madn.py:572-583), over the K + 1 unroll steps' hidden layers;
//   DynamicsNetwork4's reward / discount heads Dense_6 | Dense_7 -> relu -> reward_head | discount_head over
//   [next latent, one_hot(action)] (lines 437-455), over the K steps.
// As library GEMMs + bias adds + activations they were ~18 launches forward and ~20 backward of ~5 us each; the
// layers are tiny (<= 280 inputs, <= 64 outputs), so one wave per row does them from registers / LDS.
// Backward gives the input gradients and the pre-activation gradients (dz) the weight gradients need; the weight
// and bias gradients themselves go to the grouped launches of learner.GradSink (X^T dz, column sums).
// Sums run in k order per output (a plain fma chain, the bias added last, as x @ W + b): fp32, not bit-identical
// to the BLAS forms they replace (tests/test_gpu_learner_fused.py holds them to 1e-5 relative).
#include "launch.hpp"

namespace muz {

constexpr int kHW = 64;                 // hidden width of the value / reward / discount heads
constexpr int kHP = 128;                // policy / value hidden width (Pred4 Dense_1 / Dense_3 outputs)
constexpr int kHL = 256;                // latent
constexpr int kHMaxA = 32;              // actions (det 24)
constexpr int kHWaves = 4;

__device__ __forceinline__ float hsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(64 * kHWaves) void k_heads_fwd(muz_heads_args a) {
  __shared__ float xs[kHWaves][kHL + kHMaxA];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rw = blockIdx.x * kHWaves + w;
  float* x = xs[w];
  const int A = a.A;
  if (rw < a.R) {                                              // ---- prediction heads of row rw
    const int r = rw;
    for (int k = lane; k < kHP; k += 64) {
      x[k] = a.pol_h[(size_t)r * kHP + k];
      x[kHP + k] = a.v_h[(size_t)r * kHP + k];
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < A) {                                            // policy logits: Dense_2
      float s = 0.f;
      for (int k = 0; k < kHP; ++k) s = fmaf(x[k], a.W2[k * A + lane], s);
      a.logits[(size_t)r * A + lane] = s + a.b2[lane];
    }
    float h = 0.f;                                             // value Dense_4 -> relu
    for (int k = 0; k < kHP; ++k) h = fmaf(x[kHP + k], a.W4[k * kHW + lane], h);
    h = fmaxf(h + a.b4[lane], 0.f);
    a.h4[(size_t)r * kHW + lane] = h;
    const float v = hsum(h * a.W5[lane]) + a.b5[0];            // Dense_5 -> tanh
    if (lane == 0) a.value[r] = tanhf(v);
    return;
  }
  const int r = rw - a.R;                                      // ---- dynamics heads of step row r
  if (r >= a.Rk) return;
  const int K6 = kHL + A;
  for (int k = lane; k < K6; k += 64) {
    const float v = k < kHL ? a.head_in[(size_t)r * kHL + k] : a.onehot[(size_t)r * A + (k - kHL)];
    x[k] = v;
    a.ri[(size_t)r * K6 + k] = v;                              // [next latent, one_hot] for the weight gradients
  }
  __builtin_amdgcn_wave_barrier();
  float h6 = 0.f, h7 = 0.f;
  for (int k = 0; k < K6; ++k) {
    h6 = fmaf(x[k], a.W6[k * kHW + lane], h6);
    h7 = fmaf(x[k], a.W7[k * kHW + lane], h7);
  }
  h6 = fmaxf(h6 + a.b6[lane], 0.f);
  h7 = fmaxf(h7 + a.b7[lane], 0.f);
  a.h6[(size_t)r * kHW + lane] = h6;
  a.h7[(size_t)r * kHW + lane] = h7;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float rl = hsum(h6 * a.Wr[lane * 3 + j]) + a.br[j];
    const float dl = hsum(h7 * a.Wd[lane * 3 + j]) + a.bd[j];
    if (lane == 0) {
      a.rl[(size_t)r * 3 + j] = rl;
      a.dl[(size_t)r * 3 + j] = dl;
    }
  }
}

__global__ __launch_bounds__(64 * kHWaves) void k_heads_bwd(muz_heads_args a) {
  __shared__ float ds[kHWaves][2 * kHW + kHMaxA];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rw = blockIdx.x * kHWaves + w;
  float* d = ds[w];
  const int A = a.A;
  if (rw < a.R) {                                              // ---- prediction heads of row rw
    const int r = rw;
    if (lane < A) d[2 * kHW + lane] = a.g_logits ? a.g_logits[(size_t)r * A + lane] : 0.f;
    const float y = a.value[r];
    const float dv = (a.g_value ? a.g_value[r] : 0.f) * (1.f - y * y);   // tanh backward
    const float h = a.h4[(size_t)r * kHW + lane];
    const float dz = h > 0.f ? dv * a.W5[lane] : 0.f;                      // Dense_5, relu backward
    d[lane] = dz;
    a.dz4[(size_t)r * kHW + lane] = dz;
    if (lane == 0) a.dv5[r] = dv;
    __builtin_amdgcn_wave_barrier();
    for (int k = lane; k < kHP; k += 64) {
      float sv = 0.f, sp = 0.f;
      for (int l = 0; l < kHW; ++l) sv = fmaf(d[l], a.W4[k * kHW + l], sv);
      for (int c = 0; c < A; ++c) sp = fmaf(d[2 * kHW + c], a.W2[k * A + c], sp);
      a.d_v_h[(size_t)r * kHP + k] = sv;
      a.d_pol_h[(size_t)r * kHP + k] = sp;
    }
    return;
  }
  const int r = rw - a.R;                                      // ---- dynamics heads of step row r
  if (r >= a.Rk) return;
  float s6 = 0.f, s7 = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    s6 = fmaf(a.g_rl ? a.g_rl[(size_t)r * 3 + j] : 0.f, a.Wr[lane * 3 + j], s6);
    s7 = fmaf(a.g_dl ? a.g_dl[(size_t)r * 3 + j] : 0.f, a.Wd[lane * 3 + j], s7);
  }
  const float dz6 = a.h6[(size_t)r * kHW + lane] > 0.f ? s6 : 0.f;
  const float dz7 = a.h7[(size_t)r * kHW + lane] > 0.f ? s7 : 0.f;
  d[lane] = dz6;
  d[kHW + lane] = dz7;
  a.dz6[(size_t)r * kHW + lane] = dz6;
  a.dz7[(size_t)r * kHW + lane] = dz7;
  __builtin_amdgcn_wave_barrier();
  for (int k = lane; k < kHL; k += 64) {                      // the next latent's gradient (the one-hot has none)
    float t6 = 0.f, t7 = 0.f;
    for (int l = 0; l < kHW; ++l) {
      t6 = fmaf(d[l], a.W6[k * kHW + l], t6);
      t7 = fmaf(d[kHW + l], a.W7[k * kHW + l], t7);
    }
    a.d_head_in[(size_t)r * kHL + k] = t6 + t7;
  }
}

static int heads_check(const muz_heads_args* a) {
  if (!a || a->R < 0 || a->Rk < 0 || a->A < 1 || a->A > kHMaxA) return MUZ_E_INVALID;
  return MUZ_OK;
}

}  // namespace muz

using namespace muz;

extern "C" {

int muz_heads_fwd(const muz_heads_args* a, void* stream) {
  int rc = heads_check(a);
  if (rc) return rc;
  MUZ_HOST_CHECK(a->pol_h && a->v_h && a->W2 && a->b2 && a->W4 && a->b4 && a->W5 && a->b5 && a->logits && a->value &&
                 a->h4);
  MUZ_HOST_CHECK(a->Rk == 0 || (a->head_in && a->onehot && a->W6 && a->b6 && a->Wr && a->br && a->W7 && a->b7 && a->Wd &&
                                a->bd && a->rl && a->dl && a->h6 && a->h7 && a->ri));
  const int rows = a->R + a->Rk;
  if (rows == 0) return MUZ_OK;
  k_heads_fwd<<<(rows + kHWaves - 1) / kHWaves, 64 * kHWaves, 0, (hipStream_t)stream>>>(*a);
  return muz_last_launch_error();
}

int muz_heads_bwd(const muz_heads_args* a, void* stream) {
  int rc = heads_check(a);
  if (rc) return rc;
  MUZ_HOST_CHECK(a->d_pol_h && a->d_v_h && a->dz4 && a->dv5);
  MUZ_HOST_CHECK(a->Rk == 0 || (a->d_head_in && a->dz6 && a->dz7));
  const int rows = a->R + a->Rk;
  if (rows == 0) return MUZ_OK;
  k_heads_bwd<<<(rows + kHWaves - 1) / kHWaves, 64 * kHWaves, 0, (hipStream_t)stream>>>(*a);
  return muz_last_launch_error();
}

}  // extern "C"
