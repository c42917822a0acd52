// Probe: does f32 VALU FMA work overlap v_mfma_f32_16x16x4_f32 on one SIMD (gfx950)?
//   hipcc -O3 --offload-arch=gfx950 profiles/coissue_probe.hip -o profiles/coissue_probe
// Variants (one workgroup per CU, W waves per workgroup, each wave an independent stream):
//   0: MFMA only (4 independent accumulators)   1: VALU FMA only (16 independent chains)
//   2: both interleaved (1 MFMA : F VALU FMAs)   3: v_pk_fma only           4: MFMA + v_pk_fma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int MODE, int F>
__global__ void probe(float* out, int iters, float s) {
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  float v[16];
  f32x2 p[8];
  for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 0.001f + i;
  for (int i = 0; i < 8; ++i) p[i] = f32x2{v[2 * i], v[2 * i + 1]};
  const float a = s * threadIdx.x, b = s + 1.f;
  const f32x2 a2 = {a, a}, b2 = {b, b};
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0 || MODE == 2 || MODE == 4) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
      if (MODE == 2)
        for (int i = 0; i < F; ++i) v[i] = __builtin_fmaf(v[i], a, b);
      if (MODE == 4)
        for (int i = 0; i < F; ++i) p[i] = __builtin_elementwise_fma(p[i], a2, b2);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc1, 0, 0, 0);
      if (MODE == 2)
        for (int i = 0; i < F; ++i) v[i + 8] = __builtin_fmaf(v[i + 8], a, b);
      if (MODE == 4)
        for (int i = 0; i < F; ++i) p[(i + 4) & 7] = __builtin_elementwise_fma(p[(i + 4) & 7], a2, b2);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc3, 0, 0, 0);
    }
    if (MODE == 1)
      for (int i = 0; i < 16; ++i) v[i] = __builtin_fmaf(v[i], a, b);
    if (MODE == 3)
      for (int i = 0; i < 8; ++i) p[i] = __builtin_elementwise_fma(p[i], a2, b2);
  }
  float r = acc0[0] + acc1[1] + acc2[2] + acc3[3];
  for (int i = 0; i < 16; ++i) r += v[i];
  for (int i = 0; i < 8; ++i) r += p[i][0] + p[i][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE, int F>
double run(int waves, int iters, double flop_per_iter_wave) {
  float* out;
  hipMalloc(&out, 256 * 1024 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<MODE, F><<<256, 64 * waves>>>(out, iters, 1e-7f);
  hipEventRecord(e0);
  probe<MODE, F><<<256, 64 * waves>>>(out, iters, 1e-7f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipFree(out);
  const double tf = 256.0 * waves * iters * flop_per_iter_wave / (ms * 1e-3) / 1e12;
  printf("mode %d F=%d waves/CU %2d: %.3f ms  %.1f TFLOP/s\n", MODE, F, waves, ms, tf);
  return tf;
}

int main() {
  const int it = 20000;
  const double mf = 4 * 2048.0;   // 4 MFMAs per iter
  for (int w : {4, 8}) {
    run<0, 0>(w, it, mf);
    run<1, 0>(w, it, 16 * 64 * 2.0);
    run<3, 0>(w, it, 8 * 64 * 4.0);
    run<2, 2>(w, it, mf + 4 * 64 * 2.0);
    run<2, 4>(w, it, mf + 8 * 64 * 2.0);
    run<2, 8>(w, it, mf + 16 * 64 * 2.0);
    run<4, 2>(w, it, mf + 4 * 64 * 4.0);
    run<4, 4>(w, it, mf + 8 * 64 * 4.0);
  }
  return 0;
}
