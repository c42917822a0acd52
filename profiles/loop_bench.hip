// Isolated MFMA weight-stream loop of the search kernel (nn.hpp mfma_ring_impl): every workgroup (one per CU)
// multiplies a resident 16-row LDS tile through LAYERS 256x256 fp32 layers whose packed weights (3.5 MB) stay
// L2-resident, exactly as the fused Dyn4/Pred4 layers do, but without LayerNorm passes, epilogues or the tree.
// Reports the fraction of each SIMD's cycles the MFMA pipe was busy (s_memtime), and the shader clock.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 [-DMUZ_TILE_WAVES=4 -DLB_NT=4] [-DMUZ_RING_DEPTH=3]
//         [-DLB_SYNC=0] [-DLB_PAD=8] profiles/loop_bench.hip -o loop_bench && ./loop_bench
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../exploring-muzero-on-dog_amd/csrc/nn.hpp"

using namespace muz;

#ifndef LB_NT
#define LB_NT 2
#endif
#ifndef LB_SYNC
#define LB_SYNC 1   // workgroup barrier after every layer (as between the search kernel's layers)
#endif
#ifndef LB_PAD
#define LB_PAD kLdPad   // LDS row padding of the 16-row tile (floats)
#endif
constexpr int LDA = LAT + LB_PAD;
constexpr int LAYERS = 14;
constexpr int KB = 16;
static_assert(kWaves * LB_NT * 16 == 256, "waves x NT x 16 must cover the 256 outputs");

__global__ __launch_bounds__(kThreads, 1) void k_loop(const float* W, int reps, float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) float A[kRows * LDA];
  for (int i = threadIdx.x; i < kRows * LDA; i += kThreads) A[i] = 0.001f * (float)(i % 97);
  __syncthreads();
  constexpr int NT = LB_NT;
  const int lane = threadIdx.x & 63;
  auto group = [&](int l) { return W + (size_t)l * 65536 + (size_t)(threadIdx.x >> 6) * KB * 64 * NT * 4; };
  f32x4 b0[NT], b1[NT], acc[NT], keep[NT];
  auto pf = [&](int l) {
    const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(group(l))) + lane * NT;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      b0[t] = wp[t];
      b1[t] = wp[64 * NT + t];
    }
  };
#pragma unroll
  for (int t = 0; t < NT; ++t) keep[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  pf(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
    for (int l = 0; l < LAYERS; ++l) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      mfma_ring_impl<NT, false>(group(l), KB, A, LDA, acc, b0, b1);
      pf(l + 1 < LAYERS ? l + 1 : 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) keep[t] += acc[t];
      if (LB_SYNC) __syncthreads();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += keep[t][0] + keep[t][1] + keep[t][2] + keep[t][3];
  out[blockIdx.x * kThreads + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    cyc[2 * blockIdx.x] = t1 - t0;
    cyc[2 * blockIdx.x + 1] = r1 - r0;
  }
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 40;
  std::vector<float> h((size_t)LAYERS * 65536);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-6f;
  float *W, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&W, h.size() * 4));
  CK(hipMalloc(&out, (size_t)grid * kThreads * 4));
  CK(hipMalloc(&cyc, (size_t)grid * 16));
  CK(hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_loop<<<grid, kThreads>>>(W, reps, out, cyc);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int launches = 5;
  for (int i = 0; i < launches; ++i) k_loop<<<grid, kThreads>>>(W, reps, out, cyc);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned long long> c((size_t)grid * 2);
  CK(hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost));
  double cs = 0, rs = 0;
  for (int i = 0; i < grid; ++i) {
    cs += (double)c[2 * i];
    rs += (double)c[2 * i + 1];
  }
  cs /= grid;
  rs /= grid;
  // per SIMD: (kWaves / 4) waves x NT tiles x KB k-blocks x 4 MFMAs x 32 cycles per layer
  const double mfma_cyc = (double)reps * LAYERS * (kWaves / 4) * LB_NT * KB * 4 * 32;
  const double flop = (double)grid * reps * LAYERS * 2.0 * 16 * 256 * 256 * launches;
  printf("waves=%d NT=%d depth=%d sync=%d pad=%d: MFMA busy %.3f of SIMD cycles, clock %.2f GHz, %.1f TFLOP/s "
         "(%.1f us per layer)\n",
         kWaves, LB_NT, MUZ_RING_DEPTH, LB_SYNC, LB_PAD, mfma_cyc / cs, cs / rs * 0.1, flop / (ms * 1e-3) / 1e12, ms * 1e3 / launches / reps / LAYERS);
  return 0;
}
