// The weight-stream MFMA loop of loop_bench.hip on the 4-row blocks of v_mfma_f32_4x4x1_16b_f32 (VERDICT r4 items
// 6 / 3 / 7: a branch-sorted tile schedule -- each 4-row block of a 16-row tile picks its own trunk's weights --
// and 8-row tiles without padding rows).  Every workgroup (one per CU, 8 waves) multiplies a resident LDS tile of
// ROWS rows through LAYERS 256x256 fp32 layers whose weights (3.5 MB per trunk) stay L2-resident; wave w owns output
// columns [32w, 32w + 32).  One 4x4x1_16b instruction = 16 blocks of (4 columns x 4 rows x k 1):
//   ROWS 16: 4 column blocks x 4 row blocks (16 columns), two instructions per k-step;
//   ROWS  8: 8 column blocks x 2 row blocks (32 columns), one instruction per k-step.
// Operands (weights as the A operand, rows as B, as nn.hpp's D = W^T A^T): lane 4b + i of block b holds weight
// column 4 cb + i (A) and row 4 rb + i (B).  Weights are packed [k/4][column][4] so a lane's float4 covers 4
// k-steps and the 4 lanes of a block read 64 consecutive bytes; lanes of different row blocks read the same bytes
// (TRUNKS 1) or the other trunk's (TRUNKS 2: row blocks 2, 3 -- or row block 1 at ROWS 8 -- on trunk 1).
// Reports MFMA-busy fraction of SIMD cycles (8 cycles per 4x4x1_16b instruction), clock and TFLOP/s; the result
// values are not checked (timing only).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DQ_ROWS=16|8 -DQ_TRUNKS=1|2 profiles/loop_bench_4x4.hip -o lb4 && ./lb4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef Q_ROWS
#define Q_ROWS 16
#endif
#ifndef Q_TRUNKS
#define Q_TRUNKS 1
#endif
#ifndef Q_DEPTH
#define Q_DEPTH 8   // k4-steps of weights in flight
#endif
#ifndef Q_SYNC
#define Q_SYNC 1
#endif
constexpr int ROWS = Q_ROWS, TRUNKS = Q_TRUNKS;
constexpr int WAVES = 8, THREADS = WAVES * 64, LAT = 256, LDA = LAT + 8, LAYERS = 14;
constexpr int RB = ROWS / 4;            // row blocks per instruction
constexpr int CB = 16 / RB;             // column blocks per instruction
constexpr int COLS_PER_INSTR = 4 * CB;  // 16 or 32
constexpr int INSTR = 32 / COLS_PER_INSTR;   // instructions per k-step per wave (wave = 32 columns)
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(THREADS, 1) void k_loop4(const float* W, int reps, float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) float A[ROWS * LDA];
  for (int i = threadIdx.x; i < ROWS * LDA; i += THREADS) A[i] = 0.001f * (float)(i % 97);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = lane >> 2, q = lane & 3;
  const int rb = b / CB, cb = b % CB;
  const int trunk = (TRUNKS == 2 && rb >= RB / 2) ? 1 : 0;
  // lane's weight column (per instruction s) and row
  const int row = 4 * rb + q;
  const float* arow = A + row * LDA;
  f32x4 acc[INSTR], keep[INSTR];
#pragma unroll
  for (int s = 0; s < INSTR; ++s) keep[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
    for (int l = 0; l < LAYERS; ++l) {
      // packed [trunk][layer][k/4][256 columns][4]
      const f32x4* wl = reinterpret_cast<const f32x4*>(W) + ((size_t)(trunk * LAYERS + l) * (LAT / 4)) * LAT;
#pragma unroll
      for (int s = 0; s < INSTR; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      // ring of Q_DEPTH k4-steps of weights in flight (L2 latency ~ many steps of 4 MFMAs)
      f32x4 wr[Q_DEPTH][INSTR];
      const int col = 32 * w + 4 * cb + q;
#pragma unroll
      for (int d = 0; d < Q_DEPTH; ++d)
#pragma unroll
        for (int s = 0; s < INSTR; ++s) wr[d][s] = wl[(size_t)d * LAT + col + s * COLS_PER_INSTR];
#pragma unroll 1
      for (int k0 = 0; k0 < LAT / 4; k0 += Q_DEPTH) {
#pragma unroll
        for (int d = 0; d < Q_DEPTH; ++d) {
          const int k4 = k0 + d;
          const f32x4 a = *reinterpret_cast<const f32x4*>(arow + 4 * k4);
          f32x4 cur[INSTR];
#pragma unroll
          for (int s = 0; s < INSTR; ++s) cur[s] = wr[d][s];
          if (k4 + Q_DEPTH < LAT / 4) {
#pragma unroll
            for (int s = 0; s < INSTR; ++s) wr[d][s] = wl[(size_t)(k4 + Q_DEPTH) * LAT + col + s * COLS_PER_INSTR];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int s = 0; s < INSTR; ++s) acc[s] = __builtin_amdgcn_mfma_f32_4x4x1f32(cur[s][j], a[j], acc[s], 0, 0, 0);
        }
      }
#pragma unroll
      for (int s = 0; s < INSTR; ++s) keep[s] += acc[s];
      if (Q_SYNC) __syncthreads();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
#pragma unroll
  for (int s = 0; s < INSTR; ++s) sum += keep[s][0] + keep[s][1] + keep[s][2] + keep[s][3];
  out[blockIdx.x * THREADS + threadIdx.x] = sum;
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
  std::vector<float> h((size_t)TRUNKS * LAYERS * 65536);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-6f;
  float *W, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&W, h.size() * 4));
  CK(hipMalloc(&out, (size_t)grid * THREADS * 4));
  CK(hipMalloc(&cyc, (size_t)grid * 16));
  CK(hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_loop4<<<grid, THREADS>>>(W, reps, out, cyc);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int launches = 5;
  for (int i = 0; i < launches; ++i) k_loop4<<<grid, THREADS>>>(W, reps, out, cyc);
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
  // per SIMD: 2 waves x INSTR instructions x 256 k-steps x 8 cycles per layer
  const double mfma_cyc = (double)reps * LAYERS * (WAVES / 4) * INSTR * LAT * 8;
  const double flop = (double)grid * reps * LAYERS * 2.0 * ROWS * 256 * 256 * launches;
  printf("4x4x1_16b rows=%d trunks=%d depth=%d sync=%d: MFMA busy %.3f of SIMD cycles, clock %.2f GHz, %.1f TFLOP/s on %d rows "
         "(%.2f us per layer)\n",
         ROWS, TRUNKS, Q_DEPTH, Q_SYNC, mfma_cyc / cs, cs / rs * 0.1, flop / (ms * 1e-3) / 1e12, ROWS,
         ms * 1e3 / launches / reps / LAYERS);
  return 0;
}
