// Verdict r3 item 3: can a small batch's 16-game search tile run faster split over two CUs?
//
// The search kernel's per-simulation time is one workgroup's chain of ~15 dense layers (16 rows x 256 outputs, weights
// streamed from L2, a barrier per layer; nn.hpp mfma_ring_impl).  Below 4096 games per GPU most CUs idle, so the
// candidate is to give each tile TWO workgroups on two CUs of the same XCD, each computing 128 of a layer's 256
// output columns, and to exchange the halves (and with them the LayerNorm statistics' inputs) through L2 once per
// layer: publish 8 KB (16 rows x 128 fp32), release fence, flag; wait for the partner's flag, acquire, read its 8 KB
// into the LDS tile.  This program times exactly that loop against the one-CU loop, with LAYERS 256x256 layers per
// repetition, every tile's workgroups resident (grid <= CUs):
//
//   mode 0: one workgroup per tile, 8 waves x 2 column tiles (the search kernel's loop)
//   mode 1: two workgroups per tile (partners b and b ^ 8: the same XCD under round-robin dispatch), 8 waves x 1
//           column tile each, plus the per-layer exchange
//   mode 2: mode 1 without the exchange (the compute half alone; wrong results, timing only)
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 profiles/split_tile_bench.hip -o profiles/split_tile_bench
//   ./split_tile_bench <tiles> <mode> [reps]
// Every wait is bounded (kSpinCap polls): a workgroup that gives up reports it and the run is invalid.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../exploring-muzero-on-dog_amd/csrc/nn.hpp"

using namespace muz;

constexpr int LDA = LAT + kLdPad;
constexpr int LAYERS = 14;
constexpr int KB = 16;
constexpr long kSpinCap = 1L << 22;

template <int NT>
__device__ __forceinline__ const float* group_w(const float* W, int l, int half) {
  // packed like nets.pack_dense with nw = 8 waves x NT tiles per half: wave w of half h owns columns
  // (h * 8 + w) * NT * 16 .. +NT*16 (the layout only has to give every wave its own contiguous stream)
  return W + (size_t)l * 65536 + ((size_t)half * kWaves + (threadIdx.x >> 6)) * KB * 64 * NT * 4;
}

template <int NT, int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_split(const float* W, int reps, float* xch, unsigned* flag,
                                                       float* out, unsigned long long* cyc, int* err) {
  __shared__ __attribute__((aligned(16))) float A[kRows * LDA];
  for (int i = threadIdx.x; i < kRows * LDA; i += kThreads) A[i] = 0.001f * (float)(i % 97);
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const int partner = b ^ 8;
  const int half = MODE == 0 ? 0 : ((b >> 3) & 1);
  f32x4 b0[NT], b1[NT], acc[NT], keep[NT];
  auto pf = [&](int l) {
    const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(group_w<NT>(W, l, half))) + lane * NT;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      b0[t] = wp[t];
      b1[t] = wp[64 * NT + t];
    }
  };
#pragma unroll
  for (int t = 0; t < NT; ++t) keep[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  pf(0);
  unsigned step = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
    for (int l = 0; l < LAYERS; ++l) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      mfma_ring_impl<NT, false>(group_w<NT>(W, l, half), KB, A, LDA, acc, b0, b1);
      pf(l + 1 < LAYERS ? l + 1 : 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) keep[t] += acc[t];
      __syncthreads();   // every wave has read the tile
      // this workgroup's output columns into the tile (rows r, 4 columns per lane and tile)
      const int col0 = (half * kWaves + (threadIdx.x >> 6)) * NT * 16;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        *reinterpret_cast<f32x4*>(A + r * LDA + col0 + t * 16 + 4 * g) = acc[t] * 0.001f;
      if constexpr (MODE == 1) {
        ++step;
        // publish: 16 rows x 128 columns = one float4 per thread, then release and raise the flag
        float* mine = xch + (size_t)b * kRows * 128;
        const int pr = threadIdx.x >> 5, pc = (threadIdx.x & 31) * 4;   // row, column of this thread's float4
        __syncthreads();
        *reinterpret_cast<f32x4*>(mine + pr * 128 + pc) =
            *reinterpret_cast<const f32x4*>(A + pr * LDA + half * 128 + pc);
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(flag + b, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // wait for the partner's half of this layer
        if (threadIdx.x == 0) {
          long n = 0;
          while (__hip_atomic_load(flag + partner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < step) {
            __builtin_amdgcn_s_sleep(1);
            if (++n > kSpinCap) {
              atomicAdd(err, 1);
              break;
            }
          }
        }
        __syncthreads();
        __threadfence();
        const float* theirs = xch + (size_t)partner * kRows * 128;
        *reinterpret_cast<f32x4*>(A + pr * LDA + (1 - half) * 128 + pc) =
            *reinterpret_cast<const f32x4*>(theirs + pr * 128 + pc);
      }
      __syncthreads();
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

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 64;
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  if (mode != 0 && (tiles % 8)) {
    fprintf(stderr, "tiles must be a multiple of 8 for the paired modes\n");
    return 1;
  }
  // grid: one workgroup per tile (mode 0) or two; partners b, b ^ 8 are in consecutive groups of 8
  const int grid = mode == 0 ? tiles : 2 * tiles;
  if (grid > 256) {
    fprintf(stderr, "grid %d exceeds the 256 CUs (every partner must be resident)\n", grid);
    return 1;
  }
  std::vector<float> h((size_t)LAYERS * 65536);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-6f;
  float *W, *out, *xch;
  unsigned* flag;
  int* err;
  unsigned long long* cyc;
  CK(hipMalloc(&W, h.size() * 4));
  CK(hipMalloc(&out, (size_t)grid * kThreads * 4));
  CK(hipMalloc(&xch, (size_t)grid * kRows * 128 * 4));
  CK(hipMalloc(&flag, (size_t)grid * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&cyc, (size_t)grid * 16));
  CK(hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  auto launch = [&]() {
    CK(hipMemset(flag, 0, (size_t)grid * 4));
    if (mode == 0) k_split<2, 0><<<grid, kThreads>>>(W, reps, xch, flag, out, cyc, err);
    else if (mode == 1) k_split<1, 1><<<grid, kThreads>>>(W, reps, xch, flag, out, cyc, err);
    else k_split<1, 2><<<grid, kThreads>>>(W, reps, xch, flag, out, cyc, err);
    CK(hipGetLastError());
  };
  CK(hipMemset(err, 0, 4));
  launch();   // warm-up
  CK(hipDeviceSynchronize());
  launch();   // timed by the in-kernel clocks
  CK(hipDeviceSynchronize());
  int herr = 0;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> c((size_t)grid * 2);
  CK(hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost));
  double cs = 0, rs = 0;
  for (int i = 0; i < grid; ++i) {
    cs += (double)c[2 * i];
    rs += (double)c[2 * i + 1];
  }
  cs /= grid;
  rs /= grid;
  // per-layer time from the in-kernel clocks of the timed launch, averaged over the workgroups
  const double us_layer = rs * 0.01 / reps / LAYERS;   // s_memrealtime ticks at 100 MHz
  printf("tiles=%d mode=%d (%s): grid %d, %.2f us per 256x256 layer per tile (clock %.2f GHz)%s\n", tiles, mode,
         mode == 0 ? "one CU per tile" : (mode == 1 ? "two CUs per tile + L2 exchange" : "two CUs, no exchange"),
         grid, us_layer, cs / rs * 0.1, herr ? "  INVALID: a wait hit its cap" : "");
  return herr ? 2 : 0;
}
