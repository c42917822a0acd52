// Round-6 probe: how v_mfma_f32_16x16x4_f32 rounds.  One wave per trial: lane l supplies the
// raw A / B operand values a[t][l], b[t][l] and the accumulator c[t][l][0..3]; the wave's D registers go to d[t][l].
// profiles/mfma_rounding.py crafts the operands, maps lanes to matrix elements and compares D with candidate
// orders (fmaf chain over k, exact sum rounded once, ...) computed exactly on the host.
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k_mfma_probe(const float* a, const float* b, const float* c, float* d, int n) {
  const int t = blockIdx.x, l = threadIdx.x;
  if (t >= n) return;
  const f32x4 acc = *reinterpret_cast<const f32x4*>(c + ((size_t)t * 64 + l) * 4);
  const f32x4 r = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(size_t)t * 64 + l], b[(size_t)t * 64 + l], acc, 0, 0, 0);
  *reinterpret_cast<f32x4*>(d + ((size_t)t * 64 + l) * 4) = r;
}

// the same sums as an fmaf chain on the VALU (k = 0..3 in order, then k = 3..0) for the host to compare against
__global__ __launch_bounds__(64) void k_fma_chain(const float* a, const float* b, const float* c, float* d, int n,
                                                  int reverse) {
  const int t = blockIdx.x, l = threadIdx.x;
  if (t >= n) return;
  // D[row][col] = C + sum_k A[row][k] B[k][col]; A[row][k] is lane row + 16 k's value, B[k][col] lane col + 16 k's
  const float* at = a + (size_t)t * 64;
  const float* bt = b + (size_t)t * 64;
  const int col = l & 15, rb = (l >> 4) * 4;
  for (int j = 0; j < 4; ++j) {
    const int row = rb + j;
    float s = c[((size_t)t * 64 + l) * 4 + j];
    for (int q = 0; q < 4; ++q) {
      const int k = reverse ? 3 - q : q;
      s = __builtin_fmaf(at[row + 16 * k], bt[col + 16 * k], s);
    }
    d[((size_t)t * 64 + l) * 4 + j] = s;
  }
}

extern "C" int mfma_probe(const float* a, const float* b, const float* c, float* d, int n, void* stream) {
  k_mfma_probe<<<n, 64, 0, (hipStream_t)stream>>>(a, b, c, d, n);
  return (int)hipGetLastError();
}

extern "C" int fma_chain(const float* a, const float* b, const float* c, float* d, int n, int reverse, void* stream) {
  k_fma_chain<<<n, 64, 0, (hipStream_t)stream>>>(a, b, c, d, n, reverse);
  return (int)hipGetLastError();
}
