// Shared helpers for the libmuz HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/muz.h"

#define MUZ_HOST_CHECK(cond)           \
  do {                                 \
    if (!(cond)) return MUZ_E_INVALID; \
  } while (0)

#define MUZ_HIP_RET(expr)                  \
  do {                                     \
    hipError_t _e = (expr);                \
    if (_e != hipSuccess) return (int)_e;  \
  } while (0)

// Root scratch row (muz_nets_root_scratch_bytes): RepresentationNetwork2's flattened conv maps (k_repr_conv) and, after
// them, its Dense_0 output before LayerNorm_3 (k_dense0) -- one row per game
constexpr int kConvMapFloats = 56 * 64;
// k_dense0 splits Dense_0's K = 3584 over kD0KSplit workgroups per output tile (2: 512 workgroups, 2 per CU); each
// writes its partial plane after the maps, the consumer (repr16<.., true>) adds them in plane order, then the bias
#ifndef MUZ_D0_KSPLIT
#define MUZ_D0_KSPLIT 2
#endif
constexpr int kD0KSplit = MUZ_D0_KSPLIT;
constexpr int kConvRowFloats = kConvMapFloats + 256 * kD0KSplit;

static inline int muz_last_launch_error() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MUZ_OK : (int)e;
}

// ---- JAX integer semantics ----------------------------------------------------------
// Python/JAX floor division and modulo (x // y, x % y with the sign of y).
__device__ __forceinline__ int fdiv(int a, int b) {
  int q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
__device__ __forceinline__ int fmodp(int a, int b) {
  int r = a % b;
  if (r != 0 && ((r < 0) != (b < 0))) r += b;
  return r;
}
// jnp gather index: a negative index is normalised ONCE (i + n), then clamped to [0, n-1].
// a mod n (floor convention, result in [0, n)) for the player-count moduli of the rules (n = P in [2, 4],
// -n <= a < 4n): conditional adds / subtracts instead of a runtime integer division (~25 instructions each),
// which the legality checks and the encode ran once per action / cell.
__device__ __forceinline__ int mod_small(int a, int n) {
  a += a < 0 ? n : 0;
  a -= a >= n ? n : 0;
  a -= a >= n ? n : 0;
  a -= a >= n ? n : 0;
  return a;
}
__device__ __forceinline__ int jidx(int i, int n) {
  i = (i < 0) ? i + n : i;
  return i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
}

// Address-space qualifiers.  Pointers loaded from structs are generic ("flat") to the compiler;
// flat loads count on BOTH vmcnt and lgkmcnt, so every LDS wait would also wait for in-flight weight
// loads.  Weight tables are therefore read through the kernarg segment (AS4 -> scalar loads) and
// every global array through an AS1 (global) pointer.
#define AS1 __attribute__((address_space(1)))
#define AS4 __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ const AS1 T* gp(const T* p) {
  return (const AS1 T*)p;
}
template <class T>
__device__ __forceinline__ AS1 T* gpw(T* p) {
  return (AS1 T*)p;
}
// kernel argument 0 seen through the kernarg segment (scalar loads), laundered so the compiler
// re-reads fields at the point of use instead of pinning them all in registers.
template <class T>
__device__ __forceinline__ const AS4 T* kernarg0() {
  const AS4 T* p = (const AS4 T*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// Dynamic index into a small register array without a scratch round trip.  The empty asm after each select
// keeps LLVM from folding the chain back into a[i] -- which demotes the whole array to scratch memory (it did:
// 176 B/lane of scratch in k_det_round, round 2).
template <int N>
__device__ __forceinline__ int rsel(const int (&a)[N], int i) {
  int r = a[0];
#pragma unroll
  for (int j = 1; j < N; ++j) {
    r = (i == j) ? a[j] : r;
    asm volatile("" : "+v"(r));
  }
  return r;
}

// a[i] = v for a dynamic i, by selects over the register array (same folding guard as rsel).
template <int N>
__device__ __forceinline__ void rset(int (&a)[N], int i, int v) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    int x = (i == j) ? v : a[j];
    asm volatile("" : "+v"(x));
    a[j] = x;
  }
}
