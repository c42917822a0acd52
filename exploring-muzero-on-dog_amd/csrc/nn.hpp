// Fused fp32 MLP building blocks for 16-row tiles on CDNA4 MFMA (v_mfma_f32_16x16x4_f32).
//
// A workgroup of 8 waves (two per SIMD, so one wave's weight loads hide under the other's MFMAs)
// owns a tile of 16 rows (games).  Activations live in LDS ([16][ld] fp32 rows); a dense layer
// out = A[16][K] @ W[K][N] + b splits its N columns over the 8 waves (NT 16-column tiles each).  Per 16-deep k-block a lane reads ONE float4 of A from
// LDS (row lane&15, k = kb*16 + 4*(lane>>4) + j, j = 0..3) and NT float4 of pre-packed weights
// straight from global memory (L2/MALL resident, streamed once per tile), then issues 4*NT
// MFMAs, with the weights of the next two k-blocks in flight.  The f32-input MFMA is an exact
// k-ordered fma chain, so only the reduction order differs from the fp32 reference.  Row-wise ops
// (LayerNorm, min-max) use 32 lanes (half a wave) per row.
#pragma once
#include "common.hpp"

// Rounding pinned: no fma contraction anywhere after this point (the networks here, and the search kernels' tree
// arithmetic that includes this header); the products that should fuse are written as fmaf.  The compiler used to
// contract differently per inlined context -- e.g. the fused Pred4 LayerNorm_0 of skip_minmax16 folded the min-max
// multiply into the LayerNorm sums, which the separate ln16 pass cannot -- so the search kernel's networks and the
// root / recurrent kernels (the parity tests' oracle side) differed in the last bit.  Now every kernel built on
// these functions rounds identically.
#ifndef MUZ_PINNED_ROUNDING
#define MUZ_PINNED_ROUNDING 1
#endif
#if MUZ_PINNED_ROUNDING
#pragma clang fp contract(off)
#endif

// Every entity below lives in an inline namespace named after the tid() variant (MUZ_OPAQUE_TID, set by
// dog_search.hip only), so the two variants' inline functions and templates are distinct entities with distinct
// mangled names -- no ODR violation even if the translation units were linked into one device code object
// (-fgpu-rdc); muz::name still finds them.
#ifdef MUZ_OPAQUE_TID
#define MUZ_NN_NS nn_opaque_tid
#else
#define MUZ_NN_NS nn_direct_tid
#endif

namespace muz {
inline namespace MUZ_NN_NS {

#ifndef MUZ_TILE_WAVES
#define MUZ_TILE_WAVES 8   // waves per 16-row tile workgroup: 8 (2 per SIMD) or 16 (4 per SIMD)
#endif
// det networks' policy logits split over k (pred16 SPLITK_LOGITS; search, root and recurrent kernels alike, so
// their outputs stay bit-identical to each other)
#ifndef MUZ_SPLITK_LOGITS
#define MUZ_SPLITK_LOGITS 0
#endif
constexpr bool kSplitkLogits = MUZ_SPLITK_LOGITS != 0;
constexpr int kRows = 16;
constexpr int kWaves = MUZ_TILE_WAVES;
constexpr int kThreads = kWaves * 64;          // 512 / 1024
constexpr int kRowLanes = kThreads / kRows;    // lanes per row in row-wise phases: 32 / 64
constexpr int LAT = 256;
// The thread index for the network helpers' lane / wave offsets.  MUZ_OPAQUE_TID (dog_search.hip): an opaque copy at
// every use, so the offsets derived from it are recomputed where they are needed instead of being hoisted out of the
// search loop into registers the networks need (the compiler spilled them and reloaded them inside the MFMA loops).
#ifdef MUZ_OPAQUE_TID
__device__ __forceinline__ unsigned tid() {
  unsigned t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
#else
__device__ __forceinline__ unsigned tid() { return threadIdx.x; }
#endif
// ---- diagnostic fine-grained stamps (make EXTRA=-DMUZ_STAMPS2); compiled out otherwise -------------
enum { ST_MFMA = 0, ST_EPI = 1, ST_BAR = 2, ST_ROW = 3, ST_SEL = 4, ST_OTHER = 5, ST_TREE = 6, ST_PASS = 7, ST_DENTRY = 8,
       ST_FIRST = 11,   // (k_dog_search: a node's first-walk normaliser + top-prior list; counts at 9, 10, 12)
       ST_N = 14 };
#ifdef MUZ_STAMPS2
__device__ unsigned long long g_st2[ST_N];
struct StampState {
  unsigned long long last, acc[ST_N];
};
__device__ __forceinline__ StampState& st_state() {
  __shared__ StampState s;
  return s;
}
__device__ __forceinline__ void st_begin() {
  if (threadIdx.x == 0) {
    StampState& s = st_state();
    for (int i = 0; i < ST_N; ++i) s.acc[i] = 0;
    s.last = __builtin_amdgcn_s_memtime();
  }
}
__device__ __forceinline__ void ST(int cat) {
  if (threadIdx.x == 0) {
    StampState& s = st_state();
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    s.acc[cat] += t - s.last;
    s.last = t;
  }
}
__device__ __forceinline__ void st_end() {
  if (threadIdx.x == 0)
    for (int i = 0; i < ST_N; ++i) atomicAdd(&g_st2[i], st_state().acc[i]);
}
#define SYNC()         \
  do {                 \
    ST(ST_OTHER);      \
    __syncthreads();   \
    ST(ST_BAR);        \
  } while (0)
__device__ __forceinline__ void st_sim(int) {}
// an event count in category cat (thread 0's row): the categories past ST_DENTRY
__device__ __forceinline__ void st_count(int cat) {
  if (threadIdx.x == 0) st_state().acc[cat] += 1;
}
#elif defined(MUZ_TIMELINE)
// ---- diagnostic per-wave timeline (make EXTRA=-DMUZ_TIMELINE): lane 0 of every wave of workgroup
// MUZ_TL_WG records (s_memtime << 8 | category) at each segment end of simulation MUZ_TL_SIM.
#ifndef MUZ_TL_WG
#define MUZ_TL_WG 0
#endif
#ifndef MUZ_TL_SIM
#define MUZ_TL_SIM 20
#endif
constexpr int kTlMax = 1024;
__device__ unsigned long long g_tl[kWaves][kTlMax];
__device__ unsigned int g_tl_n[kWaves];
// per-wave record index in LDS (-1: not recording), so a stamp costs one LDS read, a vector store and an
// LDS write (no global read)
__device__ __forceinline__ int* tl_idx() {
  __shared__ int idx[kWaves];
  return idx;
}
__device__ __forceinline__ void st_begin() {
  if ((threadIdx.x & 63) == 0) tl_idx()[threadIdx.x >> 6] = -1;
}
__device__ __forceinline__ void ST(int cat) {
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    const int i = tl_idx()[w];
    if (i >= 0 && i < kTlMax) {
      g_tl[w][i] = (__builtin_amdgcn_s_memtime() << 8) | (unsigned)cat;
      tl_idx()[w] = i + 1;
      g_tl_n[w] = i + 1;
    }
  }
}
// called at the top of every simulation by every wave
__device__ __forceinline__ void st_sim(int sim) {
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    const bool on = blockIdx.x == MUZ_TL_WG && sim == MUZ_TL_SIM;
    const int i = tl_idx()[w];
    if (i > 0 && i + 1 < kTlMax) {   // end of the recorded simulation: shader clock and 100 MHz clock
      g_tl[w][i] = (__builtin_amdgcn_s_memtime() << 8) | (unsigned)(ST_N - 1);
      g_tl[w][i + 1] = (__builtin_amdgcn_s_memrealtime() << 8) | (unsigned)(ST_N - 2);
      g_tl_n[w] = i + 2;
    }
    tl_idx()[w] = on ? 0 : -1;
    if (on) {
      g_tl[w][0] = (__builtin_amdgcn_s_memrealtime() << 8) | (unsigned)(ST_N - 2);
      tl_idx()[w] = 1;
    }
  }
  ST(ST_N - 1);
}
__device__ __forceinline__ void st_end() {}
__device__ __forceinline__ void st_count(int) {}
#define SYNC()         \
  do {                 \
    ST(ST_OTHER);      \
    __syncthreads();   \
    ST(ST_BAR);        \
  } while (0)
#else
__device__ __forceinline__ void st_sim(int) {}
__device__ __forceinline__ void st_begin() {}
__device__ __forceinline__ void ST(int) {}
__device__ __forceinline__ void st_end() {}
__device__ __forceinline__ void st_count(int) {}
#define SYNC() __syncthreads()
#endif

// 16-column MFMA tiles per wave for a layer of N outputs (waves split N)
constexpr int nt_for(int N) { return (N + 16 * kWaves - 1) / (16 * kWaves); }
constexpr int NT64 = nt_for(64), NT128 = nt_for(128), NT256 = nt_for(256), NT384 = nt_for(384),
              NT512 = nt_for(512), NTA = nt_for(24);

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- cross-lane helpers on the DPP / permlane network instead of ds_bpermute (which goes through the
// LDS crossbar) ---------------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ unsigned as_u(T v) {
  return __builtin_bit_cast(unsigned, v);
}
template <class T>
__device__ __forceinline__ T from_u(unsigned u) {
  return __builtin_bit_cast(T, u);
}
template <int CTRL, class T>
__device__ __forceinline__ T dpp(T v) {
  return from_u<T>((unsigned)__builtin_amdgcn_update_dpp(0, (int)as_u(v), CTRL, 0xF, 0xF, false));
}
// (DPP_WAVE_SHL1: lane i reads lane i + 1 across the whole wave; a GFX9 DPP control)
enum { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140, DPP_WAVE_SHL1 = 0x130 };
template <class T>
struct LoHi {
  T lo, hi;
};
// {value of the lower 16-lane row, value of the upper one} of each 32-lane group, in every lane.
// (The two results are copied to plain scalars before the bit cast: bit-casting the vector element
// directly loses the second result in this compiler.)
template <class T>
__device__ __forceinline__ LoHi<T> swap16(T v) {
  const auto p = __builtin_amdgcn_permlane16_swap(as_u(v), as_u(v), false, false);
  const unsigned lo = p[0], hi = p[1];
  return {from_u<T>(lo), from_u<T>(hi)};
}
template <class T>
__device__ __forceinline__ LoHi<T> swap32(T v) {
  const auto p = __builtin_amdgcn_permlane32_swap(as_u(v), as_u(v), false, false);
  const unsigned lo = p[0], hi = p[1];
  return {from_u<T>(lo), from_u<T>(hi)};
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
#ifdef MUZ_EXPT_NOMFMA   // timing experiment only (wrong results): one VALU fma instead of each MFMA
  c[0] = fmaf(a, b, c[0]);
  return c;
#else
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
#endif
}

// acc[t] += A[16 rows][K] @ Wgroup[K][NT*16]  (KB = K/16 k-blocks; Wg = packed weights of this group).
// b0 / b1 hold k-blocks 0 and 1 on entry.  Weights for k-blocks kb+1 and kb+2 are in flight while kb is
// multiplied (3-deep register ring, written as a 3-way unrolled loop so every index is static).
// Tree traffic (node embeddings, children arrays): plain loads / stores.  Non-temporal hints (to keep the
// 3.8 MB of weights in each XCD's 4 MB L2) measured no gain on MI355X: the weights stay resident anyway.
template <class P, class V>
__device__ __forceinline__ void tree_st(P* p, V v) {
  *p = v;
}
template <class P>
__device__ __forceinline__ P tree_ld(const P* p) {
  return *p;
}

#ifndef MUZ_RING_DEPTH
#define MUZ_RING_DEPTH 2   // k-blocks of weights in flight ahead of the one being multiplied (2 or 3)
#endif
// 2: each output tile accumulates into two independent MFMA chains (even / odd k-steps, added at the end), so one
// wave alone -- its SIMD partner waiting at a barrier -- can issue back to back; 1: one chain per tile
#ifndef MUZ_ACC_CHAINS
#define MUZ_ACC_CHAINS 1
#endif

template <int NT, bool AG>
__device__ __forceinline__ void mfma_ring_impl(const float* __restrict__ Wg, int KB, const float* A, int lda,
                                               f32x4 (&acc)[NT], f32x4 (&b0)[NT], f32x4 (&b1)[NT]) {
  const int lane = tid() & 63;
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(Wg)) + lane * NT;
  const int wstep = 64 * NT;   // f32x4 per k-block
  const float* ap = A + r * lda + 4 * g;
  auto lda4 = [&](int kb) -> f32x4 {
    if constexpr (AG) return *gp(reinterpret_cast<const f32x4*>(ap + kb * 16));
    else return *reinterpret_cast<const f32x4*>(ap + kb * 16);
  };
  constexpr int D = MUZ_RING_DEPTH;
  f32x4 accb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) accb[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 a0 = lda4(0), a1 = a0;
  // step kb: issue k-block kb+D into `nxt` (the buffer consumed at step kb-1), read A of kb+1 from LDS,
  // multiply `cur` (= kb) with A of kb
  auto step = [&](int kb, const f32x4 (&cur)[NT], f32x4 (&nxt)[NT], const f32x4& acur, f32x4& anxt) {
#ifndef MUZ_EXPT_NOLOAD   // timing experiment only (wrong results): no weight stream inside the loop
    if (kb + D < KB) {
#pragma unroll
      for (int t = 0; t < NT; ++t) nxt[t] = wp[(kb + D) * wstep + t];
    }
#endif
    // Pin the issue point: without this the machine scheduler sinks each weight load next to its
    // first MFMA (one step of cover instead of D) once the loop is fully unrolled.
    __builtin_amdgcn_sched_barrier(0);
    if (kb + 1 < KB) anxt = lda4(kb + 1);
    const f32x4 a = acur;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) {   // D = W^T A^T
        if (MUZ_ACC_CHAINS == 2 && (j & 1)) accb[t] = mfma4(cur[t][j], a[j], accb[t]);
        else acc[t] = mfma4(cur[t][j], a[j], acc[t]);
      }
  };
  int kb = 0;
  if constexpr (D == 2) {
    f32x4 b2[NT];
    for (; kb + 3 <= KB; kb += 3) {
      step(kb, b0, b2, a0, a1);
      step(kb + 1, b1, b0, a1, a0);
      step(kb + 2, b2, b1, a0, a1);
      a0 = a1;
    }
    if (kb < KB) step(kb, b0, b2, a0, a1);
    if (kb + 1 < KB) step(kb + 1, b1, b0, a1, a0);
  } else {
    f32x4 b2[NT], b3[NT];
    if (KB > 2) {
#pragma unroll
      for (int t = 0; t < NT; ++t) b2[t] = wp[2 * wstep + t];
    }
    for (; kb + 4 <= KB; kb += 4) {
      step(kb, b0, b3, a0, a1);
      step(kb + 1, b1, b0, a1, a0);
      step(kb + 2, b2, b1, a0, a1);
      step(kb + 3, b3, b2, a1, a0);
    }
    if (kb < KB) step(kb, b0, b3, a0, a1);
    if (kb + 1 < KB) step(kb + 1, b1, b0, a1, a0);
    if (kb + 2 < KB) step(kb + 2, b2, b1, a0, a1);
  }
  if constexpr (MUZ_ACC_CHAINS == 2) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] += accb[t];
  }
}

template <int NT>
__device__ __forceinline__ void mfma_ring(const float* __restrict__ Wg, int KB, const float* A, int lda,
                                          f32x4 (&acc)[NT], f32x4 (&b0)[NT], f32x4 (&b1)[NT], bool a_global) {
  if (a_global)
    mfma_ring_impl<NT, true>(Wg, KB, A, lda, acc, b0, b1);
  else
    mfma_ring_impl<NT, false>(Wg, KB, A, lda, acc, b0, b1);
}

template <int NT>
__device__ __forceinline__ void mfma_rows16(const float* __restrict__ Wg, int KB, const float* A, int lda,
                                            f32x4 (&acc)[NT]) {
  const int lane = tid() & 63;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(Wg)) + lane * NT;
  f32x4 b0[NT], b1[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    b0[t] = wp[t];
    b1[t] = KB > 1 ? wp[64 * NT + t] : b0[t];
  }
  mfma_ring_impl<NT, false>(Wg, KB, A, lda, acc, b0, b1);
}

// ---- cross-layer weight prefetch ----------------------------------------------------------------
// Every dense layer issues the first two k-blocks of the NEXT layer's weights for this wave before its
// epilogue, so the loads fly across the epilogue, the barrier and the LayerNorm pass in between.
constexpr int kPfMax = NT384;
struct Pf {
  f32x4 v0[kPfMax], v1[kPfMax];
};

__device__ __forceinline__ const float* wave_group(const AS4 muz_dense& L, int KB, int NT) {
  return L.w + (size_t)(tid() >> 6) * KB * 64 * NT * 4;
}

template <int NT>
__device__ __forceinline__ void pf_issue(Pf& pf, const AS4 muz_dense* L, int K, int N) {
  static_assert(NT <= kPfMax, "prefetch buffer too small");
  if (!L) return;
  const int KB = (K + 15) >> 4;
  if ((tid() >> 6) * NT * 16 >= N) return;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(wave_group(*L, KB, NT))) + (tid() & 63) * NT;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    pf.v0[t] = wp[t];
    if (KB > 1) pf.v1[t] = wp[64 * NT + t];
  }
}

// Dense layer over the tile: out[16][N] = A @ W + b, waves split N (NT tiles of 16 columns each).
// `pf` holds this layer's first k-blocks on entry and the next layer's (Ln: K=Kn, N=Nn, NTN tiles)
// on exit.  A may live in LDS or global memory.  Caller synchronises before/after.
// split-K prefetch of a <= 32-column layer (logits16_splitk): wave w takes k-block w of column tiles 0 and 1
__device__ __forceinline__ void pf_issue_splitk(Pf& pf, const AS4 muz_dense* L, int K) {
  const int KB = (K + 15) >> 4, w = tid() >> 6;
  if (w >= KB) return;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(L->w)) + (tid() & 63);
  pf.v0[0] = wp[(0 * KB + w) * 64];   // packed [group][kb][lane][t = 0][4], groups = 16-column tiles
  pf.v1[0] = wp[(1 * KB + w) * 64];
}

template <int NT, int NTN>
__device__ __forceinline__ void dense16(const AS4 muz_dense& L, int K, int N, const float* A, int lda, float* out,
                                        int ldo, Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn,
                                        bool a_global = false, bool next_splitk = false) {
  const int lane = tid() & 63, wv = tid() >> 6;
  const int KB = (K + 15) >> 4;
  const int col0 = wv * NT * 16;
  auto pf_next = [&]() {
    if (next_splitk) pf_issue_splitk(pf, Ln, Kn);
    else pf_issue<NTN>(pf, Ln, Kn, Nn);
  };
  if (col0 >= N) {
    pf_next();
    return;
  }
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* bias4 = gp(reinterpret_cast<const f32x4*>(L.b));
  f32x4 acc[NT], b0[NT], b1[NT], bb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = col0 + t * 16 + 4 * g;
    bb[t] = col < N ? bias4[col >> 2] : f32x4{0.f, 0.f, 0.f, 0.f};   // lands under the MFMA loop
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    b0[t] = pf.v0[t];
    b1[t] = pf.v1[t];
  }
  ST(ST_DENTRY);
  mfma_ring<NT>(wave_group(L, KB, NT), KB, A, lda, acc, b0, b1, a_global);
  ST(ST_MFMA);
  pf_next();
  // The MFMA computes out^T (weights as the A operand), so lane (r, g) holds 4 CONSECUTIVE output
  // columns of row r: one 16-byte bias load and one ds_write_b128 per tile.
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = col0 + t * 16 + 4 * g;
    if (col < N) *reinterpret_cast<f32x4*>(out + r * ldo + col) = acc[t] + bb[t];
  }
  ST(ST_EPI);
}

// ---- row-wise ops: thread t -> row t/32, lane-in-row t%32 (half a wave per row) ---------------------
__device__ __forceinline__ int trow() { return tid() / kRowLanes; }
__device__ __forceinline__ int tsub() { return tid() % kRowLanes; }
// Row reductions on the DPP / permlane network (helpers above): xor-1 and xor-2 as quad_perm, then
// half-row and row mirrors, then a permlane swap across the two 16-lane rows of a 32-lane row (and
// across wave halves for 64-lane rows).  Every lane of a row ends with the same bits: each step
// combines a commutative pair in both lanes.
template <class T, class F>
__device__ __forceinline__ T row_reduce(T v, F f) {
  static_assert(kRowLanes == 16 || kRowLanes == 32 || kRowLanes == 64, "row width");
  v = f(v, dpp<DPP_XOR1>(v));
  v = f(v, dpp<DPP_XOR2>(v));
  v = f(v, dpp<DPP_HALF_MIRROR>(v));
  v = f(v, dpp<DPP_MIRROR>(v));
  if constexpr (kRowLanes >= 32) {
    const LoHi<T> p = swap16(v);
    v = f(p.lo, p.hi);
  }
  if constexpr (kRowLanes == 64) {
    const LoHi<T> p = swap32(v);
    v = f(p.lo, p.hi);
  }
  return v;
}
__device__ __forceinline__ float row_sum(float v) {
  return row_reduce(v, [](float x, float y) { return x + y; });
}
__device__ __forceinline__ float row_max(float v) {
  return row_reduce(v, [](float x, float y) { return fmaxf(x, y); });
}
__device__ __forceinline__ float row_min(float v) {
  return row_reduce(v, [](float x, float y) { return fminf(x, y); });
}
__device__ __forceinline__ int row_isum(int v) {
  return row_reduce(v, [](int x, int y) { return x + y; });
}
__device__ __forceinline__ int row_imax(int v) {
  return row_reduce(v, [](int x, int y) { return max(x, y); });
}

// Reciprocals of the networks' row ops (LayerNorm's 1 / sqrt(var + eps), min-max's 1 / (max - min + 1e-8), the
// reward / discount supports' 1 / sum(exp)): the hardware v_rsq_f32 / v_rcp_f32 (<= 1 ulp) instead of the correctly
// rounded IEEE sequences (a div_scale / div_fmas / div_fixup chain per divide): k_gumbel_search 2-3 % faster
// (profiles/r2_search_experiments.log), the networks still within 1e-5 of the fp32 oracle (tests/test_gpu_nets.py).
// The search's own tree arithmetic (mctx's completed Q, softmaxes, visit ratios) keeps IEEE division.
// MUZ_FAST_ROWOPS=0 builds the IEEE form.
#ifndef MUZ_FAST_ROWOPS
#define MUZ_FAST_ROWOPS 1
#endif
__device__ __forceinline__ float ln_rstd(float var_eps) {
#if MUZ_FAST_ROWOPS
  return __builtin_amdgcn_rsqf(var_eps);
#else
  return 1.0f / sqrtf(var_eps);
#endif
}
__device__ __forceinline__ float mm_scale(float x, float den) {
#if MUZ_FAST_ROWOPS
  return x * __builtin_amdgcn_rcpf(den);
#else
  return x / den;
#endif
}

enum LnMode { LN_PLAIN = 0, LN_RELU = 1, LN_RESID_RELU = 2 };

// Flax LayerNorm (eps 1e-6, fast variance) of in[16][N] -> out.
//   LN_PLAIN: out = y;  LN_RELU: out = relu(y);  LN_RESID_RELU: out = relu(out + y)  (ResBlock tail)
// Row-wise vector layout: lane `sub` of a row owns float4 columns sub*4 + i*4*kRowLanes.
template <int N>
struct RowVec {
  static constexpr int V = (N >= 4 * kRowLanes) ? N / (4 * kRowLanes) : 1;
  static __device__ __forceinline__ bool active(int sub) { return N >= 4 * kRowLanes || sub * 4 < N; }
  static __device__ __forceinline__ int col(int sub, int i) { return sub * 4 + i * 4 * kRowLanes; }
};

__device__ __forceinline__ f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void sts4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ f32x4 relu4(f32x4 v) {
  return f32x4{fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
}

// LayerNorm parameters of this lane's columns, loaded early (before the preceding dense layer's MFMA
// loop) so their L2 latency hides under it.
template <int N>
struct LnP {
  f32x4 sc[RowVec<N>::V], sh[RowVec<N>::V];
};
template <int N>
__device__ __forceinline__ LnP<N> ln_load(const AS4 muz_ln& P) {
  using RV = RowVec<N>;
  LnP<N> p;
  const int sub = tsub();
  const AS1 f32x4* scale = gp(reinterpret_cast<const f32x4*>(P.scale));
  const AS1 f32x4* shift = gp(reinterpret_cast<const f32x4*>(P.bias));
  if (RV::active(sub)) {
#pragma unroll
    for (int i = 0; i < RV::V; ++i) {
      p.sc[i] = scale[RV::col(sub, i) >> 2];
      p.sh[i] = shift[RV::col(sub, i) >> 2];
    }
  }
  return p;
}

template <int N, int MODE>
__device__ __forceinline__ void ln16(const float* in, int ldi, float* out, int ldo, const LnP<N>& p) {
  using RV = RowVec<N>;
  const int row = trow(), sub = tsub();
  const bool act = RV::active(sub);
  f32x4 v[RV::V];
  float s = 0.f, s2 = 0.f;
  if (act) {
#pragma unroll
    for (int i = 0; i < RV::V; ++i) {
      v[i] = lds4(in + row * ldi + RV::col(sub, i));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s += v[i][q];
        s2 = fmaf(v[i][q], v[i][q], s2);
      }
    }
  }
  s = row_sum(s);
  s2 = row_sum(s2);
  const float mean = s / (float)N;
  const float mean2 = s2 / (float)N;
  const float var = fmaxf(0.f, fmaf(-mean, mean, mean2));
  const float inv = ln_rstd(var + 1e-6f);
  if (act) {
#pragma unroll
    for (int i = 0; i < RV::V; ++i) {
      const int c = RV::col(sub, i);
      f32x4 y;
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = fmaf(v[i][q] - mean, inv * p.sc[i][q], p.sh[i][q]);
      if (MODE == LN_RELU) y = relu4(y);
      if (MODE == LN_RESID_RELU) y = relu4(lds4(out + row * ldo + c) + y);
      sts4(out + row * ldo + c, y);
    }
  }
  ST(ST_ROW);
}

template <int N, int MODE>
__device__ __forceinline__ void ln16(const float* in, int ldi, float* out, int ldo, const AS4 muz_ln& P) {
  ln16<N, MODE>(in, ldi, out, ldo, ln_load<N>(P));
}

// x <- (x - min) / (max - min + 1e-8) per row of 256 (Repr2 139-140, Dyn4 435-437).
__device__ __forceinline__ void minmax16(float* buf, int ld) {
  using RV = RowVec<LAT>;
  const int row = trow(), sub = tsub();
  f32x4 v[RV::V];
  float lo = INFINITY, hi = -INFINITY;
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    v[i] = lds4(buf + row * ld + RV::col(sub, i));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      lo = fminf(lo, v[i][q]);
      hi = fmaxf(hi, v[i][q]);
    }
  }
  lo = row_min(lo);
  hi = row_max(hi);
  const float den = hi - lo + 1e-8f;
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    f32x4 y;
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = mm_scale(v[i][q] - lo, den);
    sts4(buf + row * ld + RV::col(sub, i), y);
  }
}

// x <- minmax(x + skip) per row of 256: Dyn4's `latent + Dense_5(x)` (455) fused into the min-max pass.
// With `ln` (fused Pred4 head, search kernels): also stores the latent row to `emb` (the new node's embedding
// in the tree, when non-null) and PredictionNetwork4's LayerNorm_0 of it to `lnout`, so pred16 can start with
// its first ResBlock (same arithmetic, in the same order, as ln16<LAT, LN_PLAIN>).
__device__ __forceinline__ void skip_minmax16(float* buf, const float* skip, int ld, const LnP<LAT>* ln = nullptr,
                                              AS1 float* emb = nullptr, float* lnout = nullptr, float* dst = nullptr) {
  using RV = RowVec<LAT>;
  const int row = trow(), sub = tsub();
  f32x4 v[RV::V];
  float lo = INFINITY, hi = -INFINITY;
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    v[i] = lds4(skip + row * ld + RV::col(sub, i)) + lds4(buf + row * ld + RV::col(sub, i));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      lo = fminf(lo, v[i][q]);
      hi = fmaxf(hi, v[i][q]);
    }
  }
  lo = row_min(lo);
  hi = row_max(hi);
  const float den = hi - lo + 1e-8f;
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    f32x4 y;
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = mm_scale(v[i][q] - lo, den);
    sts4((dst ? dst : buf) + row * ld + RV::col(sub, i), y);   // (each lane reads its own skip / buf first)
    v[i] = y;
  }
  if (!ln) return;
  if (emb) {
#pragma unroll
    for (int i = 0; i < RV::V; ++i) tree_st(reinterpret_cast<AS1 f32x4*>(emb + RV::col(sub, i)), v[i]);
  }
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < RV::V; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s += v[i][q];
      s2 = fmaf(v[i][q], v[i][q], s2);
    }
  s = row_sum(s);
  s2 = row_sum(s2);
  const float mean = s / (float)LAT;
  const float mean2 = s2 / (float)LAT;
  const float var = fmaxf(0.f, fmaf(-mean, mean, mean2));
  const float inv = ln_rstd(var + 1e-6f);
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    f32x4 y;
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = fmaf(v[i][q] - mean, inv * ln->sc[i][q], ln->sh[i][q]);
    sts4(lnout + row * ld + RV::col(sub, i), y);
  }
}

__device__ __forceinline__ void relu16(float* buf, int ld, int col0, int n) {
  const int row = trow(), sub = tsub();
  for (int c = sub * 4; c < n; c += 4 * kRowLanes) sts4(buf + row * ld + col0 + c, relu4(lds4(buf + row * ld + col0 + c)));
}

// Policy logits (Dense_2: K = 128 -> A <= 32) split over the k dimension instead of the columns: wave w multiplies
// k-block w of both 16-column tiles (8 MFMAs, operands from pf_issue_splitk) and leaves its partial products in
// part[w][16][32]; logits16_splitk_sum adds the K / 16 partials and the bias per (row, column) after the next
// barrier.  The column split kept 6 of the 8 waves idle behind a 32-MFMA chain on two of them.
template <int NTN>
__device__ __forceinline__ void logits16_splitk(int K, const float* A, int lda, float* part, Pf& pf,
                                                const AS4 muz_dense* Ln, int Kn, int Nn) {
  const int lane = tid() & 63, w = tid() >> 6;
  const int KB = (K + 15) >> 4;
  if (w >= KB) {
    pf_issue<NTN>(pf, Ln, Kn, Nn);
    return;
  }
  const int r = lane & 15, g = lane >> 4;
  const f32x4 a = *reinterpret_cast<const f32x4*>(A + r * lda + w * 16 + 4 * g);
  const f32x4 b0 = pf.v0[0], b1 = pf.v1[0];
  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc0 = mfma4(b0[j], a[j], acc0);
    acc1 = mfma4(b1[j], a[j], acc1);
  }
  pf_issue<NTN>(pf, Ln, Kn, Nn);
  float* pw = part + (w * 16 + r) * 32 + 4 * g;
  *reinterpret_cast<f32x4*>(pw) = acc0;
  *reinterpret_cast<f32x4*>(pw + 16) = acc1;
}
// logit (row trow(), column tsub() < N) = bias + sum of the K / 16 partials (k-block order); this lane only
__device__ __forceinline__ float logits16_splitk_sum(const AS4 muz_dense& L, int K, const float* part) {
  const int KB = (K + 15) >> 4, row = trow(), c = tsub();
  float s = part[row * 32 + c];
  for (int w = 1; w < KB; ++w) s += part[(w * 16 + row) * 32 + c];
  return s + gp(L.b)[c];
}

// ---- LDS arena of a 16-row tile ---------------------------------------------------------------------
// Row strides (floats): +8 keeps every row 16-byte aligned and makes the MFMA loops' A-fragment
// ds_read_b128 (lane (r, g) -> row r, dword 4g) conflict-free.  With +4 each of those reads cost 4 bank-conflict
// cycles -- all of the search kernel's SQ_LDS_BANK_CONFLICT (profiles/r2_lds_conflicts.log) -- without slowing
// the loop (the read is issued a k-block ahead; profiles/r2_loop_bench.log).
constexpr int kLdPad = 8;
constexpr int LD = LAT + kLdPad;     // row stride of 256-wide buffers
constexpr int LDW = 512 + kLdPad;    // wide buffer (FiLM scale|shift 512, pred heads 384, concat 320)
constexpr int LDE = 64 + kLdPad;     // small buffer (action embed, global features)
constexpr int kLnPartFloats = kRows * kWaves * 2;   // dense_ln16's per-wave LayerNorm partial sums [16][waves][2]
constexpr int kArenaFloats = 4 * kRows * LD + kRows * LDW + kRows * LDE + 4 * kRows + kLnPartFloats;

struct Arena {
  float* L;   // latent input (parent embedding)           [16][LD]
  float* X;   // working activation                        [16][LD]
  float* T;   // scratch / next latent                     [16][LD]
  float* U;   // scratch / pred heads                      [16][LD]
  float* W;   // wide scratch                              [16][LDW]
  float* E;   // small scratch                             [16][LDE]
  float* v0;  // per-row scalars: value                    [16]
  float* v1;  // reward                                    [16]
  float* v2;  // discount                                  [16]
  float* v3;  // spare                                     [16]
  float* P;   // dense_ln16's LayerNorm partials            [16][kWaves][2]
  __device__ static Arena carve(float* base) {
    Arena a;
    a.L = base;
    a.X = a.L + kRows * LD;
    a.T = a.X + kRows * LD;
    a.U = a.T + kRows * LD;
    a.W = a.U + kRows * LD;
    a.E = a.W + kRows * LDW;
    a.v0 = a.E + kRows * LDE;
    a.v1 = a.v0 + kRows;
    a.v2 = a.v1 + kRows;
    a.v3 = a.v2 + kRows;
    a.P = a.v3 + kRows;
    return a;
  }
};

// ---- Dense + LayerNorm with the statistics in the dense epilogue ("Option A") -------------
// A 256-wide dense layer followed by its Flax LayerNorm (eps 1e-6, fast variance) [+ ReLU / residual ReLU]: each
// wave sums its 32 output columns of every row into (sum, sum of squares) partials right in the MFMA epilogue (lane
// (r, g) holds 4 consecutive columns of row r per tile: its 8 values in tile / column order, then the 4 g-lanes of
// the row pairwise over the permlane network), one barrier publishes the 8 waves' partials, and every lane
// normalises its own accumulator registers and stores the layer output once.  This replaces dense16's store, the
// barrier, ln16's row pass (reload, 32-lane reductions, store) and its barrier -- the row|row idle bucket of the
// search's timeline (profiles/r4_timeline.log).  The statistics' summation order differs from ln16's (a fixed
// order again), so every kernel built on these helpers -- search, root and recurrent alike -- rounds the same.
// MUZ_LN_EPILOGUE=0 builds the dense16 + ln16 pairs.  Caller synchronises before (A ready) and after (out ready).
#ifndef MUZ_LN_EPILOGUE
#define MUZ_LN_EPILOGUE 0   // 1: dense_ln16 (measured slower: profiles/r5_timeline.log)
#endif
template <int NT>
struct LnE {   // this lane's LayerNorm scale / bias columns in the MFMA output layout
  f32x4 sc[NT], sh[NT];
};
template <int NT>
__device__ __forceinline__ LnE<NT> lne_load(const AS4 muz_ln& P) {
  LnE<NT> p;
  const int lane = tid() & 63, col0 = (int)(tid() >> 6) * NT * 16 + 4 * (lane >> 4);
  const AS1 f32x4* sc = gp(reinterpret_cast<const f32x4*>(P.scale));
  const AS1 f32x4* sh = gp(reinterpret_cast<const f32x4*>(P.bias));
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    p.sc[t] = sc[(col0 + 16 * t) >> 2];
    p.sh[t] = sh[(col0 + 16 * t) >> 2];
  }
  return p;
}

template <int NT, int NTN, int MODE>
__device__ __forceinline__ void dense_ln16(const AS4 muz_dense& L, int K, const float* A, int lda, float* out, int ldo,
                                           Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn, const LnE<NT>& lp,
                                           float* part) {
  static_assert(NT * 16 * kWaves == LAT, "dense_ln16: the waves' columns cover exactly the 256 outputs");
  const int lane = tid() & 63, wv = tid() >> 6;
  const int KB = (K + 15) >> 4;
  const int col0 = wv * NT * 16;
  const int r = lane & 15, g = lane >> 4;
  const AS1 f32x4* bias4 = gp(reinterpret_cast<const f32x4*>(L.b));
  f32x4 acc[NT], b0[NT], b1[NT], bb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bb[t] = bias4[(col0 + t * 16 + 4 * g) >> 2];
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    b0[t] = pf.v0[t];
    b1[t] = pf.v1[t];
  }
  ST(ST_DENTRY);
  mfma_ring<NT>(wave_group(L, KB, NT), KB, A, lda, acc, b0, b1, false);
  ST(ST_MFMA);
  pf_issue<NTN>(pf, Ln, Kn, Nn);
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    acc[t] += bb[t];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s += acc[t][q];
      s2 = fmaf(acc[t][q], acc[t][q], s2);
    }
  }
  {   // the row's 4 g-lanes: (g0 + g1) + (g2 + g3)
    LoHi<float> p = swap16(s), p2 = swap16(s2);
    s = p.lo + p.hi;
    s2 = p2.lo + p2.hi;
    p = swap32(s);
    p2 = swap32(s2);
    s = p.lo + p.hi;
    s2 = p2.lo + p2.hi;
  }
  if (g == 0) {
    part[(r * kWaves + wv) * 2] = s;
    part[(r * kWaves + wv) * 2 + 1] = s2;
  }
  ST(ST_EPI);
  SYNC();
  float ps[kWaves], ps2[kWaves];
#pragma unroll
  for (int w = 0; w < kWaves; w += 2) {
    const f32x4 v = lds4(part + (r * kWaves + w) * 2);
    ps[w] = v[0];
    ps2[w] = v[1];
    ps[w + 1] = v[2];
    ps2[w + 1] = v[3];
  }
#pragma unroll
  for (int h = 1; h < kWaves; h *= 2)   // balanced tree over the waves in wave order
#pragma unroll
    for (int w = 0; w < kWaves; w += 2 * h) {
      ps[w] += ps[w + h];
      ps2[w] += ps2[w + h];
    }
  const float mean = ps[0] / (float)LAT;
  const float mean2 = ps2[0] / (float)LAT;
  const float var = fmaxf(0.f, fmaf(-mean, mean, mean2));
  const float inv = ln_rstd(var + 1e-6f);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = col0 + t * 16 + 4 * g;
    f32x4 y;
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = fmaf(acc[t][q] - mean, inv * lp.sc[t][q], lp.sh[t][q]);
    if (MODE == LN_RELU) y = relu4(y);
    if (MODE == LN_RESID_RELU) y = relu4(lds4(out + r * ldo + c) + y);
    sts4(out + r * ldo + c, y);
  }
  ST(ST_ROW);
}

// ResBlock (muzero_deterministic_madn.py:12-24): X <- relu(X + LN1(D1(relu(LN0(D0(X))))))
// pf: rb.d0 on entry, (Ln: Kn x Nn, NTN tiles) on exit.  `part`: the arena's LayerNorm partials (MUZ_LN_EPILOGUE).
template <int NTN>
__device__ __forceinline__ void resblock16(const AS4 muz_resblock& R, float* X, float* T, float* U, Pf& pf,
                                           const AS4 muz_dense* Ln, int Kn, int Nn, float* part) {
  if constexpr (MUZ_LN_EPILOGUE != 0) {
    const LnE<NT256> q0 = lne_load<NT256>(R.ln0);
    dense_ln16<NT256, NT256, LN_RELU>(R.d0, LAT, X, LD, T, LD, pf, &R.d1, LAT, LAT, q0, part);
    SYNC();
    const LnE<NT256> q1 = lne_load<NT256>(R.ln1);
    dense_ln16<NT256, NTN, LN_RESID_RELU>(R.d1, LAT, T, LD, X, LD, pf, Ln, Kn, Nn, q1, part);
    SYNC();
    return;
  }
  (void)part;
  const LnP<LAT> p0 = ln_load<LAT>(R.ln0);
  dense16<NT256, NT256>(R.d0, LAT, LAT, X, LD, T, LD, pf, &R.d1, LAT, LAT);
  SYNC();
  ln16<LAT, LN_RELU>(T, LD, T, LD, p0);
  SYNC();
  const LnP<LAT> p1 = ln_load<LAT>(R.ln1);
  dense16<NT256, NTN>(R.d1, LAT, LAT, T, LD, U, LD, pf, Ln, Kn, Nn);
  SYNC();
  ln16<LAT, LN_RESID_RELU>(U, LD, X, LD, p1);
  SYNC();
}

// 64-input heads: weights of this lane's inputs k = sub + i*kRowLanes, loaded early.
// K-input heads (K = 32 or 64) with up to 3 outputs: weights of this lane's inputs
// k = sub + i*kRowLanes, loaded early.
template <int K>
struct HeadK {
  static constexpr int kPer = (K + kRowLanes - 1) / kRowLanes;
  float w[3][kPer];
  float b[3];
};
using HeadW = HeadK<64>;
template <int K = 64>
__device__ __forceinline__ HeadK<K> head_load(const AS4 muz_dense& H, int ncol) {
  HeadK<K> h;
  const AS1 float* w = gp(H.w);
  const AS1 float* b = gp(H.b);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    h.b[j] = j < ncol ? b[j] : 0.f;
#pragma unroll
    for (int i = 0; i < HeadK<K>::kPer; ++i) {
      const int k = tsub() + i * kRowLanes;
      h.w[j][i] = (j < ncol && k < K) ? w[k * ncol + j] : 0.f;
    }
  }
  return h;
}
// sum_k relu(in[k] + add[i]) * w[k] (+ b): a head whose hidden layer's one-hot rows and ReLU are applied
// as the inputs are read (add[i] = the one-hot weight row at this lane's inputs, 0 without an action).
template <int K>
__device__ __forceinline__ float head_dot_relu(const float* in, int ld, const float (&add)[HeadK<K>::kPer],
                                               const HeadK<K>& h, int j) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < HeadK<K>::kPer; ++i) {
    const int k = tsub() + i * kRowLanes;
    if (k < K) s = fmaf(fmaxf(in[trow() * ld + k] + add[i], 0.f), h.w[j][i], s);
  }
  return row_sum(s) + h.b[j];
}
template <int K>
__device__ __forceinline__ float head_dot(const float* in, int ld, const HeadK<K>& h, int j) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < HeadK<K>::kPer; ++i) {
    const int k = tsub() + i * kRowLanes;
    if (k < K) s = fmaf(in[trow() * ld + k], h.w[j][i], s);
  }
  return row_sum(s) + h.b[j];
}

__device__ __forceinline__ float softmax3_support(float l0, float l1, float l2) {
  // sum(softmax(l) * [-1, 0, 1])  (recurrent_inference_fn 648-653)
  const float m = fmaxf(fmaxf(l0, l1), l2);
  const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = expf(l2 - m);
  const float z = e0 + e1 + e2;
  return mm_scale(e0, z) * -1.0f + mm_scale(e1, z) * 0.0f + mm_scale(e2, z) * 1.0f;
}

// PredictionNetwork4 (muzero_deterministic_madn.py:549-583) on the latent in `lat` ([16][LD]).
// Leaves policy logits in a.U[:, 0:A] and tanh value in a.v0.  Clobbers X, T, U, W.
// pf: rb[0].d0 on entry, (Ln, NTN tiles) on exit.
// LN0_DONE: the caller already left LayerNorm_0(lat) in a.X (dyn16<.., true>), so the pass and its barrier
// are skipped.
// LATE_HEADS (search kernel, with dyn16<.., true, true>): Dyn4's reward / discount trunk -- Dense_6 | Dense_7 over
// the new latent (left in a.L by dyn16) and the two 64 -> 3 support heads -- runs here, its MFMA loop in the same
// barrier interval as policy Dense_1 / value Dense_4 and its head dots in the following row pass, instead of a
// dense phase and a row phase of its own.  `D` / `ar`: Dyn4's weights and the row's action.  Leaves the reward /
// discount support values in a.v1 / a.v2 like dyn16.
// SPLITK_LOGITS: the policy logits by logits16_splitk (partials in a.W, summed per lane at the end into a.U; a
// caller reads a.U[row][c] only from lane (row, c), as all of them do).
// NO_LOGITS (DOG, A = 806 does not fit a [16][LD] buffer): stop before the policy logits and leave the policy
// hidden layer in a.T; P.d2 is then the first logits chunk (NTL tiles per wave, 256 columns), whose first k-blocks
// pf holds on exit (dog_logits16 runs the chunks).  Ln / Kn / Nn are unused then.
template <int NTN, bool LN0_DONE = false, bool LATE_HEADS = false, bool SPLITK_LOGITS = false, int NTL = NTA,
          bool NO_LOGITS = false>
__device__ __forceinline__ void pred16(const AS4 muz_pred_w& P, int A, const float* lat, const Arena& a, Pf& pf,
                                       const AS4 muz_dense* Ln, int Kn, int Nn, const AS4 muz_dyn_w* D = nullptr,
                                       int ar = 0) {
  static_assert(!(NO_LOGITS && SPLITK_LOGITS), "split-K logits need the whole logits layer");
  const int nl = NO_LOGITS ? 256 : A;   // columns of the layer after value Dense_4 (its prefetch)
  if constexpr (!LN0_DONE) {
    ln16<LAT, LN_PLAIN>(lat, LD, a.X, LD, P.ln0);
    SYNC();
  }
  resblock16<NT256>(P.rb[0], a.X, a.T, a.U, pf, &P.rb[1].d0, LAT, LAT, a.P);
  resblock16<NT384>(P.rb[1], a.X, a.T, a.U, pf, &P.d03, LAT, 384, a.P);
  const LnP<LAT> p1 = ln_load<LAT>(P.ln1);
  const LnP<128> p3 = ln_load<128>(P.ln3);
  dense16<NT384, NT128>(P.d03, LAT, 384, a.X, LD, a.W, LDW, pf, &P.d1, LAT, 128);   // [policy Dense_0 | value Dense_3]
  SYNC();
  ln16<LAT, LN_RELU>(a.W, LDW, a.W, LDW, p1);
  ln16<128, LN_RELU>(a.W + 256, LDW, a.W + 256, LDW, p3);
  SYNC();
  const LnP<128> p2 = ln_load<128>(P.ln2);
  const HeadW hv = head_load(P.d5, 1);
  if constexpr (LATE_HEADS) {
    dense16<NT128, NT128>(P.d1, LAT, 128, a.W, LDW, a.T, LD, pf, &D->d67, LAT, 128);   // policy Dense_1
    // reward / discount heads and Dense_6 | Dense_7's one-hot rows at this lane's head inputs: issued here, they
    // land under the two MFMA loops below
    const HeadW hr = head_load(D->reward_head, 3);
    const HeadW hd = head_load(D->discount_head, 3);
    const bool oh = ar >= 0 && ar < A;
    float add_r[HeadW::kPer], add_d[HeadW::kPer];
    {
      const AS1 float* w67 = gp(D->d67_onehot) + (oh ? ar : 0) * 128;
#pragma unroll
      for (int i = 0; i < HeadW::kPer; ++i) {
        const int k = tsub() + i * kRowLanes;
        add_r[i] = (oh && k < 64) ? w67[k] : 0.f;
        add_d[i] = (oh && k < 64) ? w67[64 + k] : 0.f;
      }
    }
    dense16<NT128, NT64>(D->d67, LAT, 128, a.L, LD, a.U, LD, pf, &P.d4, 128, 64);   // [reward | discount] hidden
    dense16<NT64, NTL>(P.d4, 128, 64, a.W + 256, LDW, a.X, LD, pf, &P.d2, 128, nl, false,
                       SPLITK_LOGITS);                                              // value Dense_4 (X is free)
    SYNC();
    ln16<128, LN_RELU>(a.T, LD, a.T, LD, p2);
    relu16(a.X, LD, 0, 64);
    float rl[3], dl[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      rl[j] = head_dot_relu(a.U, LD, add_r, hr, j);
      dl[j] = head_dot_relu(a.U + 64, LD, add_d, hd, j);
    }
    if (tsub() == 0) {
      a.v1[trow()] = softmax3_support(rl[0], rl[1], rl[2]);
      a.v2[trow()] = softmax3_support(dl[0], dl[1], dl[2]);
    }
  } else {
    dense16<NT128, NT64>(P.d1, LAT, 128, a.W, LDW, a.T, LD, pf, &P.d4, 128, 64);     // policy Dense_1
    dense16<NT64, NTL>(P.d4, 128, 64, a.W + 256, LDW, a.X, LD, pf, &P.d2, 128, nl, false,
                       SPLITK_LOGITS);                                              // value Dense_4 (X is free)
    SYNC();
    ln16<128, LN_RELU>(a.T, LD, a.T, LD, p2);
    relu16(a.X, LD, 0, 64);
  }
  ST(ST_PASS);
  SYNC();
  if constexpr (NO_LOGITS) {
    // (the logits chunks follow in the caller; pf keeps chunk 0's k-blocks)
  } else if constexpr (SPLITK_LOGITS) {
    logits16_splitk<NTN>(128, a.T, LD, a.W, pf, Ln, Kn, Nn);                  // policy logits, split over k
  } else {
    dense16<NTA, NTN>(P.d2, 128, A, a.T, LD, a.U, LD, pf, Ln, Kn, Nn);         // policy logits
  }
  {
    const float v = head_dot(a.X, LD, hv, 0);
    if (tsub() == 0) a.v0[trow()] = tanhf(v);
  }
  ST(ST_PASS);
  SYNC();
  if constexpr (SPLITK_LOGITS) {
    if (tsub() < A) a.U[trow() * LD + tsub()] = logits16_splitk_sum(P.d2, 128, a.W);
  }
}

// RepresentationNetwork2's dense part on the tile (muzero_deterministic_madn.py:105-138; the DOG
// RepresentationNetwork, MuZero_DOG/muzero_dog.py:51-80, is the same): Dense_0 over the flattened conv maps of
// games g0.. (convout, global memory, rows padded to a multiple of 16), the global stream x[:, 6:, 0], the concat,
// 6 ResBlocks and Dense_4 into a.T -- the head (min-max / LayerNorm) is the caller's.  pf: on exit Ln's first
// k-blocks.  Ends without a barrier after Dense_4.
__device__ __forceinline__ bool gr_valid(int g, int n) { return g < n; }
template <int NTN, bool D0_DONE = false>
__device__ __forceinline__ void repr16(const AS4 muz_repr_w& R, const float* __restrict__ obs, int C,
                                       const float* __restrict__ convout, int g0, int n, const Arena& a, Pf& pf,
                                       const AS4 muz_dense* Ln, int Kn, int Nn) {
  const int row = trow(), sub = tsub();
  const int gr = g0 + row;
  const bool valid = gr < n;
  // global stream input: x[:, 6:, 0]
  const int Kg = C - 6;
  if (sub < 32) a.E[row * LDE + sub] = (valid && sub < Kg) ? obs[((size_t)gr * C + 6 + sub) * 56] : 0.f;
  // spatial: Dense_0 over the flattened conv maps (scratch rows padded to a multiple of 16; row stride
  // kConvRowFloats), or -- D0_DONE -- its output, computed by k_dense0 into the scratch row after the maps
  if constexpr (D0_DONE) {
    pf_issue<NT64>(pf, &R.d1, Kg, 64);
    const int rr = tid() >> 5, q = tid() & 31;   // 16 rows x 64 float4: 2 per thread
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c4 = q + 32 * i;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (gr_valid(g0 + rr, n)) {
        const AS1 f32x4* src = gp(reinterpret_cast<const f32x4*>(convout + (size_t)(g0 + rr) * kConvRowFloats +
                                                                 kConvMapFloats)) + c4;
        v = src[0];
#pragma unroll
        for (int s = 1; s < kD0KSplit; ++s) v = v + src[64 * s];   // k_dense0's partial planes, in plane order
        if (kD0KSplit > 1) v = v + gp(reinterpret_cast<const f32x4*>(R.d0.b))[c4];
      }
      *reinterpret_cast<f32x4*>(a.W + rr * LDW + 4 * c4) = v;
    }
  } else {
    pf_issue<NT256>(pf, &R.d0, kConvMapFloats, LAT);
    dense16<NT256, NT64>(R.d0, kConvMapFloats, LAT, convout + (size_t)g0 * kConvRowFloats, kConvRowFloats, a.W, LDW,
                         pf, &R.d1, Kg, 64, true);
  }
  __syncthreads();
  ln16<LAT, LN_RELU>(a.W, LDW, a.W, LDW, R.ln3);
  dense16<NT64, NT64>(R.d1, Kg, 64, a.E, LDE, a.X, LD, pf, &R.d2, 64, 64);
  __syncthreads();
  ln16<64, LN_RELU>(a.X, LD, a.X, LD, R.ln4);
  __syncthreads();
  dense16<NT64, NT256>(R.d2, 64, 64, a.X, LD, a.W + 256, LDW, pf, &R.d3, 320, LAT);
  __syncthreads();
  ln16<64, LN_RELU>(a.W + 256, LDW, a.W + 256, LDW, R.ln5);
  __syncthreads();
  dense16<NT256, NT256>(R.d3, 320, LAT, a.W, LDW, a.X, LD, pf, &R.rb[0].d0, LAT, LAT);
  __syncthreads();
  ln16<LAT, LN_RELU>(a.X, LD, a.X, LD, R.ln6);
  __syncthreads();
#pragma unroll 1
  for (int b = 0; b < 6; ++b)
    resblock16<NT256>(R.rb[b], a.X, a.T, a.U, pf, b < 5 ? &R.rb[b + 1].d0 : &R.d4, LAT, LAT, a.P);
  dense16<NT256, NTN>(R.d4, LAT, LAT, a.X, LD, a.T, LD, pf, Ln, Kn, Nn);
}

// Dyn4 inputs of this thread's row, loaded as soon as the parent node and action are known (end of the
// tree walk) so their latency hides under the selection barrier: the parent latent (RowVec<LAT> layout),
// the action's FiLM rows and LayerNorm_0's parameters.  FiLM scale | shift depend on the action only
// (Dense_1/2(relu(Dense_0(one_hot(a))))), so they come from the per-weight-set table dyn.film
// (muz_net_prepare); row A is the zero one-hot of an out-of-range action.
struct DynIn {
  f32x4 lat[RowVec<LAT>::V], sc[RowVec<LAT>::V], sh[RowVec<LAT>::V];
  LnP<LAT> ln0;
};
__device__ __forceinline__ DynIn dyn_load(const AS4 muz_dyn_w& D, int A, const AS1 float* lat, int action) {
  using RV = RowVec<LAT>;
  DynIn in;
  const int sub = tsub();
  const int fr = (action >= 0 && action < A) ? action : A;
  const AS1 f32x4* film = gp(reinterpret_cast<const f32x4*>(D.film)) + fr * (2 * LAT / 4);
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    const int c = RV::col(sub, i);
    in.lat[i] = lat ? tree_ld(reinterpret_cast<const AS1 f32x4*>(lat + c)) : f32x4{0.f, 0.f, 0.f, 0.f};
    in.sc[i] = film[c >> 2];
    in.sh[i] = film[(LAT + c) >> 2];
  }
  in.ln0 = ln_load<LAT>(D.ln0);
  return in;
}

// DynamicsNetwork4 (muzero_deterministic_madn.py:391-457) on the tile.  `in` = this thread's row inputs,
// `ar` = this row's action.  Out: next latent in a.T, reward / discount support values in a.v1 / a.v2.
// pf: d3 on entry, (Ln: Kn x Nn, NTN tiles) on exit.
// PRED_LN0: fuse the following pred16's LayerNorm_0 (params `pln0`) into the latent's min-max pass, store the
// latent to the tree at `emb` there (null: no store), and end without the final barrier; the caller then runs
// pred16<.., true>, whose first writes (ResBlock_0's Dense_0 into a.T) come after d67 has consumed a.T.
// LATE_HEADS (with PRED_LN0): stop after the min-max pass, which leaves the new latent in a.L (and a.T is free),
// and let pred16<.., true, true> run Dense_6 | Dense_7 and the reward / discount heads; ends with a barrier.
template <int NTN, bool PRED_LN0 = false, bool LATE_HEADS = false>
__device__ __forceinline__ void dyn16(const AS4 muz_dyn_w& D, int A, const DynIn& in, int ar, const Arena& a, Pf& pf,
                                      const AS4 muz_dense* Ln, int Kn, int Nn, const AS4 muz_ln* pln0 = nullptr,
                                      AS1 float* emb = nullptr) {
  static_assert(!LATE_HEADS || PRED_LN0, "late heads need the fused Pred4 LayerNorm_0");
  using RV = RowVec<LAT>;
  const int row = trow(), sub = tsub();
  const bool oh = ar >= 0 && ar < A;   // jax.nn.one_hot: out-of-range -> zero row
  // LayerNorm_0 of the latent + FiLM, in registers: X = LN0(L) * (1 + scale) + shift; L kept for the skip
  {
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < RV::V; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s += in.lat[i][q];
        s2 = fmaf(in.lat[i][q], in.lat[i][q], s2);
      }
    s = row_sum(s);
    s2 = row_sum(s2);
    const float mean = s / (float)LAT;
    const float mean2 = s2 / (float)LAT;
    const float inv = ln_rstd(fmaxf(0.f, fmaf(-mean, mean, mean2)) + 1e-6f);
#pragma unroll
    for (int i = 0; i < RV::V; ++i) {
      const int c = RV::col(sub, i);
      f32x4 x;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float y = fmaf(in.lat[i][q] - mean, inv * in.ln0.sc[i][q], in.ln0.sh[i][q]);
        x[q] = fmaf(y, 1.0f + in.sc[i][q], in.sh[i][q]);
      }
      sts4(a.X + row * LD + c, x);
      sts4(a.L + row * LD + c, in.lat[i]);
    }
    ST(ST_ROW);
  }
  SYNC();
  if constexpr (MUZ_LN_EPILOGUE != 0) {
    const LnE<NT256> q1 = lne_load<NT256>(D.ln1);
    dense_ln16<NT256, NT256, LN_RELU>(D.d3, LAT, a.X, LD, a.T, LD, pf, &D.d4, LAT, LAT, q1, a.P);
    SYNC();
    const LnE<NT256> q2 = lne_load<NT256>(D.ln2);
    dense_ln16<NT256, NT256, LN_RELU>(D.d4, LAT, a.T, LD, a.X, LD, pf, &D.rb[0].d0, LAT, LAT, q2, a.P);
    SYNC();
  } else {
    const LnP<LAT> p1 = ln_load<LAT>(D.ln1);
    dense16<NT256, NT256>(D.d3, LAT, LAT, a.X, LD, a.T, LD, pf, &D.d4, LAT, LAT);
    SYNC();
    ln16<LAT, LN_RELU>(a.T, LD, a.T, LD, p1);
    SYNC();
    const LnP<LAT> p2 = ln_load<LAT>(D.ln2);
    dense16<NT256, NT256>(D.d4, LAT, LAT, a.T, LD, a.X, LD, pf, &D.rb[0].d0, LAT, LAT);
    SYNC();
    ln16<LAT, LN_RELU>(a.X, LD, a.X, LD, p2);
    SYNC();
  }
  resblock16<NT256>(D.rb[0], a.X, a.T, a.U, pf, &D.rb[1].d0, LAT, LAT, a.P);
  resblock16<NT256>(D.rb[1], a.X, a.T, a.U, pf, &D.d5, LAT, LAT, a.P);
  if constexpr (LATE_HEADS) {
    dense16<NT256, NTN>(D.d5, LAT, LAT, a.X, LD, a.T, LD, pf, Ln, Kn, Nn);
    const LnP<LAT> pl = ln_load<LAT>(*pln0);
    SYNC();
    skip_minmax16(a.T, a.L, LD, &pl, emb, a.X, a.L);
    ST(ST_PASS);
    SYNC();
    return;
  }
  const HeadW hr = head_load(D.reward_head, 3);
  const HeadW hd = head_load(D.discount_head, 3);
  dense16<NT256, NT128>(D.d5, LAT, LAT, a.X, LD, a.T, LD, pf, &D.d67, LAT, 128);
  // Dense_6 | Dense_7's one-hot rows at this lane's head inputs (k = sub + i*kRowLanes), loaded early
  float add_r[HeadW::kPer], add_d[HeadW::kPer];
  {
    const AS1 float* w67 = gp(D.d67_onehot) + (oh ? ar : 0) * 128;
#pragma unroll
    for (int i = 0; i < HeadW::kPer; ++i) {
      const int k = sub + i * kRowLanes;
      add_r[i] = (oh && k < 64) ? w67[k] : 0.f;
      add_d[i] = (oh && k < 64) ? w67[64 + k] : 0.f;
    }
  }
  if constexpr (PRED_LN0) {
    const LnP<LAT> pl = ln_load<LAT>(*pln0);
    SYNC();
    skip_minmax16(a.T, a.L, LD, &pl, emb, a.X);
  } else {
    SYNC();
    skip_minmax16(a.T, a.L, LD);
  }
  ST(ST_PASS);
  SYNC();
  dense16<NT128, NTN>(D.d67, LAT, 128, a.T, LD, a.W, LDW, pf, Ln, Kn, Nn);   // [reward | discount] hidden
  SYNC();
  float rl[3], dl[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    rl[j] = head_dot_relu(a.W, LDW, add_r, hr, j);
    dl[j] = head_dot_relu(a.W + 64, LDW, add_d, hd, j);
  }
  if (sub == 0) {
    a.v1[row] = softmax3_support(rl[0], rl[1], rl[2]);
    a.v2[row] = softmax3_support(dl[0], dl[1], dl[2]);
  }
  ST(ST_PASS);
  if constexpr (!PRED_LN0) SYNC();
}

}  // namespace MUZ_NN_NS
}  // namespace muz
