// The unrolled dynamics chain of a learner step as ONE launch each way (learner._TrunkChain; reference
// train_with_reward.py:98-107, train_stochastic.py:95-121; the trunk is DynamicsNetwork4's FiLM trunk,
// muzero_deterministic_madn.py:391-457).  At batch 128 x 10 applications the per-layer form was ~150 forward and
// ~90 backward launches of a few microseconds each (library GEMMs at 128 rows, row kernels); here one workgroup
// carries 16 rows through every application, its activations in LDS, the weights streamed from L2 (all tiles
// read the same matrices), and writes exactly what the per-layer kernels saved for the backward (so the weight /
// LayerNorm gradients stay the grouped launches of learner.GradSink).
//
// Workgroup = 8 waves, 512 threads.  GEMM: wave w owns output columns 32 w .. + 31 (two 16-column tiles),
//   v_mfma_f32_16x16x4_f32 with the streamed matrix as the A operand: out[m][c] = sum_k in[m][k] Mt[c][k], Mt = W^T
//   forward (y = x W) and Mt = W backward (dx = dz W^T), so both directions are the same loop: lane (i, g) reads
//   Mt[32 w + 16 t + i][16 b + 4 g .. + 3] (one 16-byte load per tile and k-block from the packed copy that
//   muz_trunk_chain_pack makes per step, 1 KB contiguous per load instruction; 2 k-blocks ahead) and ends with
//   out[i][32 w + 16 t + 4 g .. + 3].  The next GEMM's first k-blocks are issued before the row phase between
//   two GEMMs, so their latency hides behind it.
// Rows: thread (row = tid / 32, sub = tid % 32) owns columns 8 sub .. + 7 of one row; row sums over the 32
//   lanes of a half-wave.  The row arithmetic is k_ln_fwd / k_ln_bwd / k_minmax_fwd / k_minmax_bwd's
//   (learner_ln.hip: Flax LayerNorm eps 1e-6 with the fast variance, min-max with the extremum gradient split
//   evenly over tied columns), compiled without fma contraction like them.
#include "launch.hpp"

namespace muz {
namespace chain {

typedef float f4 __attribute__((ext_vector_type(4)));
// k-blocks of weights in flight (+1 being multiplied); measured at batch 128 x 10 applications (fwd / bwd us,
// profiles/r4g_chain_bench.log): 2: 414 / 435, 3: 407 / 431, 4: 424 / 454, 8: 447 / 485
#ifndef MUZ_CHAIN_RING
#define MUZ_CHAIN_RING 3
#endif
// waves per workgroup: 8 (2 per SIMD, each owning two 16-column tiles) or 16 (4 per SIMD, one tile each)
#ifndef MUZ_CHAIN_WAVES
#define MUZ_CHAIN_WAVES 8
#endif
constexpr int NWAVE = MUZ_CHAIN_WAVES, NT = 16 / NWAVE, LNT = NT == 2 ? 1 : 0;
constexpr int N = 256, R = 16, LD = N + 4, NTH = 64 * NWAVE, KB = N / 16, D = MUZ_CHAIN_RING;
constexpr int TPR = NTH / R, E = N / TPR;   // row phases: threads per row, columns per thread
static_assert(NWAVE == 8 || NWAVE == 16, "8 or 16 waves");
constexpr int kLayers = 6;   // Dense + LayerNorm layers; weight layer 6 = the projection
// The per-layer vectors (LayerNorm scale / bias, Dense bias) staged in LDS once per launch, and the backward's saved
// values loaded a layer ahead: bit-identical, and measured neutral (forward 407 -> 402 us, backward 431 -> 434 us,
// profiles/r6l_chain_bench.log) -- the row phases were not waiting on those loads; the DPP row sums below were
// what paid.  Forward, per group: gamma[6], beta[6], bias[7], LayerNorm_0 scale, LayerNorm_0 bias; backward:
// gamma[6], LayerNorm_0 scale.
constexpr int kPf = 21 * N, kPfBeta = 6 * N, kPfBias = 12 * N, kPfL0g = 19 * N, kPfL0b = 20 * N;
constexpr int kPb = 7 * N, kPbL0g = 6 * N;

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Row reductions over the TPR lanes of a row.  MUZ_CHAIN_DPP (default): on the DPP / permlane network -- xor-1, xor-2
// (quad_perm), half-row and row mirrors, then v_permlane16_swap across the two 16-lane rows -- instead of a
// ds_bpermute butterfly through the LDS crossbar (5 dependent round trips per sum).  Every step combines a
// commutative pair in both lanes, so all lanes of a row end with the same bits (a different summation order from the
// butterfly's: not bit-identical to the round-5 kernels; the learner tests bound it).  Forward 402.8 -> 389.6 us,
// backward 434.6 -> 421.3 us; det step 1.585 -> 1.548 ms (profiles/r6m_chain_bench.log, r6m_steps.log).
#ifndef MUZ_CHAIN_DPP
#define MUZ_CHAIN_DPP 1
#endif
template <int CTRL>
__device__ __forceinline__ unsigned dppu(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <class T, class F>
__device__ __forceinline__ T row_reduce(T v, F f) {
  if constexpr (MUZ_CHAIN_DPP && TPR == 32) {
    auto step = [&](unsigned o) { v = f(v, __builtin_bit_cast(T, o)); };
    step(dppu<0xB1>(__builtin_bit_cast(unsigned, v)));    // xor 1
    step(dppu<0x4E>(__builtin_bit_cast(unsigned, v)));    // xor 2
    step(dppu<0x141>(__builtin_bit_cast(unsigned, v)));   // half-row mirror
    step(dppu<0x140>(__builtin_bit_cast(unsigned, v)));   // row mirror
    const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                    false, false);
    const unsigned lo = p[0], hi = p[1];
    return f(__builtin_bit_cast(T, lo), __builtin_bit_cast(T, hi));
  } else {
#pragma unroll
    for (int o = TPR / 2; o >= 1; o >>= 1) v = f(v, __shfl_xor(v, o, 64));
    return v;
  }
}

__device__ __forceinline__ float row_sum(float v) {
  return row_reduce(v, [](float x, float y) { return x + y; });
}

__device__ __forceinline__ int row_isum(int v) {
  return row_reduce(v, [](int x, int y) { return x + y; });
}

// the lowest column of the row's extremum (k_minmax_fwd's wave_argext over the TPR lanes of a row); the pair rides
// the same network as one 64-bit value (value bits low, column high)
__device__ __forceinline__ void row_argext(float& v, int& i, bool is_max) {
  if constexpr (MUZ_CHAIN_DPP && TPR == 32) {
    auto pick = [is_max](float a, int ia, float b, int ib, float& r, int& ir) {
      const bool take_b = (is_max ? b > a : b < a) || (b == a && ib < ia);
      r = take_b ? b : a;
      ir = take_b ? ib : ia;
    };
    auto step = [&](unsigned ov, unsigned oi) { pick(v, i, __builtin_bit_cast(float, ov), (int)oi, v, i); };
    step(dppu<0xB1>(__builtin_bit_cast(unsigned, v)), dppu<0xB1>((unsigned)i));
    step(dppu<0x4E>(__builtin_bit_cast(unsigned, v)), dppu<0x4E>((unsigned)i));
    step(dppu<0x141>(__builtin_bit_cast(unsigned, v)), dppu<0x141>((unsigned)i));
    step(dppu<0x140>(__builtin_bit_cast(unsigned, v)), dppu<0x140>((unsigned)i));
    const auto pv = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                     false, false);
    const auto pi = __builtin_amdgcn_permlane16_swap((unsigned)i, (unsigned)i, false, false);
    const unsigned vlo = pv[0], vhi = pv[1], ilo = pi[0], ihi = pi[1];
    pick(__builtin_bit_cast(float, vlo), (int)ilo, __builtin_bit_cast(float, vhi), (int)ihi, v, i);
  } else {
#pragma unroll
    for (int o = TPR / 2; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(i, o, 64);
      if ((is_max ? ov > v : ov < v) || (ov == v && oi < i)) v = ov, i = oi;
    }
  }
}

// The streamed matrix of the next GEMM, packed by muz_trunk_chain_pack so that every load instruction reads 1 KB
// contiguous (lane l: 16 bytes at l * 16): packed[w][kb][t][lane][j] = Mt[16 NT w + 16 t + (lane & 15)][16 kb +
// 4 (lane >> 4) + j].  D slots of NT loads (one per 16-column tile); prime() issues k-blocks 0 .. D - 2, gemm()
// keeps D - 1 blocks ahead.  All slot indices are compile-time.
struct Ring {
  f4 w[D][NT];
  const AS1 float* p;

  __device__ __forceinline__ void load(int slot, int blk) {
#pragma unroll
    for (int t = 0; t < NT; ++t) w[slot][t] = *reinterpret_cast<const AS1 f4*>(p + 256 * (NT * blk + t));
  }
  __device__ __forceinline__ void prime(const float* packed) {
    p = gp(packed) + ((size_t)(threadIdx.x >> 6) * KB * NT * 64 + (threadIdx.x & 63)) * 4;
#pragma unroll
    for (int b = 0; b < D - 1; ++b) load(b, b);
  }
};

// muz_trunk_chain_pack: one thread per packed float4 of one matrix and direction
constexpr int kPackMax = 32;   // matrices per launch: the det step's chain (7) + ResBlock stacks (12 + 4) in one
struct PackTable {
  const float* src[kPackMax];
  int count;
};

__global__ __launch_bounds__(256) void k_chain_pack(PackTable tb, float* fwd, float* bwd) {
  const int q = blockIdx.x * 256 + threadIdx.x;     // float4 index within matrix blockIdx.y
  const int i = blockIdx.y;
  const int lane = q & 63, t = (q >> 6) & (NT - 1), kb = (q >> (6 + LNT)) & (KB - 1), w = q >> (10 + LNT);
  const int r = 16 * NT * w + 16 * t + (lane & 15), c = 16 * kb + 4 * (lane >> 4);
  const float* W = tb.src[i];
  f4 vf, vb;
#pragma unroll
  for (int j = 0; j < 4; ++j) vf[j] = W[(size_t)(c + j) * N + r];     // Mt = W^T (forward, y = x W)
  vb = *reinterpret_cast<const f4*>(W + (size_t)r * N + c);           // Mt = W (backward, dx = dz W^T)
  *reinterpret_cast<f4*>(fwd + (size_t)i * N * N + 4 * q) = vf;
  *reinterpret_cast<f4*>(bwd + (size_t)i * N * N + 4 * q) = vb;
}

// out[t] = rows (lane & 15) of in[16][LD] times the primed matrix, columns 16 NT w + 16 t + 4 (lane >> 4) .. + 3
__device__ __forceinline__ void gemm(Ring& rg, const float* in, f4 (&out)[NT]) {
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  f4 acc[NT][2] = {};
  const float* xp = in + i * LD + 4 * g;
  f4 x = *reinterpret_cast<const f4*>(xp);
#pragma unroll
  for (int b = 0; b < KB; ++b) {
    if (b + D - 1 < KB) rg.load((b + D - 1) % D, b + D - 1);
    __builtin_amdgcn_sched_barrier(0);   // keep the loads D - 1 blocks ahead of their MFMAs
    // the next block's input row is read from LDS while this block's MFMAs run
    const f4 xn = b + 1 < KB ? *reinterpret_cast<const f4*>(xp + 16 * (b + 1)) : x;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t][j & 1] = mfma(rg.w[b % D][t][j], x[j], acc[t][j & 1]);
    x = xn;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) out[t] = acc[t][0] + acc[t][1];
}

// E consecutive floats (E = 4 or 8) as 16-byte accesses
__device__ __forceinline__ void ldE(const float* p, float (&v)[E]) {
#pragma unroll
  for (int k = 0; k < E; k += 4) *reinterpret_cast<f4*>(v + k) = *reinterpret_cast<const f4*>(p + k);
}
__device__ __forceinline__ void ldEg(const float* p, float (&v)[E]) {
#pragma unroll
  for (int k = 0; k < E; k += 4) *reinterpret_cast<f4*>(v + k) = *reinterpret_cast<const AS1 f4*>(gp(p + k));
}
__device__ __forceinline__ void stE(float* p, const float (&v)[E]) {
#pragma unroll
  for (int k = 0; k < E; k += 4) *reinterpret_cast<f4*>(p + k) = *reinterpret_cast<const f4*>(v + k);
}
__device__ __forceinline__ void stEg(float* p, const float (&v)[E]) {
#pragma unroll
  for (int k = 0; k < E; k += 4) *reinterpret_cast<AS1 f4*>(gpw(p + k)) = *reinterpret_cast<const f4*>(v + k);
}

__device__ __forceinline__ float rstd_of(float s, float s2) {
  const float mean = s / (float)N;
  return 1.0f / sqrtf(fmaxf(0.f, s2 / (float)N - mean * mean) + 1e-6f);
}

// one f4 of a group's per-layer vectors per thread and step (forward: kPf floats, backward: kPb)
template <bool FWD>
__device__ __forceinline__ void stage_params(const AS4 muz_chain_args* a, float* prm) {
  constexpr int P4 = (FWD ? kPf : kPb) / 4;
  for (int q = threadIdx.x; q < a->ngroups * P4; q += NTH) {
    const int g = q / P4, s = (q % P4) / (N / 4), c = 4 * (q % (N / 4));
    const AS4 muz_chain_group* G = &a->group[g];
    const float* src;
    if (FWD)
      src = s < 6 ? G->gamma[s] : s < 12 ? G->beta[s - 6] : s < 19 ? G->bias[s - 12] : s == 19 ? G->ln0_gamma
                                                                                                  : G->ln0_beta;
    else
      src = s < 6 ? G->gamma[s] : G->ln0_gamma;
    *reinterpret_cast<f4*>(prm + g * (FWD ? kPf : kPb) + s * N + c) = *reinterpret_cast<const AS1 f4*>(gp(src + c));
  }
}

// ---- forward ---------------------------------------------------------------------------------------------
// Loads retire in order for s_waitcnt vmcnt: a global operand is issued right AFTER a prime, so the GEMM's first
// k-blocks do not wait for it, and early enough that the GEMM's later k-blocks find it arrived.
struct Ln0Ops {   // the FiLM operands of one application
  float sc[E], sh[E];
};

__device__ __forceinline__ void load_ln0(const AS4 muz_chain_args* a, int i, size_t MN, size_t o, bool live,
                                         Ln0Ops& p) {
  if (live) {
    ldEg(a->scale1 + i * MN + o, p.sc);
    ldEg(a->shift + i * MN + o, p.sh);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) p.sc[e] = p.sh[e] = 0.f;
  }
}

__global__ __launch_bounds__(NTH, 1) void k_chain_fwd(muz_chain_args) {
#pragma clang fp contract(off)
  const AS4 muz_chain_args* a = kernarg0<muz_chain_args>();
  __shared__ __attribute__((aligned(16))) float xs[R * LD];    // the current GEMM's input
  __shared__ __attribute__((aligned(16))) float ys[R * LD];    // its output (+ bias)
  __shared__ __attribute__((aligned(16))) float rs[R * LD];    // the current ResBlock's input
  __shared__ __attribute__((aligned(16))) float lat[R * LD];   // x_i
  __shared__ __attribute__((aligned(16))) float prm[2 * kPf];   // the groups' per-layer vectors
  const int tid = threadIdx.x, M = a->M, T = a->T;
  const int row = tid / TPR, c0 = E * (tid % TPR), m = blockIdx.x * R + row;
  const bool live = m < M;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4, w = tid >> 6;
  const size_t MN = (size_t)M * N, o = (size_t)m * N + c0;
  stage_params<true>(a, prm);
  {
    float v[E] = {};
    if (live) ldEg(a->latent0 + o, v);
    if (live && a->stack0) stEg(a->stack0 + o, v);
    stE(lat + row * LD + c0, v);
  }
  Ln0Ops n0;
  load_ln0(a, 0, MN, o, live, n0);
  Ring rg;
  rg.prime(a->group[a->app[0]].wf[0]);
  __syncthreads();   // prm
#pragma unroll 1
  for (int i = 0; i < T; ++i) {
    const AS4 muz_chain_group* G = &a->group[a->app[i]];
    const float* pg = prm + a->app[i] * kPf;
    const size_t js = (size_t)a->slot[i] * MN + o;     // this row's offset in the group's stacks
    float* st = a->stats + (size_t)i * 7 * 2 * M;
    // LayerNorm_0 + FiLM (k_ln_fwd<256, true>)
    {
      float v[E], ga[E], be[E];
      ldE(lat + row * LD + c0, v);
      ldE(pg + kPfL0g + c0, ga);
      ldE(pg + kPfL0b + c0, be);
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        s += v[e];
        s2 += v[e] * v[e];
      }
      s = row_sum(s);
      s2 = row_sum(s2);
      const float mean = s / (float)N, rstd = rstd_of(s, s2);
      float ln[E], f[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        ln[e] = (v[e] - mean) * (rstd * ga[e]) + be[e];
        float p = ln[e] * n0.sc[e];
        asm volatile("" : "+v"(p));   // a multiply, then an add (torch's addcmul; no fma)
        f[e] = n0.sh[e] + p;
      }
      stE(xs + row * LD + c0, f);
      if (live) {
        stEg(a->ln0_out + i * MN + o, ln);
        stEg(G->X[0] + js, f);
        if ((tid % TPR) == 0) st[m] = mean, st[M + m] = rstd;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int l = 0; l <= kLayers; ++l) {
      f4 acc[NT];
      gemm(rg, xs, acc);
      f4 bb[NT] = {};
      if (l < kLayers) {
        rg.prime(G->wf[l + 1]);   // the next GEMM's matrix flies during the row phase
        if (l == 2 && i + 1 < T) load_ln0(a, i + 1, MN, o, live, n0);   // (behind the prime: see above)
#pragma unroll
        for (int t = 0; t < NT; ++t) bb[t] = *reinterpret_cast<const f4*>(pg + kPfBias + l * N + 16 * NT * w + 16 * t + 4 * lg);
      } else if (i + 1 < T) {
        rg.prime(a->group[a->app[i + 1]].wf[0]);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) *reinterpret_cast<f4*>(ys + li * LD + 16 * NT * w + 16 * t + 4 * lg) = acc[t] + bb[t];
      __syncthreads();
      float ga[E], be[E];
      if (l < kLayers) {
        ldE(pg + l * N + c0, ga);
        ldE(pg + kPfBeta + l * N + c0, be);
      } else {
        ldE(pg + kPfBias + 6 * N + c0, ga);
      }
      if (l < kLayers) {
        // Dense epilogue (k_ln_fwd): z = y + bias, LayerNorm, ReLU / residual ReLU
        const bool resid = l == 3 || l == 5;
        float v[E], res[E];
        ldE(ys + row * LD + c0, v);
        if (resid) ldE(rs + row * LD + c0, res);
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          s += v[e];
          s2 += v[e] * v[e];
        }
        s = row_sum(s);
        s2 = row_sum(s2);
        const float mean = s / (float)N, rstd = rstd_of(s, s2);
        float out[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float t = (v[e] - mean) * (rstd * ga[e]) + be[e];
          out[e] = resid ? fmaxf(res[e] + t, 0.f) : fmaxf(t, 0.f);
        }
        stE(xs + row * LD + c0, out);
        if (l == 1 || l == 3) stE(rs + row * LD + c0, out);   // the next ResBlock's input
        if (live) {
          stEg(G->X[l + 1] + js, out);
          stEg(a->z + ((size_t)i * kLayers + l) * MN + o, v);
          if ((tid % TPR) == 0) st[(2 + 2 * l) * M + m] = mean, st[(3 + 2 * l) * M + m] = rstd;
        }
        __syncthreads();
      } else {
        // min-max (k_minmax_fwd): q = x + (y + bias), out = (q - lo) / (hi - lo + 1e-8).  No barrier after it:
        // x_{i+1} is read back by this row's own threads, and xs / ys are free (the last GEMM is done)
        float x[E], y[E], q[E];
        ldE(lat + row * LD + c0, x);
        ldE(ys + row * LD + c0, y);
        float lo = INFINITY, hi = -INFINITY;
        int ilo = N, ihi = N;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          q[e] = x[e] + (y[e] + ga[e]);
          if (q[e] < lo) lo = q[e], ilo = c0 + e;
          if (q[e] > hi) hi = q[e], ihi = c0 + e;
        }
        row_argext(lo, ilo, false);
        row_argext(hi, ihi, true);
        const float den = (hi - lo) + 1e-8f;
        float out[E];
#pragma unroll
        for (int e = 0; e < E; ++e) out[e] = (q[e] - lo) / den;
        stE(lat + row * LD + c0, out);
        if (live) {
          stEg(a->out + i * MN + o, out);
          if (a->out_twin) stEg(a->out_twin + i * MN + o, out);
          stEg(a->q + i * MN + o, q);
          if ((tid % TPR) == 0) {
            const size_t r2 = (size_t)i * 2 * M + 2 * m;
            a->lohi[r2] = lo, a->lohi[r2 + 1] = hi;
            a->idx[r2] = ilo, a->idx[r2 + 1] = ihi;
          }
        }
      }
    }
  }
}

// ---- backward --------------------------------------------------------------------------------------------
// Column partials of one layer and application (k_dense_ln_bwd's: rows summed in order): [3][N] at p.
__device__ __forceinline__ void partials(const float* pgs, const float* pbs, const float* dzs, float* p) {
  const int tid = threadIdx.x;
  if constexpr (NTH >= 3 * N) {   // one column sum per thread
    if (tid >= 3 * N) return;
    const int q = tid / N, c = tid % N;
    const float* s = q == 0 ? pgs : pbs;
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) acc += q == 2 ? dzs[r * LD + c] : s[r * N + c];
    p[q * N + c] = acc;
  } else if (tid < N) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      sg += pgs[r * N + tid];
      sb += pbs[r * N + tid];
    }
    p[tid] = sg;
    p[N + tid] = sb;
  } else {
    const int c = tid - N;
    float sd = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) sd += dzs[r * LD + c];
    p[2 * N + c] = sd;
  }
}

struct MmOps {   // min-max backward of one application; lohi = (min, max) of q
  float g[E], q[E], h[E], lohi[2];
};
struct RowOps {  // a Dense + LayerNorm layer's saved forward values (LayerNorm_0: out = its output, sc = its FiLM scale)
  float out[E], z[E], sc[E];
  float mean, rstd;
};

// The saved values of dense layer k (k >= 0) or, k < 0, of LayerNorm_0, of application i.  Loaded one layer ahead
// of the row phase that uses them (they come from HBM / MALL: the forward wrote them a whole chain earlier).
__device__ __forceinline__ void load_rows(const AS4 muz_chain_args* a, int i, int k, size_t MN, size_t o, int m,
                                          bool live, RowOps& r) {
  if (live) {
    const int M = a->M;
    const AS1 float* st = gp(a->stats) + (size_t)i * 7 * 2 * M;
    if (k >= 0) {
      const AS4 muz_chain_group* G = &a->group[a->app[i]];
      ldEg(G->X[k + 1] + (size_t)a->slot[i] * MN + o, r.out);
      ldEg(a->z + ((size_t)i * kLayers + k) * MN + o, r.z);
      r.mean = st[(2 + 2 * k) * M + m], r.rstd = st[(3 + 2 * k) * M + m];
    } else {
      ldEg(a->ln0_out + i * MN + o, r.out);
      ldEg((i == 0 ? a->latent0 : a->out + (i - 1) * MN) + o, r.z);
      r.mean = st[m], r.rstd = st[M + m];
      ldEg(a->scale1 + i * MN + o, r.sc);
    }
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) r.out[e] = r.z[e] = r.sc[e] = 0.f;
    r.mean = r.rstd = 0.f;
  }
}

__device__ __forceinline__ void load_mm(const AS4 muz_chain_args* a, int i, size_t MN, size_t o, int m, bool live,
                                        MmOps& p) {
  if (live) {
    ldEg(a->g + i * MN + o, p.g);
    ldEg(a->q + i * MN + o, p.q);
    if (a->h) ldEg(a->h + i * MN + o, p.h);
    const size_t r2 = (size_t)i * 2 * a->M + 2 * m;
    p.lohi[0] = gp(a->lohi)[r2];
    p.lohi[1] = gp(a->lohi)[r2 + 1];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) p.g[e] = p.q[e] = p.h[e] = 0.f;
    p.lohi[0] = p.lohi[1] = 0.f;
  }
}

__global__ __launch_bounds__(NTH, 1) void k_chain_bwd(muz_chain_args) {
#pragma clang fp contract(off)
  const AS4 muz_chain_args* a = kernarg0<muz_chain_args>();
  __shared__ __attribute__((aligned(16))) float dzs[R * LD];     // the current GEMM's input (an output gradient)
  __shared__ __attribute__((aligned(16))) float dxs[R * LD];     // its output (the next row phase's dout)
  __shared__ __attribute__((aligned(16))) float dres[R * LD];    // a ResBlock's residual gradient
  __shared__ __attribute__((aligned(16))) float carry[R * LD];   // dq of application i, then + dz of its LayerNorm_0
  __shared__ __attribute__((aligned(16))) float pgs[R * N];      // per-row do * xhat, do (column partials)
  __shared__ __attribute__((aligned(16))) float pbs[R * N];
  __shared__ __attribute__((aligned(16))) float prm[2 * kPb];    // the groups' LayerNorm scales
  const int tid = threadIdx.x, M = a->M, T = a->T;
  const int row = tid / TPR, c0 = E * (tid % TPR), m = blockIdx.x * R + row;
  const bool live = m < M;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4, w = tid >> 6;
  const size_t MN = (size_t)M * N, o = (size_t)m * N + c0;
  const int tiles = (M + R - 1) / R;
  stage_params<false>(a, prm);   // (published by the barrier after the first min-max phase)
  MmOps mm;
  load_mm(a, T - 1, MN, o, m, live, mm);
  Ring rg;
  rg.prime(a->group[a->app[T - 1]].wb[6]);
  // ro: the saved values of the row phase after the current GEMM; nx: of the one after that, loaded a whole layer
  // ahead (ro = nx right after a GEMM: nx's loads are older than the GEMM's weight loads, so they have arrived)
  RowOps ro, nx;
  load_rows(a, T - 1, kLayers - 1, MN, o, m, live, nx);
#pragma unroll 1
  for (int i = T - 1; i >= 0; --i) {
    const AS4 muz_chain_group* G = &a->group[a->app[i]];
    const float* pg = prm + a->app[i] * kPb;
    const size_t js = (size_t)a->slot[i] * MN + o;
    const size_t pj = ((size_t)a->slot[i] * tiles + blockIdx.x) * 3 * N;   // this tile's partial block
    // min-max backward (k_minmax_bwd): d = (g + carry) x scale + h
    {
      float d[E];
#pragma unroll
      for (int e = 0; e < E; ++e) d[e] = mm.g[e];
      if (i + 1 < T) {
        float c[E];
        ldE(carry + row * LD + c0, c);
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = d[e] + c[e];
      }
      if (a->scaled[i]) {
        const float s = a->grad_scale;
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = d[e] * s;
      }
      if (a->h) {
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = d[e] + mm.h[e];
      }
      const float lo = mm.lohi[0], hi = mm.lohi[1], den = (hi - lo) + 1e-8f;
      float sd = 0.f, sq = 0.f;
      int nlo = 0, nhi = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        sd += d[e];
        sq += d[e] * (mm.q[e] - lo);
        nlo += mm.q[e] == lo;
        nhi += mm.q[e] == hi;
      }
      sd = row_sum(sd);
      sq = row_sum(sq) / (den * den);
      nlo = row_isum(nlo);
      nhi = row_isum(nhi);
      const float glo = (-sd / den + sq) / (float)nlo, ghi = (-sq) / (float)nhi;
      float dq[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float r = d[e] / den;
        if (mm.q[e] == lo) r = r + glo;
        if (mm.q[e] == hi) r = r + ghi;
        dq[e] = live ? r : 0.f;
      }
      stE(dzs + row * LD + c0, dq);
      stE(carry + row * LD + c0, dq);
      if (live) stEg(G->DZ[6] + js, dq);
    }
    __syncthreads();
#pragma unroll 1
    for (int l = kLayers; l >= 0; --l) {
      // GEMM: dx = dz W_l^T (+ the residual gradient after a ResBlock's first layer)
      f4 acc[NT];
      gemm(rg, dzs, acc);
      // the next matrix, then the saved values of the row phase after next
      const int k = l - 1;
      ro = nx;
      if (l > 0) {
        rg.prime(G->wb[k]);
        load_rows(a, i, k - 1, MN, o, m, live, nx);   // (k - 1 < 0: LayerNorm_0's)
        if (l == 3 && i > 0) load_mm(a, i - 1, MN, o, m, live, mm);   // (mm was consumed by this application)
      } else if (i > 0) {
        rg.prime(a->group[a->app[i - 1]].wb[6]);
        load_rows(a, i - 1, kLayers - 1, MN, o, m, live, nx);
      }
      const bool add_res = l == 2 || l == 4;
      const int mr = blockIdx.x * R + li;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = 16 * NT * w + 16 * t + 4 * lg;
        f4 v = acc[t];
        if (add_res) v += *reinterpret_cast<const f4*>(dres + li * LD + c);
        *reinterpret_cast<f4*>(dxs + li * LD + c) = v;
        if (l == 0 && mr < M) *reinterpret_cast<AS1 f4*>(gpw(a->dshift + i * MN + (size_t)mr * N + c)) = v;
      }
      // the previous layer's column partials (its rows are complete since the last barrier); the GEMM above read
      // dzs too, so they share the interval before the barrier
      if (l < kLayers) partials(pgs, pbs, dzs, G->part[l + 1] + pj);
      __syncthreads();
      if (l == 0) break;
      // LayerNorm / ReLU backward of Dense layer k (k_dense_ln_bwd's row half)
      const bool resid = k == 3 || k == 5;
      float d[E], ga[E];
      ldE(dxs + row * LD + c0, d);
      ldE(pg + k * N + c0, ga);
      float xh[E], gg[E], sa = 0.f, sb = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (!(ro.out[e] > 0.f)) d[e] = 0.f;
        xh[e] = (ro.z[e] - ro.mean) * ro.rstd;
        gg[e] = d[e] * ga[e];
        sa += gg[e];
        sb += gg[e] * xh[e];
      }
      if (resid) stE(dres + row * LD + c0, d);
      sa = row_sum(sa) / (float)N;
      sb = row_sum(sb) / (float)N;
      float dz[E], pg[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        dz[e] = ro.rstd * (gg[e] - sa - xh[e] * sb);
        pg[e] = d[e] * xh[e];
      }
      stE(dzs + row * LD + c0, dz);
      stE(pgs + row * N + c0, pg);
      stE(pbs + row * N + c0, d);
      if (live) stEg(G->DZ[k] + js, dz);
      __syncthreads();
    }
    // LayerNorm_0 + FiLM backward (k_ln_bwd<256, true>; ro = its saved values, scale1 below); then
    // carry = dz_0 + dq, the gradient of x_i
    {
      float d[E], ga[E];
      ldE(dxs + row * LD + c0, d);
      ldE(pg + kPbL0g + c0, ga);
      float ds[E], xh[E], gg[E], sa = 0.f, sb = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        ds[e] = d[e] * ro.out[e];
        d[e] = d[e] * (live ? ro.sc[e] : 0.f);
        xh[e] = (ro.z[e] - ro.mean) * ro.rstd;
        gg[e] = d[e] * ga[e];
        sa += gg[e];
        sb += gg[e] * xh[e];
      }
      if (live) stEg(a->dscale + i * MN + o, ds);
      sa = row_sum(sa) / (float)N;
      sb = row_sum(sb) / (float)N;
      float dz[E], pg[E], c[E];
      ldE(carry + row * LD + c0, c);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        dz[e] = ro.rstd * (gg[e] - sa - xh[e] * sb);
        pg[e] = d[e] * xh[e];
        c[e] = dz[e] + c[e];
      }
      stE(dzs + row * LD + c0, dz);
      stE(pgs + row * N + c0, pg);
      stE(pbs + row * N + c0, d);
      stE(carry + row * LD + c0, c);
    }
    __syncthreads();
    partials(pgs, pbs, dzs, G->part[0] + pj);
    __syncthreads();
  }
  if (live) {
    float c[E];
    ldE(carry + row * LD + c0, c);
    if (a->g0) {   // + the stack's block-0 gradient (what autograd's accumulation added, same single rounding)
      float g[E];
      ldEg(a->g0 + o, g);
#pragma unroll
      for (int e = 0; e < E; ++e) c[e] = c[e] + g[e];
    }
    stEg(a->dlatent0 + o, c);
  }
}

// ---- ResBlock stacks (muz_rbstack_*) ---------------------------------------------------------------------
// The same tile, GEMM loop and row arithmetic as the chain: weight layer l = 2 b + k of block b; the ResBlock input
// stays in LDS (rs) for the second layer's residual.
struct RowOpsRb {   // a layer's saved forward values for its backward rows; ms = (mean, rstd)
  float out[E], z[E], ms[2];
};

// the stack's per-layer vectors in LDS (as the chain's): forward gamma / beta / bias of each layer, backward gamma
constexpr int kRbMax = 2 * MUZ_RBSTACK_MAX, kRbBeta = kRbMax * N, kRbBias = 2 * kRbMax * N;
template <bool FWD>
__device__ __forceinline__ void stage_rb_params(const AS4 muz_rbstack_args* a, float* prm) {
  const int L = 2 * a->nb;
  for (int q = threadIdx.x; q < (FWD ? 3 : 1) * L * (N / 4); q += NTH) {
    const int s = q / (N / 4), c = 4 * (q % (N / 4)), v = s / L, l = s % L;
    const float* src = v == 0 ? a->gamma[l] : v == 1 ? a->beta[l] : a->bias[l];
    *reinterpret_cast<f4*>(prm + v * kRbMax * N + l * N + c) = *reinterpret_cast<const AS1 f4*>(gp(src + c));
  }
}

__device__ __forceinline__ void load_rb_rows(const AS4 muz_rbstack_args* a, int l, size_t MN, size_t o, int m,
                                             bool live, RowOpsRb& p) {
  const int L = 2 * a->nb, M = a->M;
  if (live) {
    ldEg((l + 1 < L ? a->X + (l + 1) * MN : a->out) + o, p.out);
    ldEg(a->z + l * MN + o, p.z);
    p.ms[0] = gp(a->stats)[(size_t)(2 * l) * M + m];
    p.ms[1] = gp(a->stats)[(size_t)(2 * l + 1) * M + m];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) p.out[e] = p.z[e] = 0.f;
    p.ms[0] = p.ms[1] = 0.f;
  }
}

__global__ __launch_bounds__(NTH, 1) void k_rbstack_fwd(muz_rbstack_args) {
#pragma clang fp contract(off)
  const AS4 muz_rbstack_args* a = kernarg0<muz_rbstack_args>();
  __shared__ __attribute__((aligned(16))) float xs[R * LD];    // the current GEMM's input
  __shared__ __attribute__((aligned(16))) float ys[R * LD];    // its output (+ bias)
  __shared__ __attribute__((aligned(16))) float rs[R * LD];    // the current ResBlock's input
  __shared__ __attribute__((aligned(16))) float prm[3 * kRbMax * N];
  const int tid = threadIdx.x, M = a->M, L = 2 * a->nb;
  const int row = tid / TPR, c0 = E * (tid % TPR), m = blockIdx.x * R + row;
  const bool live = m < M;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4, w = tid >> 6;
  const size_t MN = (size_t)M * N, o = (size_t)m * N + c0;
  stage_rb_params<true>(a, prm);   // (published by the barrier below)
  {
    float v[E] = {};
    if (live) ldEg(a->x + o, v);
    stE(xs + row * LD + c0, v);
    stE(rs + row * LD + c0, v);
    if (live) stEg(a->X + o, v);
  }
  Ring rg;
  rg.prime(a->wf[0]);
  __syncthreads();
#pragma unroll 1
  for (int l = 0; l < L; ++l) {
    f4 acc[NT];
    gemm(rg, xs, acc);
    float ga[E], be[E];
    f4 bb[NT];
    if (l + 1 < L) rg.prime(a->wf[l + 1]);
#pragma unroll
    for (int t = 0; t < NT; ++t) bb[t] = *reinterpret_cast<const f4*>(prm + kRbBias + l * N + 16 * NT * w + 16 * t + 4 * lg);
#pragma unroll
    for (int t = 0; t < NT; ++t) *reinterpret_cast<f4*>(ys + li * LD + 16 * NT * w + 16 * t + 4 * lg) = acc[t] + bb[t];
    __syncthreads();
    const bool resid = l & 1;
    float v[E], res[E];
    ldE(prm + l * N + c0, ga);
    ldE(prm + kRbBeta + l * N + c0, be);
    ldE(ys + row * LD + c0, v);
    if (resid) ldE(rs + row * LD + c0, res);
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      s += v[e];
      s2 += v[e] * v[e];
    }
    s = row_sum(s);
    s2 = row_sum(s2);
    const float mean = s / (float)N, rstd = rstd_of(s, s2);
    float out[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float t = (v[e] - mean) * (rstd * ga[e]) + be[e];
      out[e] = resid ? fmaxf(res[e] + t, 0.f) : fmaxf(t, 0.f);
    }
    stE(xs + row * LD + c0, out);
    if (resid) stE(rs + row * LD + c0, out);   // the next ResBlock's input
    if (live) {
      stEg((l + 1 < L ? a->X + (l + 1) * MN : a->out) + o, out);
      stEg(a->z + l * MN + o, v);
      if ((tid % TPR) == 0) a->stats[(size_t)(2 * l) * M + m] = mean, a->stats[(size_t)(2 * l + 1) * M + m] = rstd;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NTH, 1) void k_rbstack_bwd(muz_rbstack_args) {
#pragma clang fp contract(off)
  const AS4 muz_rbstack_args* a = kernarg0<muz_rbstack_args>();
  __shared__ __attribute__((aligned(16))) float dzs[R * LD];     // the current GEMM's input (an output gradient)
  __shared__ __attribute__((aligned(16))) float dxs[R * LD];     // its output (the next row phase's dout)
  __shared__ __attribute__((aligned(16))) float dres[R * LD];    // the ResBlock's residual gradient
  __shared__ __attribute__((aligned(16))) float pgs[R * N];      // per-row do * xhat, do (column partials)
  __shared__ __attribute__((aligned(16))) float pbs[R * N];
  __shared__ __attribute__((aligned(16))) float prm[kRbMax * N];   // the layers' LayerNorm scales
  const int tid = threadIdx.x, M = a->M, L = 2 * a->nb;
  const int row = tid / TPR, c0 = E * (tid % TPR), m = blockIdx.x * R + row;
  const bool live = m < M;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4, w = tid >> 6;
  const size_t MN = (size_t)M * N, o = (size_t)m * N + c0;
  const int tiles = (M + R - 1) / R;
  stage_rb_params<false>(a, prm);
  {
    float v[E] = {};
    if (live) ldEg(a->g + o, v);
    stE(dxs + row * LD + c0, v);
  }
  // ro: the saved values of the current row phase; nx: of the next one, loaded a layer ahead (ro = nx right after
  // a GEMM, whose later weight loads are younger than nx's)
  RowOpsRb ro, nx;
  load_rb_rows(a, L - 1, MN, o, m, live, ro);
  Ring rg;
  rg.prime(a->wb[L - 1]);
  if (L > 1) load_rb_rows(a, L - 2, MN, o, m, live, nx);
  __syncthreads();
#pragma unroll 1
  for (int l = L - 1; l >= 0; --l) {
    // LayerNorm / ReLU backward of layer l (k_dense_ln_bwd's row half); odd l: the residual ReLU
    const bool resid = l & 1;
    float d[E], ga[E];
    ldE(dxs + row * LD + c0, d);
    ldE(prm + l * N + c0, ga);
    float xh[E], gg[E], sa = 0.f, sb = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!(ro.out[e] > 0.f)) d[e] = 0.f;
      xh[e] = (ro.z[e] - ro.ms[0]) * ro.ms[1];
      gg[e] = d[e] * ga[e];
      sa += gg[e];
      sb += gg[e] * xh[e];
    }
    if (resid) stE(dres + row * LD + c0, d);
    sa = row_sum(sa) / (float)N;
    sb = row_sum(sb) / (float)N;
    float dz[E], pg[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      dz[e] = ro.ms[1] * (gg[e] - sa - xh[e] * sb);
      pg[e] = d[e] * xh[e];
    }
    stE(dzs + row * LD + c0, dz);
    stE(pgs + row * N + c0, pg);
    stE(pbs + row * N + c0, d);
    if (live) stEg(a->DZ + l * MN + o, dz);
    __syncthreads();
    // dx = dz W_l^T (+ the residual gradient after a ResBlock's first layer); the next layer's operands first
    f4 acc[NT];
    gemm(rg, dzs, acc);
    if (l > 0) {
      ro = nx;
      rg.prime(a->wb[l - 1]);
      if (l > 1) load_rb_rows(a, l - 2, MN, o, m, live, nx);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = 16 * NT * w + 16 * t + 4 * lg;
      f4 v = acc[t];
      if (!resid) v += *reinterpret_cast<const f4*>(dres + li * LD + c);
      *reinterpret_cast<f4*>(dxs + li * LD + c) = v;
    }
    partials(pgs, pbs, dzs, a->part + ((size_t)l * tiles + blockIdx.x) * 3 * N);
    __syncthreads();
  }
  if (live) {
    float v[E];
    ldE(dxs + row * LD + c0, v);
    stEg(a->dx + o, v);
  }
}

static int check_rbstack(const muz_rbstack_args* a, bool bwd) {
  MUZ_HOST_CHECK(a && a->nb >= 1 && a->nb <= MUZ_RBSTACK_MAX && a->M >= 0);
  for (int l = 0; l < 2 * a->nb; ++l)
    MUZ_HOST_CHECK(a->bias[l] && a->gamma[l] && a->beta[l] && (bwd ? a->wb[l] != nullptr : a->wf[l] != nullptr));
  MUZ_HOST_CHECK(a->x && a->X && a->out && a->z && a->stats);
  if (bwd) MUZ_HOST_CHECK(a->g && a->DZ && a->part && a->dx);
  return MUZ_OK;
}

static int check_args(const muz_chain_args* a, bool bwd) {
  MUZ_HOST_CHECK(a && a->T >= 1 && a->T <= MUZ_CHAIN_MAX_T && a->M >= 0 && a->ngroups >= 1 && a->ngroups <= 2);
  for (int i = 0; i < a->T; ++i) MUZ_HOST_CHECK(a->app[i] >= 0 && a->app[i] < a->ngroups && a->slot[i] >= 0);
  for (int g = 0; g < a->ngroups; ++g) {
    const muz_chain_group& G = a->group[g];
    MUZ_HOST_CHECK(G.ln0_gamma && G.ln0_beta);
    for (int l = 0; l < 7; ++l) MUZ_HOST_CHECK(G.bias[l] && G.X[l] && (bwd ? G.wb[l] && G.DZ[l] && G.part[l] : G.wf[l] != nullptr));
    for (int l = 0; l < 6; ++l) MUZ_HOST_CHECK(G.gamma[l] && G.beta[l]);
  }
  MUZ_HOST_CHECK(a->latent0 && a->scale1 && a->out && a->q && a->lohi && a->ln0_out && a->z && a->stats);
  if (bwd) MUZ_HOST_CHECK(a->g && a->dscale && a->dshift && a->dlatent0);
  else MUZ_HOST_CHECK(a->shift && a->idx);
  return MUZ_OK;
}

}  // namespace chain
}  // namespace muz

using namespace muz;

extern "C" {

int muz_trunk_chain_pack(const float* const* W, int32_t count, float* fwd, float* bwd, void* stream) {
  MUZ_HOST_CHECK(count >= 0 && (count == 0 || (W && fwd && bwd)));
  for (int s0 = 0; s0 < count; s0 += chain::kPackMax) {
    chain::PackTable tb{};
    tb.count = count - s0 < chain::kPackMax ? count - s0 : chain::kPackMax;
    for (int i = 0; i < tb.count; ++i) {
      MUZ_HOST_CHECK(W[s0 + i] != nullptr);
      tb.src[i] = W[s0 + i];
    }
    const size_t off = (size_t)s0 * chain::N * chain::N;
    chain::k_chain_pack<<<dim3(chain::N * chain::N / 4 / 256, tb.count), 256, 0, (hipStream_t)stream>>>(tb, fwd + off,
                                                                                                        bwd + off);
    const int rc = muz_last_launch_error();
    if (rc) return rc;
  }
  return MUZ_OK;
}

int muz_trunk_chain_fwd(const muz_chain_args* args, void* stream) {
  const int rc = chain::check_args(args, false);
  if (rc) return rc;
  if (args->M == 0) return MUZ_OK;
  chain::k_chain_fwd<<<(args->M + chain::R - 1) / chain::R, chain::NTH, 0, (hipStream_t)stream>>>(*args);
  return muz_last_launch_error();
}

int muz_rbstack_fwd(const muz_rbstack_args* args, void* stream) {
  const int rc = chain::check_rbstack(args, false);
  if (rc) return rc;
  if (args->M == 0) return MUZ_OK;
  chain::k_rbstack_fwd<<<(args->M + chain::R - 1) / chain::R, chain::NTH, 0, (hipStream_t)stream>>>(*args);
  return muz_last_launch_error();
}

int muz_rbstack_bwd(const muz_rbstack_args* args, void* stream) {
  const int rc = chain::check_rbstack(args, true);
  if (rc) return rc;
  if (args->M == 0) return MUZ_OK;
  chain::k_rbstack_bwd<<<(args->M + chain::R - 1) / chain::R, chain::NTH, 0, (hipStream_t)stream>>>(*args);
  return muz_last_launch_error();
}

int muz_trunk_chain_bwd(const muz_chain_args* args, void* stream) {
  const int rc = chain::check_args(args, true);
  if (rc) return rc;
  if (args->M == 0) return MUZ_OK;
  chain::k_chain_bwd<<<(args->M + chain::R - 1) / chain::R, chain::NTH, 0, (hipStream_t)stream>>>(*args);
  return muz_last_launch_error();
}

}  // extern "C"
