// DynamicsNetwork4 + PredictionNetwork4 on a 16-row tile with every LayerNorm applied ON LOAD: the layer that
// consumes a LayerNorm's output normalises (and activates) its A operand as it reads it from LDS, with the row
// statistics assembled from per-wave partial sums the PRODUCING layer left in its epilogue.  A layer boundary is
// then one workgroup barrier instead of barrier + LayerNorm row pass + barrier: the round-4 timeline of
// k_gumbel_search (profiles/r4a_timeline.log) charged ~10.7 k of its ~55 k pipe-idle cycles per simulation to both
// waves of a SIMD sitting in row passes, and ~12 k to barrier waits.
//
// Arithmetic per element is nn.hpp's (fmaf(x - mean, rstd * scale, shift), then ReLU / residual + ReLU); only the
// statistics' summation order differs from ln16 (per wave over its columns, then over the 8 waves in order), so
// every kernel that builds its networks from these functions -- the search, the root and recurrent kernels --
// rounds identically.
//
// LDS of the chain (Lol): statistics partials [2 buffers][2 groups][16 rows][8 waves][s, s2] and the LayerNorm
// parameters the next layer reads, staged by the producing layer [2 buffers][scale 384 | shift 384].  Buffers
// alternate per layer, so a wave one barrier ahead never overwrites what a slower wave still reads.
#pragma once
#include "nn.hpp"

namespace muz {

static_assert(kWaves == 8 && kRowLanes == 32, "LayerNorm on load: 8 waves, 32 lanes per row");

#ifndef MUZ_LOL_DEEP
#define MUZ_LOL_DEEP 0   // 1: the A fragments' LDS reads two k-blocks ahead (more registers)
#endif

constexpr int kLolStFloats = 2 * 2 * kRows * kWaves * 2;
constexpr int kLolLnStride = 768;   // scale [0, 384) | shift [384, 768)
constexpr int kLolFloats = kLolStFloats + 2 * kLolLnStride;

struct Lol {
  float* base;
  __device__ __forceinline__ float* st(int buf, int grp) const { return base + ((buf * 2 + grp) * kRows) * kWaves * 2; }
  __device__ __forceinline__ float* ln(int buf) const { return base + kLolStFloats + buf * kLolLnStride; }
};

enum AMode { A_PLAIN = 0, A_RELU = 1, A_RESID = 2 };

// A operand of a dense layer: rows x [16][ldx] in LDS; for A_RELU / A_RESID the rows are a LayerNorm's input,
// normalised with the statistics partials `st` and the staged parameters (scale at lnp[lnoff + c], shift at
// lnp[384 + lnoff + c]), then a = relu(y) or relu(res + y).  keep: the transformed rows are also stored there
// (k-block kb by wave kb % 8), for a later residual.
struct ASrc {
  const float* x;
  int ldx;
  const float* st;
  const float* lnp;
  int lnoff;
  float n;
  const float* res;
  int ldr;
  float* keep;
  int ldk;
};
__device__ __forceinline__ ASrc a_plain(const float* x, int ldx) {
  return ASrc{x, ldx, nullptr, nullptr, 0, 1.f, nullptr, 0, nullptr, 0};
}
__device__ __forceinline__ ASrc a_ln(const float* x, int ldx, const float* st, const float* lnp, int lnoff, int n,
                                     const float* res = nullptr, int ldr = 0, float* keep = nullptr, int ldk = 0) {
  return ASrc{x, ldx, st, lnp, lnoff, (float)n, res, ldr, keep, ldk};
}

// mean and 1 / sqrt(var + eps) of row r from the 8 waves' partials (Flax fast variance E[z^2] - E[z]^2)
__device__ __forceinline__ void lol_row_stats(const float* st, int r, float n, float& mean, float& rstd) {
  const float* p = st + r * kWaves * 2;
  const f32x4 q0 = lds4(p), q1 = lds4(p + 4), q2 = lds4(p + 8), q3 = lds4(p + 12);
  const float s = ((q0[0] + q0[2]) + (q1[0] + q1[2])) + ((q2[0] + q2[2]) + (q3[0] + q3[2]));
  const float s2 = ((q0[1] + q0[3]) + (q1[1] + q1[3])) + ((q2[1] + q2[3]) + (q3[1] + q3[3]));
  mean = s / n;
  const float var = fmaxf(0.f, fmaf(-mean, mean, s2 / n));
  rstd = ln_rstd(var + 1e-6f);
}

// The ring of mfma_ring_impl with the A fragment of k-block kb + 1 read (x, scale, shift, residual) at the start of
// step kb and transformed after step kb's MFMAs are issued, so the VALU work runs while they execute.
template <int NT, int MODE>
__device__ __forceinline__ void mfma_ring_lol(const float* __restrict__ Wg, int KB, const ASrc& s, f32x4 (&acc)[NT],
                                              f32x4 (&b0)[NT], f32x4 (&b1)[NT]) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const AS1 f32x4* wp = gp(reinterpret_cast<const f32x4*>(Wg)) + lane * NT;
  const int wstep = 64 * NT;
  const float* xp = s.x + r * s.ldx + 4 * g;
  const float* rp = MODE == A_RESID ? s.res + r * s.ldr + 4 * g : nullptr;
  float* kp = s.keep ? s.keep + r * s.ldk + 4 * g : nullptr;
  const float* scp = MODE == A_PLAIN ? nullptr : s.lnp + s.lnoff + 4 * g;
  const float* shp = MODE == A_PLAIN ? nullptr : s.lnp + 384 + s.lnoff + 4 * g;
  float mean = 0.f, rstd = 0.f;
  if constexpr (MODE != A_PLAIN) lol_row_stats(s.st, r, s.n, mean, rstd);
  struct Raw {
    f32x4 x, sc, sh, res;
  };
  auto raw = [&](int kb, Raw& o) {
    o.x = lds4(xp + kb * 16);
    if constexpr (MODE != A_PLAIN) {
      o.sc = lds4(scp + kb * 16);
      o.sh = lds4(shp + kb * 16);
    }
    if constexpr (MODE == A_RESID) o.res = lds4(rp + kb * 16);
  };
  auto fin = [&](int kb, const Raw& o) -> f32x4 {
    if constexpr (MODE == A_PLAIN) {
      return o.x;
    } else {
      f32x4 y;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float t = fmaf(o.x[q] - mean, rstd * o.sc[q], o.sh[q]);
        if constexpr (MODE == A_RESID) t = o.res[q] + t;
        y[q] = fmaxf(t, 0.f);
      }
      if (kp && (kb & (kWaves - 1)) == wv) sts4(kp + kb * 16, y);
      return y;
    }
  };
#if MUZ_LOL_DEEP
  // two-deep: step kb reads the raw fragment of kb + 2 and transforms the one of kb + 1 read a step earlier
  Raw r0, r1, r2;
  raw(0, r0);
  if (KB > 1) raw(1, r1);
  f32x4 a0 = fin(0, r0), a1 = a0;
  auto step = [&](int kb, const f32x4 (&cur)[NT], f32x4 (&nxt)[NT], const f32x4& acur, f32x4& anxt, const Raw& rc,
                  Raw& rf) {
    if (kb + 2 < KB) {
#pragma unroll
      for (int t = 0; t < NT; ++t) nxt[t] = wp[(kb + 2) * wstep + t];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kb + 2 < KB) raw(kb + 2, rf);
    const f32x4 a = acur;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma4(cur[t][j], a[j], acc[t]);
    if (kb + 1 < KB) anxt = fin(kb + 1, rc);
  };
  int kb = 0;
  f32x4 b2[NT];
  for (; kb + 3 <= KB; kb += 3) {
    step(kb, b0, b2, a0, a1, r1, r2);
    step(kb + 1, b1, b0, a1, a0, r2, r0);
    step(kb + 2, b2, b1, a0, a1, r0, r1);
    a0 = a1;
  }
  if (kb < KB) step(kb, b0, b2, a0, a1, r1, r2);
  if (kb + 1 < KB) step(kb + 1, b1, b0, a1, a0, r2, r0);
#else
  Raw rw;
  raw(0, rw);
  f32x4 a0 = fin(0, rw), a1 = a0;
  auto step = [&](int kb, const f32x4 (&cur)[NT], f32x4 (&nxt)[NT], const f32x4& acur, f32x4& anxt) {
    if (kb + 2 < KB) {
#pragma unroll
      for (int t = 0; t < NT; ++t) nxt[t] = wp[(kb + 2) * wstep + t];
    }
    __builtin_amdgcn_sched_barrier(0);
    Raw rn;
    if (kb + 1 < KB) raw(kb + 1, rn);
    const f32x4 a = acur;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma4(cur[t][j], a[j], acc[t]);
    if (kb + 1 < KB) anxt = fin(kb + 1, rn);
  };
  int kb = 0;
  f32x4 b2[NT];
  for (; kb + 3 <= KB; kb += 3) {
    step(kb, b0, b2, a0, a1);
    step(kb + 1, b1, b0, a1, a0);
    step(kb + 2, b2, b1, a0, a1);
    a0 = a1;
  }
  if (kb < KB) step(kb, b0, b2, a0, a1);
  if (kb + 1 < KB) step(kb + 1, b1, b0, a1, a0);
#endif
}

// LayerNorm parameters for the layer after next, loaded by the producing layer before its MFMA loop and stored to
// the staging buffer after it (threads 0..191: one float4 each of scale | shift of up to two LayerNorms, widths n1 +
// n2 <= 384, the second at column offset n1)
struct LnStage {
  f32x4 v;
  int at;   // float index in the staging buffer, -1: nothing
};
__device__ __forceinline__ LnStage ln_stage_issue(const AS4 muz_ln* P1, int n1, const AS4 muz_ln* P2 = nullptr,
                                                  int n2 = 0) {
  LnStage s;
  s.at = -1;
  const int t = threadIdx.x, c = 4 * t;
  const int n = n1 + n2;
  if (!P1 || c >= 2 * n) return s;
  const bool shift = c >= n;
  const int col = shift ? c - n : c;
  const AS4 muz_ln* P = col < n1 ? P1 : P2;
  const int pc = col < n1 ? col : col - n1;
  s.v = *gp(reinterpret_cast<const f32x4*>((shift ? P->bias : P->scale) + pc));
  s.at = (shift ? 384 : 0) + col;
  return s;
}
__device__ __forceinline__ void ln_stage_store(const LnStage& s, float* dst) {
  if (s.at >= 0) sts4(dst + s.at, s.v);
}

// Dense layer over the tile with its A operand from `a` (MODE), out[16][N] = A @ W + b stored raw (the next
// LayerNorm's input), plus this wave's statistics partials of row r: group 0 over columns < split (into st0), group
// 1 over columns >= split (into st1); st0 null: none.  Columns >= split go to out2 (column - split) when given.
// pf: this layer's first k-blocks on entry, the next layer's (Ln) on exit.
template <int NT, int NTN, int MODE>
__device__ __forceinline__ void dense16_lol(const AS4 muz_dense& L, int K, int N, const ASrc& a, float* out, int ldo,
                                            Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn, float* st0,
                                            float* st1 = nullptr, int split = 1 << 30, float* out2 = nullptr,
                                            int ldo2 = 0) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int KB = (K + 15) >> 4;
  const int col0 = wv * NT * 16;
  if (col0 >= N) {
    pf_issue<NTN>(pf, Ln, Kn, Nn);
    if (st0 && g == 0) *reinterpret_cast<float2*>(st0 + (r * kWaves + wv) * 2) = make_float2(0.f, 0.f);
    if (st1 && g == 0) *reinterpret_cast<float2*>(st1 + (r * kWaves + wv) * 2) = make_float2(0.f, 0.f);
    return;
  }
  const AS1 f32x4* bias4 = gp(reinterpret_cast<const f32x4*>(L.b));
  f32x4 acc[NT], b0[NT], b1[NT], bb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = col0 + t * 16 + 4 * g;
    bb[t] = col < N ? bias4[col >> 2] : f32x4{0.f, 0.f, 0.f, 0.f};
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    b0[t] = pf.v0[t];
    b1[t] = pf.v1[t];
  }
  ST(ST_DENTRY);
  mfma_ring_lol<NT, MODE>(wave_group(L, KB, NT), KB, a, acc, b0, b1);
  ST(ST_MFMA);
  pf_issue<NTN>(pf, Ln, Kn, Nn);
  float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = col0 + t * 16 + 4 * g;
    if (col < N) {
      const f32x4 z = acc[t] + bb[t];
      if (out2 && col >= split)
        sts4(out2 + r * ldo2 + col - split, z);
      else
        sts4(out + r * ldo + col, z);
      if (st0) {
        float ps = 0.f, pq = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ps += z[q];
          pq = fmaf(z[q], z[q], pq);
        }
        if (col < split) {
          s0 += ps;
          q0 += pq;
        } else {
          s1 += ps;
          q1 += pq;
        }
      }
    }
  }
  if (st0) {
    // the row's 4 lanes (g = 0..3: lanes r, r + 16, r + 32, r + 48)
    auto red = [](float v) {
      const LoHi<float> p = swap32(v);
      const float u = p.lo + p.hi;
      const LoHi<float> q = swap16(u);
      return q.lo + q.hi;
    };
    s0 = red(s0);
    q0 = red(q0);
    if (g == 0) *reinterpret_cast<float2*>(st0 + (r * kWaves + wv) * 2) = make_float2(s0, q0);
    if (st1) {
      s1 = red(s1);
      q1 = red(q1);
      if (g == 0) *reinterpret_cast<float2*>(st1 + (r * kWaves + wv) * 2) = make_float2(s1, q1);
    }
  }
  ST(ST_EPI);
}

// Policy logits (Dense_2, K = 128 -> A <= 32) split over k (as logits16_splitk) with the A operand through LN2 on
// load; partials in part[8][16][32], summed by logits16_splitk_sum.
template <int NTN>
__device__ __forceinline__ void logits16_splitk_lol(int K, const ASrc& a, float* part, Pf& pf, const AS4 muz_dense* Ln,
                                                    int Kn, int Nn) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int KB = (K + 15) >> 4;
  if (w >= KB) {
    pf_issue<NTN>(pf, Ln, Kn, Nn);
    return;
  }
  const int r = lane & 15, g = lane >> 4;
  float mean, rstd;
  lol_row_stats(a.st, r, a.n, mean, rstd);
  const f32x4 x = lds4(a.x + r * a.ldx + w * 16 + 4 * g);
  const f32x4 sc = lds4(a.lnp + a.lnoff + w * 16 + 4 * g), sh = lds4(a.lnp + 384 + a.lnoff + w * 16 + 4 * g);
  f32x4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = fmaxf(fmaf(x[q] - mean, rstd * sc[q], sh[q]), 0.f);
  const f32x4 b0 = pf.v0[0], b1 = pf.v1[0];
  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc0 = mfma4(b0[j], v[j], acc0);
    acc1 = mfma4(b1[j], v[j], acc1);
  }
  pf_issue<NTN>(pf, Ln, Kn, Nn);
  float* pw = part + (w * 16 + r) * 32 + 4 * g;
  *reinterpret_cast<f32x4*>(pw) = acc0;
  *reinterpret_cast<f32x4*>(pw + 16) = acc1;
}

// DynamicsNetwork4's trunk (muzero_deterministic_madn.py:391-455) with LayerNorm on load, from the LayerNorm_0 +
// FiLM pass through Dense_5 + the skip min-max; the min-max pass also stores the latent to `emb` (null: no store),
// leaves PredictionNetwork4's LayerNorm_0 of it in a.X and the latent itself in a.L (for the reward / discount trunk
// that pred16_lol runs).  Ends with a barrier.  pf: d3 on entry, Ln (Pred4's first layer) on exit.  Scratch: T, U, W
// (the two ResBlock residuals at W[0:256] and W[256:512]).
template <int NTN>
__device__ __forceinline__ void dyn16_lol(const AS4 muz_dyn_w& D, int A, const DynIn& in, const Arena& a, const Lol& lo,
                                          Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn, const AS4 muz_ln& pln0,
                                          AS1 float* emb) {
  using RV = RowVec<LAT>;
  const int row = trow(), sub = tsub();
  {   // LayerNorm_0 of the latent + FiLM (registers), as dyn16
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
  float* R0 = a.W;          // ResBlock_0's output (ResBlock_1's residual)
  float* R1 = a.W + 256;    // ResBlock_1's input (ResBlock_0's residual)
  LnStage ls = ln_stage_issue(&D.ln1, LAT);
  SYNC();
  // Dense_3: X -> T;  stats buffer 0, LN_1 parameters staged in buffer 0
  dense16_lol<NT256, NT256, A_PLAIN>(D.d3, LAT, LAT, a_plain(a.X, LD), a.T, LD, pf, &D.d4, LAT, LAT, lo.st(0, 0));
  ln_stage_store(ls, lo.ln(0));
  ls = ln_stage_issue(&D.ln2, LAT);
  SYNC();
  // Dense_4: relu(LN_1(T)) -> X
  dense16_lol<NT256, NT256, A_RELU>(D.d4, LAT, LAT, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.X, LD, pf,
                                    &D.rb[0].d0, LAT, LAT, lo.st(1, 0));
  ln_stage_store(ls, lo.ln(1));
  ls = ln_stage_issue(&D.rb[0].ln0, LAT);
  SYNC();
  // ResBlock_0 Dense_0: input r0 = relu(LN_2(X)) (kept in R1 for the residual) -> T
  dense16_lol<NT256, NT256, A_RELU>(D.rb[0].d0, LAT, LAT,
                                    a_ln(a.X, LD, lo.st(1, 0), lo.ln(1), 0, LAT, nullptr, 0, R1, LDW), a.T, LD, pf,
                                    &D.rb[0].d1, LAT, LAT, lo.st(0, 0));
  ln_stage_store(ls, lo.ln(0));
  ls = ln_stage_issue(&D.rb[0].ln1, LAT);
  SYNC();
  // ResBlock_0 Dense_1: relu(LN(T)) -> U
  dense16_lol<NT256, NT256, A_RELU>(D.rb[0].d1, LAT, LAT, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.U, LD, pf,
                                    &D.rb[1].d0, LAT, LAT, lo.st(1, 0));
  ln_stage_store(ls, lo.ln(1));
  ls = ln_stage_issue(&D.rb[1].ln0, LAT);
  SYNC();
  // ResBlock_1 Dense_0: input r1 = relu(r0 + LN(U)) (kept in R0) -> T
  dense16_lol<NT256, NT256, A_RESID>(D.rb[1].d0, LAT, LAT,
                                     a_ln(a.U, LD, lo.st(1, 0), lo.ln(1), 0, LAT, R1, LDW, R0, LDW), a.T, LD, pf,
                                     &D.rb[1].d1, LAT, LAT, lo.st(0, 0));
  ln_stage_store(ls, lo.ln(0));
  ls = ln_stage_issue(&D.rb[1].ln1, LAT);
  SYNC();
  // ResBlock_1 Dense_1: relu(LN(T)) -> U
  dense16_lol<NT256, NT256, A_RELU>(D.rb[1].d1, LAT, LAT, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.U, LD, pf,
                                    &D.d5, LAT, LAT, lo.st(1, 0));
  ln_stage_store(ls, lo.ln(1));
  SYNC();
  // Dense_5: relu(r1 + LN(U)) -> T (no LayerNorm after it); Pred4's LayerNorm_0 parameters land under its loop
  const LnP<LAT> pl = ln_load<LAT>(pln0);
  dense16_lol<NT256, NTN, A_RESID>(D.d5, LAT, LAT, a_ln(a.U, LD, lo.st(1, 0), lo.ln(1), 0, LAT, R0, LDW), a.T, LD, pf,
                                   Ln, Kn, Nn, nullptr);
  SYNC();
  // latent = minmax(L + T) -> L (and the tree), Pred4 LayerNorm_0 of it -> X
  skip_minmax16(a.T, a.L, LD, &pl, emb, a.X, a.L);
  ST(ST_PASS);
  SYNC();
}

// PredictionNetwork4 (muzero_deterministic_madn.py:549-583) with LayerNorm on load, its LayerNorm_0 already in a.X
// (LN0_DONE; otherwise computed here from `lat`), plus -- with D -- Dyn4's reward / discount trunk on the latent in
// a.L (Dense_6 | Dense_7 in the Dense_1 phase, the support heads in the last phase).  Leaves the policy logits in
// a.U[:, 0:A] (read back only by lane (row, column)), tanh value in a.v0 and reward / discount in a.v1 / a.v2.
// pf: rb[0].d0 on entry, Ln on exit.
template <int NTN, bool LN0_DONE>
__device__ __forceinline__ void pred16_lol(const AS4 muz_pred_w& P, int A, const float* lat, const Arena& a,
                                           const Lol& lo, Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn,
                                           const AS4 muz_dyn_w* D = nullptr, int ar = 0) {
  if constexpr (!LN0_DONE) {
    ln16<LAT, LN_PLAIN>(lat, LD, a.X, LD, P.ln0);
    SYNC();
  }
  float* R0 = a.W;   // ResBlock_1's input (the residual of d03's input)
  LnStage ls = ln_stage_issue(&P.rb[0].ln0, LAT);
  // ResBlock_0 Dense_0: X (LayerNorm_0 output) -> T
  dense16_lol<NT256, NT256, A_PLAIN>(P.rb[0].d0, LAT, LAT, a_plain(a.X, LD), a.T, LD, pf, &P.rb[0].d1, LAT, LAT,
                                     lo.st(0, 0));
  ln_stage_store(ls, lo.ln(0));
  ls = ln_stage_issue(&P.rb[0].ln1, LAT);
  SYNC();
  dense16_lol<NT256, NT256, A_RELU>(P.rb[0].d1, LAT, LAT, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.U, LD, pf,
                                    &P.rb[1].d0, LAT, LAT, lo.st(1, 0));
  ln_stage_store(ls, lo.ln(1));
  ls = ln_stage_issue(&P.rb[1].ln0, LAT);
  SYNC();
  // ResBlock_1 Dense_0: input relu(X + LN(U)) (kept in R0) -> T
  dense16_lol<NT256, NT256, A_RESID>(P.rb[1].d0, LAT, LAT,
                                     a_ln(a.U, LD, lo.st(1, 0), lo.ln(1), 0, LAT, a.X, LD, R0, LDW), a.T, LD, pf,
                                     &P.rb[1].d1, LAT, LAT, lo.st(0, 0));
  ln_stage_store(ls, lo.ln(0));
  ls = ln_stage_issue(&P.rb[1].ln1, LAT);
  SYNC();
  dense16_lol<NT256, NT256, A_RELU>(P.rb[1].d1, LAT, LAT, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.U, LD, pf,
                                    &P.d03, LAT, 384, lo.st(1, 0));
  ln_stage_store(ls, lo.ln(1));
  ls = ln_stage_issue(&P.ln1, LAT, &P.ln3, 128);
  SYNC();
  // [policy Dense_0 | value Dense_3]: relu(R0 + LN(U)) -> policy half T, value half X[0:128]; two statistics groups
  dense16_lol<NT384, NT128, A_RESID>(P.d03, LAT, 384, a_ln(a.U, LD, lo.st(1, 0), lo.ln(1), 0, LAT, R0, LDW), a.T, LD,
                                     pf, &P.d1, LAT, 128, lo.st(0, 0), lo.st(0, 1), LAT, a.X, LD);
  ln_stage_store(ls, lo.ln(0));
  ls = ln_stage_issue(&P.ln2, 128);
  const HeadW hv = head_load(P.d5, 1);
  SYNC();
  // policy Dense_1: relu(LN_1(T)) -> U[0:128];  [Dyn4 Dense_6 | Dense_7]: latent L -> W[0:128];
  // value Dense_4: relu(LN_3(X[0:128])) -> W[256:320]
  HeadW hr, hd;
  float add_r[HeadW::kPer], add_d[HeadW::kPer];
  if (D) {
    dense16_lol<NT128, NT128, A_RELU>(P.d1, LAT, 128, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.U, LD, pf,
                                      &D->d67, LAT, 128, lo.st(1, 0));
    // the reward / discount heads and Dense_6 | Dense_7's one-hot rows at this lane's head inputs: issued here, they
    // land under the next two MFMA loops
    hr = head_load(D->reward_head, 3);
    hd = head_load(D->discount_head, 3);
    const bool oh = ar >= 0 && ar < A;
    const AS1 float* w67 = gp(D->d67_onehot) + (oh ? ar : 0) * 128;
#pragma unroll
    for (int i = 0; i < HeadW::kPer; ++i) {
      const int k = tsub() + i * kRowLanes;
      add_r[i] = (oh && k < 64) ? w67[k] : 0.f;
      add_d[i] = (oh && k < 64) ? w67[64 + k] : 0.f;
    }
    dense16_lol<NT128, NT64, A_PLAIN>(D->d67, LAT, 128, a_plain(a.L, LD), a.W, LDW, pf, &P.d4, 128, 64, nullptr);
  } else {
    dense16_lol<NT128, NT64, A_RELU>(P.d1, LAT, 128, a_ln(a.T, LD, lo.st(0, 0), lo.ln(0), 0, LAT), a.U, LD, pf,
                                     &P.d4, 128, 64, lo.st(1, 0));
  }
  // value Dense_4 (waves 0-3: 64 columns), then every wave's k-block of the split-K policy logits
  dense16_lol<NT64, 1, A_RELU>(P.d4, 128, 64, a_ln(a.X, LD, lo.st(0, 1), lo.ln(0), LAT, 128), a.W + 256, LDW, pf,
                               nullptr, 0, 0, nullptr);
  pf_issue_splitk(pf, &P.d2, 128);
  ln_stage_store(ls, lo.ln(1));
  SYNC();
  // last phase: policy logits (split-K, LayerNorm_2 on load) as partials in a.L; value head on relu(Dense_4);
  // reward / discount heads on relu(W[0:128] + one-hot rows)
  logits16_splitk_lol<NTN>(128, a_ln(a.U, LD, lo.st(1, 0), lo.ln(1), 0, 128), a.L, pf, Ln, Kn, Nn);
  {
    const float zero[HeadW::kPer] = {};
    const float v = head_dot_relu(a.W + 256, LDW, zero, hv, 0);
    if (tsub() == 0) a.v0[trow()] = tanhf(v);
  }
  if (D) {
    float rl[3], dl[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      rl[j] = head_dot_relu(a.W, LDW, add_r, hr, j);
      dl[j] = head_dot_relu(a.W + 64, LDW, add_d, hd, j);
    }
    if (tsub() == 0) {
      a.v1[trow()] = softmax3_support(rl[0], rl[1], rl[2]);
      a.v2[trow()] = softmax3_support(dl[0], dl[1], dl[2]);
    }
  }
  ST(ST_PASS);
  SYNC();
  if (tsub() < A) a.U[trow() * LD + tsub()] = logits16_splitk_sum(P.d2, 128, a.L);
}

}  // namespace muz
