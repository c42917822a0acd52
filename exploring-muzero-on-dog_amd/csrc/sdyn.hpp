// StochasticDynamicsNetwork4 (MuZero_Classic_MADN/muzero_classic_madn.py:314-408) on 16-row tiles, built
// from the same fused fp32 MFMA blocks as the det Dyn4 (nn.hpp).  Both halves share one trunk shape:
//   x = LN_in(s) * (1 + scale[o]) + shift[o]        (FiLM rows tabulated per outcome o, in registers)
//   x = relu(LN1(dense1 x)); x = relu(LN2(dense2 x)); 2 ResBlocks; x = proj x
//   out = minmax(s + x)
// action_dynamics adds the reward head (on [afterstate, one_hot(a)]), the discount head (on the INPUT
// latent) and the chance head (on the afterstate).
#pragma once
#include "nn.hpp"

namespace muz {
inline namespace MUZ_NN_NS {   // (nn.hpp)

constexpr int NT32 = nt_for(32), NT70 = nt_for(70);

// One row's trunk inputs: the input state (RowVec<LAT> layout), its FiLM rows and LN_in's parameters.
struct FilmIn {
  f32x4 s[RowVec<LAT>::V], sc[RowVec<LAT>::V], sh[RowVec<LAT>::V];
  LnP<LAT> ln;
};

// film_tab row-major [rows][512] = [scale | shift]; an outcome outside [0, nrow) reads row nrow
// (jax.nn.one_hot of an out-of-range index is the zero vector).
__device__ __forceinline__ FilmIn film_load(const float* film_tab, int nrow, const AS4 muz_ln& ln, const AS1 float* state,
                                            int outcome) {
  using RV = RowVec<LAT>;
  FilmIn in;
  const int sub = tsub();
  const int fr = (outcome >= 0 && outcome < nrow) ? outcome : nrow;
  const AS1 f32x4* film = gp(reinterpret_cast<const f32x4*>(film_tab)) + fr * (2 * LAT / 4);
#pragma unroll
  for (int i = 0; i < RV::V; ++i) {
    const int c = RV::col(sub, i);
    in.s[i] = state ? *reinterpret_cast<const AS1 f32x4*>(state + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    in.sc[i] = film[c >> 2];
    in.sh[i] = film[(LAT + c) >> 2];
  }
  in.ln = ln_load<LAT>(ln);
  return in;
}

struct TrunkW {
  const AS4 muz_dense* d1;
  const AS4 muz_ln* l1;
  const AS4 muz_dense* d2;
  const AS4 muz_ln* l2;
  const AS4 muz_resblock* rb;   // [2]
  const AS4 muz_dense* proj;
};

// Trunk: pf holds d1's first k-blocks on entry and (Ln, Kn x Nn, NTN) on exit.
// Out: a.T = minmax(state + proj(...)), a.L = state.
template <int NTN>
__device__ __forceinline__ void film_trunk16(const TrunkW& W, const FilmIn& in, const Arena& a, Pf& pf,
                                             const AS4 muz_dense* Ln, int Kn, int Nn) {
  using RV = RowVec<LAT>;
  const int row = trow(), sub = tsub();
  {
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < RV::V; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s += in.s[i][q];
        s2 = fmaf(in.s[i][q], in.s[i][q], s2);
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
        const float y = fmaf(in.s[i][q] - mean, inv * in.ln.sc[i][q], in.ln.sh[i][q]);
        x[q] = fmaf(y, 1.0f + in.sc[i][q], in.sh[i][q]);
      }
      sts4(a.X + row * LD + c, x);
      sts4(a.L + row * LD + c, in.s[i]);
    }
    ST(ST_ROW);
  }
  SYNC();
  if constexpr (MUZ_LN_EPILOGUE != 0) {
    const LnE<NT256> q1 = lne_load<NT256>(*W.l1);
    dense_ln16<NT256, NT256, LN_RELU>(*W.d1, LAT, a.X, LD, a.T, LD, pf, W.d2, LAT, LAT, q1, a.P);
    SYNC();
    const LnE<NT256> q2 = lne_load<NT256>(*W.l2);
    dense_ln16<NT256, NT256, LN_RELU>(*W.d2, LAT, a.T, LD, a.X, LD, pf, &W.rb[0].d0, LAT, LAT, q2, a.P);
    SYNC();
  } else {
    const LnP<LAT> p1 = ln_load<LAT>(*W.l1);
    dense16<NT256, NT256>(*W.d1, LAT, LAT, a.X, LD, a.T, LD, pf, W.d2, LAT, LAT);
    SYNC();
    ln16<LAT, LN_RELU>(a.T, LD, a.T, LD, p1);
    SYNC();
    const LnP<LAT> p2 = ln_load<LAT>(*W.l2);
    dense16<NT256, NT256>(*W.d2, LAT, LAT, a.T, LD, a.X, LD, pf, &W.rb[0].d0, LAT, LAT);
    SYNC();
    ln16<LAT, LN_RELU>(a.X, LD, a.X, LD, p2);
    SYNC();
  }
  resblock16<NT256>(W.rb[0], a.X, a.T, a.U, pf, &W.rb[1].d0, LAT, LAT, a.P);
  resblock16<NT256>(W.rb[1], a.X, a.T, a.U, pf, W.proj, LAT, LAT, a.P);
  dense16<NT256, NTN>(*W.proj, LAT, LAT, a.X, LD, a.T, LD, pf, Ln, Kn, Nn);
  SYNC();
  skip_minmax16(a.T, a.L, LD);
  ST(ST_PASS);
  SYNC();
}

__device__ __forceinline__ TrunkW act_trunk(const AS4 muz_sdyn_w& D) {
  return TrunkW{&D.act_dense1, &D.act_ln1, &D.act_dense2, &D.act_ln2, D.act_rb, &D.act_proj};
}
__device__ __forceinline__ TrunkW chance_trunk(const AS4 muz_sdyn_w& D) {
  return TrunkW{&D.chance_dense1, &D.chance_ln1, &D.chance_dense2, &D.chance_ln2, D.chance_rb, &D.chance_proj};
}

// action_dynamics (329-371) + the decision_recurrent_fn reductions (420-423).
// In: `in` = (latent, act FiLM rows), ar = this row's action.  pf: act_dense1 on entry, (Ln...) on exit.
// Out: a.T afterstate, a.v1 reward, a.v2 discount (support expectations), a.E[row][0:6] chance logits.
template <int NTN>
__device__ __forceinline__ void sdyn_action16(const AS4 muz_sdyn_w& D, int A, const FilmIn& in, int ar, const Arena& a,
                                              Pf& pf, const AS4 muz_dense* Ln, int Kn, int Nn) {
  const int row = trow(), sub = tsub();
  const bool oh = ar >= 0 && ar < A;
  film_trunk16<NT70>(act_trunk(D), in, a, pf, &D.rc, LAT, 70);
  const HeadK<64> hr = head_load<64>(D.reward_head, 3);
  const HeadK<32> hd = head_load<32>(D.discount_head, 3);
  const LnP<32> pdl = ln_load<32>(D.discount_ln);
  // [reward_dense afterstate rows | chance_head] on the afterstate, discount_dense on the input latent
  dense16<NT70, NT32>(D.rc, LAT, 70, a.T, LD, a.W, LDW, pf, &D.discount_dense, LAT, 32);
  dense16<NT32, NTN>(D.discount_dense, LAT, 32, a.L, LD, a.W + 128, LDW, pf, Ln, Kn, Nn);
  SYNC();
  const AS1 float* won = gp(D.reward_onehot);
  for (int c = sub; c < 64; c += kRowLanes) {
    const float h = a.W[row * LDW + c];
    a.W[row * LDW + c] = fmaxf(oh ? h + won[ar * 64 + c] : h, 0.f);
  }
  if (sub < MUZ_CHANCE_OUTCOMES) a.E[row * LDE + sub] = a.W[row * LDW + 64 + sub];
  ln16<32, LN_RELU>(a.W + 128, LDW, a.W + 128, LDW, pdl);
  ST(ST_PASS);
  SYNC();
  float rl[3], dl[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    rl[j] = head_dot<64>(a.W, LDW, hr, j);
    dl[j] = head_dot<32>(a.W + 128, LDW, hd, j);
  }
  if (sub == 0) {
    a.v1[row] = softmax3_support(rl[0], rl[1], rl[2]);
    a.v2[row] = softmax3_support(dl[0], dl[1], dl[2]);
  }
  ST(ST_PASS);
  SYNC();
}

// chance_dynamics (373-408).  In: `in` = (afterstate, chance FiLM rows).  Out: a.T next state.
template <int NTN>
__device__ __forceinline__ void sdyn_chance16(const AS4 muz_sdyn_w& D, const FilmIn& in, const Arena& a, Pf& pf,
                                              const AS4 muz_dense* Ln, int Kn, int Nn) {
  film_trunk16<NTN>(chance_trunk(D), in, a, pf, Ln, Kn, Nn);
}

}  // namespace MUZ_NN_NS
}  // namespace muz
