// DOG MuZero slice: the pieces of the networks at A = 806 shared by dog_muzero.hip (root / recurrent kernels) and
// dog_search.hip (the search).  See include/muz.h (muz_dog_net_w) for what the reference defines and what is defined
// here (MuZero_DOG/muzero_dog.py:25-137, DOG/dog.py:1264-1272).
#pragma once
#include "nn.hpp"

namespace muz {
inline namespace MUZ_NN_NS {   // (nn.hpp)

constexpr int kDogA = 806;                  // MUZ_DOG_ACTIONS
constexpr int kDogC = 34;                   // MUZ_DOG_OBS_CHANNELS
constexpr int kDogLastCols = kDogA - 768;   // 38 columns in the last logits chunk
constexpr int NTDL = nt_for(kDogLastCols);  // its 16-column tiles per wave

// PredictionNetwork4's policy logits Dense_2 (128 -> 806) over the tile, after pred16<.., NO_LOGITS> left the
// policy hidden layer in a.T and chunk 0's first k-blocks in pf: four column chunks (256, 256, 256, 38), each
// multiplied into LDS (a.U / a.W alternately) and handed to out(row, column, logit) by the row's lanes after the
// following barrier.  pf: (Ln: Kn x Nn, NTN tiles) on exit.  Ends with a barrier; a.U / a.W clobbered.
template <int NTN, class Out>
__device__ __forceinline__ void dog_logits16(const AS4 muz_dog_net_w* W, const Arena& a, Pf& pf, Out out,
                                             const AS4 muz_dense* Ln, int Kn, int Nn) {
  const int row = trow(), sub = tsub();
  auto hand = [&](const float* buf, int ld, int c0, int nc) {
#pragma unroll 1
    for (int c = sub; c < nc; c += kRowLanes) out(row, c0 + c, buf[row * ld + c]);
  };
  dense16<NT256, NT256>(W->logits[0], 128, 256, a.T, LD, a.U, LD, pf, &W->logits[1], 128, 256);
  SYNC();
  hand(a.U, LD, 0, 256);
  dense16<NT256, NT256>(W->logits[1], 128, 256, a.T, LD, a.W, LDW, pf, &W->logits[2], 128, 256);
  SYNC();
  hand(a.W, LDW, 256, 256);
  dense16<NT256, NTDL>(W->logits[2], 128, 256, a.T, LD, a.U, LD, pf, &W->logits[3], 128, kDogLastCols);
  SYNC();
  hand(a.U, LD, 512, 256);
  dense16<NTDL, NTN>(W->logits[3], 128, kDogLastCols, a.T, LD, a.W, LDW, pf, Ln, Kn, Nn);
  SYNC();
  hand(a.W, LDW, 768, kDogLastCols);
}

}  // namespace MUZ_NN_NS
}  // namespace muz
