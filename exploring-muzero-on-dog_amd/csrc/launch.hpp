// Internal (C++) launchers shared between translation units.  `n_dev`, when non-null, is a
// device-resident row count that overrides `n` (grids are sized for `n`; surplus workgroups exit),
// so a device-compacted batch can be processed without a host round trip.
#pragma once
#include "common.hpp"

namespace muz {

struct SearchArgs {
  int S, D, max_considered;
  float value_scale, maxvisit_init, gumbel_scale;
  unsigned long long seed;
  int turn;
  // Optional noise keys of a self-play driver: the game id of lane l is key_game[l] (else l) and its
  // turn key_turn[game id] (else `turn`) -- the game's own step count, so a game draws the same noise
  // whichever lane and global turn it is played in.
  const int32_t* key_game = nullptr;
  const int32_t* key_turn = nullptr;
  int exact_select = 0;   // k_dog_search: every interior selection on the exact path (MUZ_DOG_EXACT_SELECT)
  int games_per_wg = 8;   // k_dog_search one-game-per-wave form: games per workgroup (<= 8; MUZ_DOG_GPW)
};

// host_counts (optional): the self-play ledger's mapped pinned slot; k_repr_conv's first workgroup copies n_dev[0..1]
// (the turn's searching / active counts, final once the turn head has run) into it
int launch_root_inference(const muz_net_w& w, const float* obs, int n, const int* n_dev, float* conv_scratch,
                          float* logits, float* value, float* emb, hipStream_t s, int32_t* host_counts = nullptr);

int launch_root_inference(const muz_classic_net_w& w, const float* obs, int n, const int* n_dev, float* conv_scratch,
                          float* logits, float* value, float* emb, hipStream_t s);

// k_repr_conv (RepresentationNetwork2's convolutions, nets.hip) and k_film (the per-action FiLM table)
int launch_repr_conv(const muz_repr_w& r, const float* obs, int C, int n, const int* n_dev, float* conv,
                     hipStream_t s, int32_t* host_counts = nullptr);
// k_dense0 (nets.hip): Dense_0 (3584 -> 256) of every row of the root scratch, 64 x 64 output tiles
int launch_dense0(const muz_dense& d0, int n, const int* n_dev, float* conv, hipStream_t s);
int launch_film(const muz_dyn_w& d, int A, hipStream_t s);

int launch_gumbel_search(const muz_net_w& w, const SearchArgs& sa, const float* root_logits, const float* root_value,
                         const float* root_emb, const uint32_t* legal, const float* gumbel, const int32_t* game_id,
                         int n, const int* n_dev, void* workspace, int32_t* action, float* weights, float* value,
                         hipStream_t s);

int64_t search_workspace_bytes(int n, int S);

// Stochastic MuZero (stochastic.hip)
struct SArgs {
  int S, D, A;
  float dir_frac, dir_alpha, pb_c_init, pb_c_base, temperature;
  unsigned long long seed;
  int turn;
  // optional noise keys of a self-play driver (see SearchArgs): game id key_game[lane], turn key_turn[game id]
  const int32_t* key_game = nullptr;
  const int32_t* key_turn = nullptr;
};
SArgs make_sargs(const muz_stoch_cfg& cfg, int A);
int launch_stochastic_search(const muz_classic_net_w& w, const SArgs& sa, const float* root_logits,
                             const float* root_value, const float* root_emb, const uint32_t* legal,
                             const float* dirichlet, const float* gumbel, const int32_t* game_id, int n, const int* n_dev,
                             void* workspace, int32_t* action, float* weights, float* value, hipStream_t s);
int64_t stochastic_workspace_bytes(int n, int S);
int check_classic_net(const muz_classic_net_w* w);

}  // namespace muz
