// Host-side construction of rule constants (mirrors env_reset's fix-ups,
// MADN/deterministic_madn.py:62-78).
#pragma once
#include "detmadn.hpp"

namespace muz {

// allow_random_start: the entry point can draw a random starting player (env_reset's starting_player < 0 or >= P,
// deterministic_madn.py:60-62, classic_madn.py:70-72, dog.py:102-104) -- it has a reset seed; c->starting_player is
// then -1 and the reset kernels draw the seat (rng.hpp start_seat).  Elsewhere such rules are MUZ_E_UNSUPPORTED.
static inline int make_det_consts(const muz_rules* r, DetConsts* c, bool allow_random_start = false) {
  if (!r || !c) return MUZ_E_INVALID;
  const int P = r->num_players;
  if (P < 2 || P > 4) return MUZ_E_UNSUPPORTED;
  if (r->distance != kDist) return MUZ_E_UNSUPPORTED;
  const bool random_start = r->starting_player < 0 || r->starting_player >= P;
  if (random_start && !allow_random_start) return MUZ_E_UNSUPPORTED;
  bool layout[4];
  int nset = 0, nall = 1;
  for (int i = 0; i < 4; ++i) {
    layout[i] = r->layout[i] != 0;
    nset += layout[i] ? 1 : 0;
    nall &= layout[i] ? 1 : 0;
  }
  if (nset != P || (nall && P < 4))
    for (int i = 0; i < 4; ++i) layout[i] = i < P;
  c->P = P;
  c->starting_player = random_start ? -1 : r->starting_player;
  uint32_t f = 0;
  if (r->enable_teams && P == 4) f |= R_TEAMS;
  if (r->enable_initial_free_pin) f |= R_FREE_PIN;
  if (r->enable_circular_board) f |= R_CIRCULAR;
  if (r->enable_start_blocking) f |= R_START_BLOCK;
  if (r->enable_jump_in_goal_area) f |= R_JUMP_GOAL;
  if (r->enable_friendly_fire) f |= R_FRIENDLY;
  if (r->enable_start_on_1) f |= R_START_ON_1;
  if (r->enable_bonus_turn_on_6) f |= R_BONUS_6;
  if (r->must_traverse_start) f |= R_MUST_TRAVERSE;
  if (r->enable_dice_rethrow) f |= R_DICE_RETHROW;
  c->flags = f;
  int p = 0;
  for (int i = 0; i < 4; ++i) {
    c->start[i] = 0;
    c->target[i] = 0;
    for (int g = 0; g < 4; ++g) c->goal[i][g] = kTrack;
  }
  for (int i = 0; i < 4; ++i) {
    if (!layout[i]) continue;
    c->start[p] = i * kDist;
    c->target[p] = ((i * kDist - 1) % kTrack + kTrack) % kTrack;
    for (int g = 0; g < 4; ++g) c->goal[p][g] = kTrack + 4 * i + g;
    ++p;
  }
  return MUZ_OK;
}

}  // namespace muz
