/*
 * muz.h -- C ABI of libmuz.so, the MI355X-native MuZero self-play engine.
 *
 * Drop-in boundary for the reference's hot path (marco-wojtek/Exploring-MuZero-on-DOG).
 * The reference is pure JAX; every function below replaces one of its functional
 * entry points (file:line relative to the reference root) with a batched,
 * stream-ordered HIP launch over caller-owned device buffers.
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless a comment says "host".
 *   - Buffers are owned by the caller (PyTorch tensors in the Python host);
 *     the library owns only opaque workspaces created/destroyed explicitly.
 *   - Every function returns 0 (MUZ_OK) or an error code; hipError_t values are
 *     passed through unchanged, library errors are >= MUZ_E_BASE.  Nothing aborts.
 *   - Illegal actions are NOT errors: they keep the reference semantics
 *     (reward -1, board unchanged, turn passes -- deterministic_madn.py:186,242-246).
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream).
 *   - State is struct-of-arrays, FIELD-MAJOR: element (field c, game b) lives at
 *     ptr[c * stride + b].  One board per wavefront lane.
 */
#ifndef MUZ_H_
#define MUZ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MUZ_OK 0
#define MUZ_E_BASE 10000
#define MUZ_E_INVALID (MUZ_E_BASE + 1)     /* bad argument (null pointer, n < 0, ...) */
#define MUZ_E_UNSUPPORTED (MUZ_E_BASE + 2) /* configuration outside what the kernels implement */

#define MUZ_DET_ACTIONS 24   /* pin*6 + (move-1), deterministic_madn.py:469-479 */
#define MUZ_BOARD_CELLS 56   /* 4*distance + 16 goal cells at distance 10 */

/* Rule set (deterministic_madn.py:42-58 keyword arguments).  Flags are 0/1. */
typedef struct muz_rules {
  int32_t num_players;        /* 2..4 */
  int32_t distance;           /* must be 10 (board of 56 cells) */
  int32_t layout[4];          /* seat mask; fixed up exactly like env_reset:70-74 */
  int32_t starting_player;    /* 0 <= s < num_players (random start is not restated) */
  int32_t enable_teams;
  int32_t enable_initial_free_pin;
  int32_t enable_circular_board;
  int32_t enable_start_blocking;
  int32_t enable_jump_in_goal_area;
  int32_t enable_friendly_fire;
  int32_t enable_start_on_1;
  int32_t enable_bonus_turn_on_6;
  int32_t must_traverse_start;
} muz_rules;

/* Deterministic-MADN batch state, SoA (deterministic_madn.py:24-40).
 * start/target/goal are rule constants and are not stored per game. */
typedef struct muz_detmadn_soa {
  int8_t* board;          /* [56][stride]       -1 empty, else player id         */
  int8_t* pins;           /* [P*4][stride]      -1 home, 0..39 track, 40..55 goal */
  int8_t* current_player; /* [stride]                                             */
  int8_t* reward;         /* [stride]                                             */
  uint8_t* done;          /* [stride]                                             */
  int8_t* action_set;     /* [P*6][stride]      remaining copies of moves 1..6    */
  int32_t stride;         /* >= n                                                 */
} muz_detmadn_soa;

/* ---- library ---------------------------------------------------------------- */
const char* muz_version(void);                 /* host string */
const char* muz_error_string(int code);        /* host string */

/* ---- deterministic MADN environment ----------------------------------------- */

/* env_reset (deterministic_madn.py:42-120) for games [0, n); game_agent.py:24-44 batch_reset. */
int muz_detmadn_reset(const muz_rules* rules /*host*/, muz_detmadn_soa state, int32_t n, void* stream);

/* valid_action (deterministic_madn.py:299-393): legal_bits[b] bit (pin*6+move-1). */
int muz_detmadn_legal(const muz_rules* rules, muz_detmadn_soa state, uint32_t* legal_bits, int32_t n,
                      void* stream);

/* env_step (deterministic_madn.py:170-257) with action index a -> map_action(a) = (a/6, a%6+1).
 * reward/done/next_legal may be null.  next_legal = valid_action of the NEW state (fused). */
int muz_detmadn_step(const muz_rules* rules, muz_detmadn_soa state, const int32_t* action, int8_t* reward,
                     uint8_t* done, uint32_t* next_legal, int32_t n, void* stream);

/* env_step with an explicit (pin, move) pair per game, move in 1..6 (MADN/test.py:932-945 calls this form). */
int muz_detmadn_step_pin_move(const muz_rules* rules, muz_detmadn_soa state, const int32_t* pin,
                              const int32_t* move, int8_t* reward, uint8_t* done, int32_t n, void* stream);

/* no_step (deterministic_madn.py:283-297). reward (always 0) / done may be null. */
int muz_detmadn_nostep(const muz_rules* rules, muz_detmadn_soa state, int8_t* reward, uint8_t* done, int32_t n,
                       void* stream);

/* encode_board (deterministic_madn.py:395-438): obs[b][c][w], C = 8P+2 channels, W = 56. */
int muz_detmadn_encode_f32(const muz_rules* rules, muz_detmadn_soa state, float* obs, int32_t n, void* stream);
int muz_detmadn_encode_i8(const muz_rules* rules, muz_detmadn_soa state, int8_t* obs, int32_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MUZ_H_ */
