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
  int32_t starting_player;    /* 0 <= s < num_players, or out of range = a random seat per game (env_reset's
                                 jax randint, restated on the counter RNG: see muz_detmadn_reset_seeded); accepted
                                 by the seeded resets and every DOG entry point, MUZ_E_UNSUPPORTED elsewhere */
  int32_t enable_teams;
  int32_t enable_initial_free_pin;
  int32_t enable_circular_board;
  int32_t enable_start_blocking;
  int32_t enable_jump_in_goal_area;
  int32_t enable_friendly_fire;
  int32_t enable_start_on_1;
  int32_t enable_bonus_turn_on_6;
  int32_t must_traverse_start;
  int32_t enable_dice_rethrow;  /* classic only (classic_madn.py:66, dice_probabilities 208-228) */
  int32_t disable_swapping;     /* DOG only (dog.py:83-100); the device implements the full 14-card game, */
  int32_t disable_hot_seven;    /* so a non-zero value is MUZ_E_UNSUPPORTED for the DOG entry points       */
  int32_t disable_joker;
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

/* Classic-MADN batch state, SoA (classic_madn.py:33-49): the det fields without the action set, plus
 * the die of the turn (set by muz_classic_set_die / muz_classic_throw_die before legal / step). */
typedef struct muz_classic_soa {
  int8_t* board;          /* [56][stride] */
  int8_t* pins;           /* [P*4][stride] */
  int8_t* current_player; /* [stride] */
  int8_t* reward;         /* [stride] */
  uint8_t* done;          /* [stride] */
  int8_t* die;            /* [stride]       1..6 (0 after reset) */
  int32_t stride;
} muz_classic_soa;

#define MUZ_CLASSIC_ACTIONS 4   /* pin index */

/* ---- library ---------------------------------------------------------------- */
const char* muz_version(void);                 /* host string */
const char* muz_error_string(int code);        /* host string */

/* ---- deterministic MADN environment ----------------------------------------- */

/* env_reset (deterministic_madn.py:42-120) for games [0, n); game_agent.py:24-44 batch_reset. */
int muz_detmadn_reset(const muz_rules* rules /*host*/, muz_detmadn_soa state, int32_t n, void* stream);

/* valid_action (deterministic_madn.py:299-393): legal_bits[b] bit (pin*6+move-1). */
/* env_reset with the reference's seed argument (deterministic_madn.py:42-62): as muz_detmadn_reset, and when
 * rules->starting_player is out of range each game's seat is drawn from its seed seeds[g] (the reference draws it
 * with jax.random.randint(split(PRNGKey(seed))[1], (), 0, P); here floor(U * P) of the counter RNG of the seed --
 * threefry is not restated, so the seat a seed gives differs from jax's; the distribution is the same). */
int muz_detmadn_reset_seeded(const muz_rules* rules /*host*/, muz_detmadn_soa state, const int32_t* seeds, int32_t n,
                             void* stream);
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

/* One env-step of uniform random legal play for every game (the env-only micro-benchmark of SURVEY §8(d)(b'),
 * and a random-play actor): legal_bits holds each game's mask on entry (muz_detmadn_legal before the first
 * round) and the next round's mask on exit; the action is the k-th legal one, k = floor(u * count), u =
 * (mix64(game_key(seed ^ 0xD37A11D0, g, turn)) >> 40) / 2^24; no_step when nothing is legal; a game that
 * finishes is reset in place (done[g] = 1 for that round).  obs (nullable) receives encode_board of the state
 * the next round acts on, int8 [n][8P+2][56], 16-byte aligned (else MUZ_E_INVALID).  Replaces the vmapped valid_action -> env_step / no_step ->
 * encode_board sequence of MuZero_det_MADN/game_agent.py:84-119 (MADN/deterministic_madn.py:170-438). */
int muz_detmadn_random_round(const muz_rules* rules, muz_detmadn_soa state, uint32_t* legal_bits, uint64_t seed,
                             int32_t turn, int8_t* obs, int8_t* reward, uint8_t* done, int32_t n, void* stream);
/* The same round with the kernel chosen explicitly: variant 1 = one game per lane (k_det_round, for batches that
 * fill the GPU), 2 / 3 / 4 / 5 = one game per 32 / 8 / 4 / 16 lanes (k_det_round_g<G>), 0 = by batch size (as
 * muz_detmadn_random_round).  Identical results. */
int muz_detmadn_random_round_variant(const muz_rules* rules, muz_detmadn_soa state, uint32_t* legal_bits,
                                     uint64_t seed, int32_t turn, int8_t* obs, int8_t* reward, uint8_t* done,
                                     int32_t n, int32_t variant, void* stream);

/* Evaluation agents of MuZero_det_MADN/evaluate_agent.py: mode 0 = the random agent (do_random, 770-775),
 * mode 1 = the rule-based agent (do_rule_based, 777-864; weights in `agent`, the reference's
 * {0.25, 5.0, 3.0, 2.0, 2.0}; the multiactor_step variant 509-603 uses {0.5, 5.0, 3.0, 1.5, 2.5}).  Both
 * sample jax.random.categorical as argmax(logits + Gumbel) with the Gumbel draw of the counter RNG
 * (seed ^ 0x9011C7A6E47, game_id[g] (or g), turn, action).  action[g] = -1 when legal_bits[g] == 0. */
typedef struct muz_rule_agent {
  float temperature;   /* softmax temperature of the scores */
  float goal_bonus;    /* landing on an own goal cell from outside the goal area */
  float out_many;      /* leaving home with >= 2 pins at home */
  float out_few;       /* leaving home with < 2 pins at home */
  float hit_bonus;     /* moving onto an opponent pin */
} muz_rule_agent;
int muz_detmadn_policy_action(const muz_rules* rules, muz_detmadn_soa state, const uint32_t* legal_bits, int32_t mode,
                              const muz_rule_agent* agent /*host, mode 1*/, uint64_t seed, int32_t turn,
                              const int32_t* game_id, int32_t* action, int32_t n, void* stream);


/* ---- classic MADN environment (MADN/classic_madn.py) -------------------------------------- */

/* env_reset (classic_madn.py:51-131); game_agent_stochastic.py:25-44 batch_reset. */
int muz_classic_reset(const muz_rules* rules /*host*/, muz_classic_soa state, int32_t n, void* stream);

/* set_die (classic_madn.py:244-255): die[b] (1..6) into the state. */
/* env_reset with the reference's seed argument (classic_madn.py:51-72): random seat as muz_detmadn_reset_seeded. */
int muz_classic_reset_seeded(const muz_rules* rules /*host*/, muz_classic_soa state, const int32_t* seeds, int32_t n,
                             void* stream);
int muz_classic_set_die(const muz_rules* rules, muz_classic_soa state, const int32_t* die, int32_t n, void* stream);

/* dice_probabilities (208-228) -> probs[b][6] fp32; soft_locked[b] (is_soft_locked 180-206) may be null. */
int muz_classic_dice_probs(const muz_rules* rules, muz_classic_soa state, float* probs, uint8_t* soft_locked,
                           int32_t n, void* stream);

/* throw_die (230-242) with the uniform draw as an input: die = jax.random.choice([1..6], p=dice_probabilities)
 * evaluated as 1 + searchsorted_left(cumsum(p), cumsum(p)[5] * (1 - uniform[b])).  die_out may be null. */
int muz_classic_throw_die(const muz_rules* rules, muz_classic_soa state, const float* uniform, int32_t* die_out,
                          int32_t n, void* stream);

/* valid_action (367-461): legal_bits[b] bit pin (4 bits), for the die in the state. */
int muz_classic_legal(const muz_rules* rules, muz_classic_soa state, uint32_t* legal_bits, int32_t n, void* stream);

/* env_step (257-337) moving pin[b] by the state's die.  reward/done may be null. */
int muz_classic_step(const muz_rules* rules, muz_classic_soa state, const int32_t* pin, int8_t* reward,
                     uint8_t* done, int32_t n, void* stream);

/* no_step (353-365): advance the player. */
int muz_classic_nostep(const muz_rules* rules, muz_classic_soa state, int8_t* reward, uint8_t* done, int32_t n,
                       void* stream);

/* encode_board (463-497): obs[b][c][w], C = 2P+3 (last channel = die), W = 56. */
/* The classic evaluation agents of MuZero_Classic_MADN/evaluate_agent_stochastic.py play_eval_loop_jitted (the harness
 * evaluate_agent_parallel runs): mode 0 = the random agent (do_random, 800-804), mode 1 = the rule-based agent
 * (do_rule_based, 806-866: per pin goal / out-of-home / hit bonuses for the landing cell of cur + die, base score 0;
 * the reference's weights {0.25, 5.0, 3.0, 2.0, 2.5}).  Sampling as muz_detmadn_policy_action (argmax(logits +
 * Gumbel), the same counter draws for actions 0..3).  legal_bits: muz_classic_legal's 4-bit masks for the die in the
 * state; action[g] = -1 when no pin is legal. */
int muz_classic_policy_action(const muz_rules* rules, muz_classic_soa state, const uint32_t* legal_bits, int32_t mode,
                              const muz_rule_agent* agent /*host, mode 1*/, uint64_t seed, int32_t turn,
                              const int32_t* game_id, int32_t* action, int32_t n, void* stream);
int muz_classic_encode_f32(const muz_rules* rules, muz_classic_soa state, float* obs, int32_t n, void* stream);
int muz_classic_encode_i8(const muz_rules* rules, muz_classic_soa state, int8_t* obs, int32_t n, void* stream);

/* ---- DOG environment (DOG/dog.py + utils/utility_funcs.py) ---------------------------------
 * Action layout (806): [0,396) joker copies, [396,792) real-card copies, each = swaps pin*56+pos [0,224),
 * hot-7 distribution all_pin_distributions(7)[i] [224,344), normal pin*12+(move index over 1..6,8..13)
 * [344,392), -4 pin [392,396); [792,806) swap-phase card.  Masks are bitsets uint32[n][26] (bit a%32 of
 * word a/32).  The deck shuffle draws its 120 keys from a counter RNG instead of jax threefry:
 *   key_k = U24(mix64(seed ^ 0xDEA1C0DE5EED ^ mix64(game << 32 | deal) ^ (k+1) * 0xA24BAED4963EE407)),
 * deal = number of distribute_cards calls so far (oracle/dog.py:engine_shuffle_keys restates it). */
typedef struct muz_dog_soa {
  int8_t* board;          /* [56][stride] */
  int8_t* pins;           /* [P*4][stride]  (the reference keeps int32; values -1..55) */
  int8_t* deck;           /* [14][stride] */
  int8_t* hands;          /* [P*14][stride] */
  int8_t* swap_choices;   /* [4][stride] */
  int8_t* current_player; /* [stride] */
  int8_t* round_starter;  /* [stride] */
  int8_t* phase;          /* [stride]  0 play, 1 swap */
  int8_t* hand_size;      /* [stride]  size of the NEXT deal */
  int8_t* reward;         /* [stride] */
  uint8_t* done;          /* [stride] */
  uint32_t* deal;         /* [stride]  distribute_cards calls (the jax key's role) */
  int32_t stride;
} muz_dog_soa;

#define MUZ_DOG_ACTIONS 806
#define MUZ_DOG_MASK_WORDS 26

/* env_reset (dog.py:83-186) + the first distribute_cards (201-298) for games [0, n). */
int muz_dog_reset(const muz_rules* rules /*host*/, muz_dog_soa state, uint64_t seed, int32_t n, void* stream);

/* valid_actions (dog.py:693-711) -> mask[n][26]. */
int muz_dog_legal(const muz_rules* rules, muz_dog_soa state, uint32_t* mask, int32_t n, void* stream);

/* env_step (dog.py:1117-1131) with action[b] in [0, 806); a negative action applies no_step instead.
 * A deal that follows draws from `seed`.  reward / done may be null. */
int muz_dog_step(const muz_rules* rules, muz_dog_soa state, const int32_t* action, uint64_t seed, int8_t* reward,
                 uint8_t* done, int32_t n, void* stream);

/* no_step (dog.py:713-752). */
/* muz_dog_step for the self-play loop: env_step(action[g]) (no_step when action[g] < 0), then a game the step
 * finished restarts in place (env_reset with the deal counter continued, as muz_dog_random_play's auto reset);
 * reward / done are the step's, episodes[g] (nullable) counts the restarts. */
int muz_dog_step_restart(const muz_rules* rules /*host*/, muz_dog_soa state, const int32_t* action, uint64_t seed,
                         int8_t* reward, uint8_t* done, uint32_t* episodes, int32_t n, void* stream);
int muz_dog_nostep(const muz_rules* rules, muz_dog_soa state, uint64_t seed, int8_t* reward, uint8_t* done,
                   int32_t n, void* stream);

/* Config (d)'s actor turn in one launch: valid_actions -> the random legal action of muz_dog_random_action
 * (counter uniform, stream `seed`, `turn`) -> env_step, or no_step when nothing is legal.  Games already
 * done are not touched (action -2, reward 0, done 1).  action / reward / done may be null. */
int muz_dog_random_turn(const muz_rules* rules, muz_dog_soa state, uint64_t seed, int32_t turn, int32_t* action,
                        int8_t* reward, uint8_t* done, int32_t n, void* stream);

/* `nturns` consecutive muz_dog_random_turn turns (turn0, turn0+1, ...) in ONE launch: each workgroup keeps
 * its game resident in LDS for all turns.  A finished game stops, or with auto_reset != 0 restarts in place
 * (env_reset + first deal, the deal counter continued so the new episode draws new keys) and keeps playing.
 * env_steps[b] / episodes[b] (may be null) += turns played / games finished.  Without auto_reset the states
 * equal nturns separate muz_dog_random_turn calls. */
int muz_dog_random_play(const muz_rules* rules, muz_dog_soa state, uint64_t seed, int32_t turn0, int32_t nturns,
                        int32_t auto_reset, uint32_t* env_steps, uint32_t* episodes, int32_t n, void* stream);

/* Per-turn records of the DOG actor (config (d)'s "trajectories"; the reference's DOG agent is a stub,
 * MuZero_DOG/game_agent.py:52-57, so this minimal record is this engine's own and parity-unpinned): row
 * idx[b] + t of game lane b holds the turn's action (-1 = no legal action, no_step), the player who moved
 * (current player before the move), the reward, the number of legal actions and whether the game finished
 * on it (with auto_reset the next row starts the new game).  idx[b] advances by the turns played, capped at
 * max_steps (rows past it are dropped). */
typedef struct muz_dog_traj {
  int32_t* act;      /* [n][max_steps] */
  int32_t* player;   /* [n][max_steps] */
  int32_t* reward;   /* [n][max_steps] */
  int32_t* legal;    /* [n][max_steps] */
  uint8_t* done;     /* [n][max_steps] */
  int32_t* idx;      /* [n] rows recorded (in / out) */
  int32_t max_steps;
} muz_dog_traj;
/* muz_dog_random_play that also writes the per-turn records into `rec` (all pointers non-null). */
int muz_dog_random_play_record(const muz_rules* rules, muz_dog_soa state, uint64_t seed, int32_t turn0, int32_t nturns,
                               int32_t auto_reset, uint32_t* env_steps, uint32_t* episodes, muz_dog_traj rec, int32_t n,
                               void* stream);

/* One step function on its own, the form DOG/test.py calls (dog.py:754-984): kind[b] 0 step_swap(pin, pos),
 * 1 step_normal_move(pin, move), 2 step_neg_move(pin, move), 3 step_hot_7(dist); args[b][4] = (pin, pos|move,
 * -, -) or dist[4].  Writes board and pins; reward / done (may be null) are the function's results. */
int muz_dog_step_move(const muz_rules* rules, muz_dog_soa state, const int32_t* kind, const int32_t* args,
                      int8_t* reward, uint8_t* done, int32_t n, void* stream);

/* Uniform random legal action (SURVEY config (d) policy): the k-th set bit of mask[b], k = floor(u * count),
 * u = uniform[b] or, when uniform is null, U24(mix64(seed ^ 0x52A4D0DA11 ^ mix64(b << 32 | turn))).
 * -1 when the mask is empty (the caller then applies no_step). */
int muz_dog_random_action(const uint32_t* mask, const float* uniform, uint64_t seed, int32_t turn, int32_t* action,
                          int32_t n, void* stream);

/* ---- MuZero networks (MuZero_det_MADN/muzero_deterministic_madn.py) --------------------------
 * Dense layers used by the MFMA kernels take their kernel W[K][N] PACKED for
 * v_mfma_f32_16x16x4_f32 B-fragments: [group][K/16][lane 64][tile NT][j 4] (group = wave, see muz_tile_waves) with
 * element = W[kb*16 + 4*(lane>>4) + j][(group*NT + t)*16 + (lane&15)], zero padded
 * (exploring-muzero-on-dog_amd/nets.py:pack_dense).  Layers marked "plain" are row-major [K][N].
 * Biases / LayerNorm scale+bias are plain fp32 vectors. */
typedef struct muz_dense { const float* w; const float* b; } muz_dense;
typedef struct muz_ln { const float* scale; const float* bias; } muz_ln;
typedef struct muz_resblock { muz_dense d0; muz_ln ln0; muz_dense d1; muz_ln ln1; } muz_resblock;

/* RepresentationNetwork2 (lines 75-141) */
typedef struct muz_repr_w {
  muz_dense conv0;              /* plain [3][6][32] */
  muz_ln ln0;
  muz_dense conv1;              /* packed, 4 groups x 1 tile, K=96  N=64 */
  muz_ln ln1;
  muz_dense conv2;              /* packed, 4 groups x 1 tile, K=320 N=64 */
  muz_ln ln2;
  muz_dense d0;                 /* packed 3584 -> 256 */
  muz_ln ln3;
  muz_dense d1;                 /* packed (C-6) -> 64 (K zero-padded to 16) */
  muz_ln ln4;
  muz_dense d2;                 /* packed 64 -> 64 */
  muz_ln ln5;
  muz_dense d3;                 /* packed 320 -> 256 */
  muz_ln ln6;
  muz_resblock rb[6];
  muz_dense d4;                 /* packed 256 -> 256 */
} muz_repr_w;

/* DynamicsNetwork4 (lines 391-457) */
typedef struct muz_dyn_w {
  muz_dense d0;                 /* plain [A][64]: one_hot(action) @ W = row gather */
  muz_ln ln0;
  muz_dense d12;                /* packed, Dense_1 | Dense_2 fused: 64 -> 512 (FiLM scale | shift) */
  muz_dense d3;
  muz_ln ln1;
  muz_dense d4;
  muz_ln ln2;
  muz_resblock rb[2];
  muz_dense d5;
  muz_dense d67;                /* packed, Dense_6 | Dense_7 latent rows fused: 256 -> 128 */
  const float* d67_onehot;      /* plain [A][128]: one-hot rows 256.. of Dense_6 | Dense_7 */
  muz_dense reward_head;        /* plain [64][3] */
  muz_dense discount_head;      /* plain [64][3] */
  float* film;                  /* derived [A+1][512], filled by muz_net_prepare: FiLM scale | shift of
                                   each action (lines 399-411 depend on the action only); row A = the
                                   zero one-hot of an out-of-range action */
} muz_dyn_w;

/* PredictionNetwork4 (lines 549-583) */
typedef struct muz_pred_w {
  muz_ln ln0;
  muz_resblock rb[2];
  muz_dense d03;                /* packed, Dense_0 | Dense_3 fused: 256 -> 384 */
  muz_ln ln1;
  muz_dense d1;                 /* packed 256 -> 128 */
  muz_ln ln2;
  muz_dense d2;                 /* packed 128 -> A */
  muz_ln ln3;
  muz_dense d4;                 /* packed 128 -> 64 */
  muz_dense d5;                 /* plain [64][1] */
} muz_pred_w;

typedef struct muz_net_w {
  int32_t obs_channels;         /* C = 8P+2 */
  int32_t num_actions;          /* 24 */
  muz_repr_w repr;
  muz_dyn_w dyn;
  muz_pred_w pred;
} muz_net_w;

/* Waves per 16-row tile workgroup the kernels were built for = number of column groups in the packed
 * layout of every 16-row dense layer (the host packs weights with this value). */
int32_t muz_tile_waves(void);

/* Fills the derived tables of a weight set (dyn.film) from its raw layers; call once after the weights
 * change and before any muz_nets_recurrent / muz_gumbel_search / muz_detmadn_selfplay on them.
 * Replaces nothing in the reference: the FiLM sub-graph of DynamicsNetwork4.__call__
 * (MuZero_det_MADN/muzero_deterministic_madn.py:398-411) depends on the action only, so it is
 * evaluated once per action instead of once per simulation. */
int muz_net_prepare(const muz_net_w* w, void* stream);

/* Scratch bytes muz_nets_root needs for n observations (conv feature maps). */
int64_t muz_nets_root_scratch_bytes(int32_t n);

/* root_inference_fn (lines 621-630): obs [n][C][56] fp32 -> prior_logits [n][A], value [n], embedding [n][256]. */
int muz_nets_root(const muz_net_w* w /*host*/, const float* obs, int32_t n, void* scratch, int64_t scratch_bytes,
                  float* prior_logits, float* value, float* embedding, void* stream);

/* recurrent_inference_fn (lines 632-661): (action [n], embedding [n][256]) ->
 * reward [n], discount [n] (E[softmax(logits)]·{-1,0,1}), prior_logits [n][A], value [n], next_embedding [n][256]. */
int muz_nets_recurrent(const muz_net_w* w /*host*/, const int32_t* action, const float* embedding, int32_t n,
                       float* reward, float* discount, float* prior_logits, float* value, float* next_embedding,
                       void* stream);

/* ---- Gumbel MuZero search (run_muzero_mcts, muzero_deterministic_madn.py:663-704 -> mctx 0.0.6) ---- */
typedef struct muz_search_cfg {
  int32_t num_simulations;      /* S */
  int32_t max_depth;            /* D */
  int32_t max_num_considered;   /* 16 (mctx default) */
  float value_scale;            /* 0.5 (qtransform_completed_by_mix_value) */
  float maxvisit_init;          /* 50 */
  float gumbel_scale;           /* = temperature */
  uint64_t seed;                /* used only when gumbel == NULL */
  int32_t turn;                 /* mixed into the noise counter when gumbel == NULL */
} muz_search_cfg;

/* Workspace bytes for n searches (tree arrays + node embeddings). */
int64_t muz_search_workspace_bytes(int32_t n, const muz_search_cfg* cfg /*host*/);

/* Batched gumbel_muzero_policy.  legal_bits: 24-bit valid_action masks (invalid = ~legal).
 * gumbel [n][A] already scaled by gumbel_scale, or NULL to draw it on device from (seed, game_id, turn).
 * game_id [n] (nullable: identity) only feeds the device noise counter.
 * Outputs: action [n], action_weights [n][A] (softmax of masked prior+completedQ), root_value [n]. */
int muz_gumbel_search(const muz_net_w* w /*host*/, const muz_search_cfg* cfg /*host*/, const float* root_logits,
                      const float* root_value, const float* root_embedding, const uint32_t* legal_bits,
                      const float* gumbel, const int32_t* game_id, int32_t n, void* workspace,
                      int64_t workspace_bytes, int32_t* action, float* action_weights, float* root_value_out,
                      void* stream);

/* ---- self-play (MuZero_det_MADN/game_agent.py:50-192) ----------------------------------------------
 * Trajectory buffers [n][T] per game, T = max_steps, mirroring play_batch_of_games_jitted's dict
 * (game_agent.py:158-169); obs is stored int8 (values 0..4, the reference keeps them as fp32). */
typedef struct muz_traj {
  int8_t* obs;        /* [n][T][C][56] */
  int32_t* act;       /* [n][T]  action index, -1 on no-move turns */
  int32_t* rew;       /* [n][T]  reward class {0:-1, 1:0, 2:+1} */
  float* val;         /* [n][T]  root value (search_tree.summary().value) */
  float* pol;         /* [n][T][A] action_weights (A = 24 det, 4 classic) */
  float* mask;        /* [n][T]  1 = search turn, 0 = no-move turn */
  int32_t* player;    /* [n][T]  current player before the move */
  int32_t* team;      /* [n][T]  player % 2 with teams, else -1 */
  int32_t* discount;  /* [n][T]  discount class {0: other side moves next, 1: terminal, 2: same side} */
  int32_t* idx;       /* [n]     recorded steps per game */
  int32_t max_steps;  /* T */
} muz_traj;

/* Optional per-call statistics (host struct).  search_ms sums HIP-event durations of the search
 * kernel launches (events are recorded only when stats != NULL). */
typedef struct muz_sp_stats {
  int32_t turns;      /* batched turns that found an active game */
  int64_t searches;   /* MCTS searches run (sum over turns of games with a legal move) */
  double search_ms;   /* device time of the Gumbel-search launches */
  double total_ms;    /* device time of the whole call */
} muz_sp_stats;

int64_t muz_selfplay_workspace_bytes(int32_t n, int32_t obs_channels, const muz_search_cfg* cfg /*host*/);

/* play_n_games_v3 + play_batch_of_games_jitted: reset n games (rules->starting_player), then play
 * until every game is done or max_steps turns ran.  Searches use cfg (S, D, temperature = gumbel_scale,
 * device Gumbel noise from cfg->seed).  stats (host, nullable) receives turns / searches / timings.  The
 * workspace and traj.obs must be 16-byte aligned (else MUZ_E_INVALID; the same for the streaming form). */
int muz_detmadn_selfplay(const muz_rules* rules /*host*/, const muz_net_w* w /*host*/,
                         const muz_search_cfg* cfg /*host*/, muz_detmadn_soa state, muz_traj traj, int32_t n,
                         void* workspace, int64_t workspace_bytes, muz_sp_stats* stats /*host*/, void* stream);

/* The same self-play, streamed: num_games games through `lanes` concurrently played lanes (state stride
 * >= lanes, workspace = muz_selfplay_workspace_bytes(lanes, ...)).  Lane l starts game l; whenever a game
 * ends (done, or max_steps recorded) its lane takes the next game number (deterministic, lane order) and
 * is reset, so the search batch stays full until the last games.  traj is [num_games][T]; game k's
 * record, including its Gumbel noise (keyed by game number and the game's own step), is identical to
 * game k of a muz_detmadn_selfplay batch of num_games games. */
int muz_detmadn_selfplay_stream(const muz_rules* rules /*host*/, const muz_net_w* w /*host*/,
                                const muz_search_cfg* cfg /*host*/, muz_detmadn_soa state, muz_traj traj,
                                int32_t num_games, int32_t lanes, void* workspace, int64_t workspace_bytes,
                                muz_sp_stats* stats /*host*/, void* stream);

/* ---- Stochastic MuZero for classic MADN (MuZero_Classic_MADN/muzero_classic_madn.py) ----------
 * Same packing conventions as the det networks.  RepresentationNetwork2 (69-135) and
 * PredictionNetwork4 (192-226, A = 4) reuse muz_repr_w / muz_pred_w. */

/* StochasticDynamicsNetwork4 (314-408). */
typedef struct muz_sdyn_w {
  /* action_dynamics (329-371) */
  muz_dense act_embed;          /* plain [A][64] */
  muz_ln act_input_ln;
  muz_dense act_film;           /* packed, act_film_scale | act_film_shift fused: 64 -> 512 */
  muz_dense act_dense1;
  muz_ln act_ln1;
  muz_dense act_dense2;
  muz_ln act_ln2;
  muz_resblock act_rb[2];
  muz_dense act_proj;
  muz_dense rc;                 /* packed, reward_dense afterstate rows | chance_head fused: 256 -> 70 */
  const float* reward_onehot;   /* plain [A][64]: one-hot rows 256.. of reward_dense */
  muz_dense reward_head;        /* plain [64][3] */
  muz_dense discount_dense;     /* packed 256 -> 32, applied to the INPUT latent (366) */
  muz_ln discount_ln;           /* 32 */
  muz_dense discount_head;      /* plain [32][3] */
  /* chance_dynamics (373-408) */
  muz_dense chance_embed;       /* plain [6][64] */
  muz_ln chance_input_ln;
  muz_dense chance_film;        /* packed 64 -> 512 */
  muz_dense chance_dense1;
  muz_ln chance_ln1;
  muz_dense chance_dense2;
  muz_ln chance_ln2;
  muz_resblock chance_rb[2];
  muz_dense chance_proj;
  float* act_film_tab;          /* derived [A+1][512]  (muz_classic_net_prepare) */
  float* chance_film_tab;       /* derived [6+1][512] */
} muz_sdyn_w;

typedef struct muz_classic_net_w {
  int32_t obs_channels;         /* 2P+3 */
  int32_t num_actions;          /* 4 */
  muz_repr_w repr;
  muz_sdyn_w sdyn;
  muz_pred_w pred;
} muz_classic_net_w;

#define MUZ_CHANCE_OUTCOMES 6

/* Fills sdyn.act_film_tab / chance_film_tab from the raw layers (the FiLM sub-graphs depend on the
 * action / chance outcome only).  Call after the weights change. */
int muz_classic_net_prepare(const muz_classic_net_w* w, void* stream);

/* root_inference_fn (453-462): Repr2 + Pred4 -> prior_logits [n][4], value [n], embedding [n][256]. */
int muz_classic_nets_root(const muz_classic_net_w* w, const float* obs, int32_t n, void* scratch,
                          int64_t scratch_bytes, float* prior_logits, float* value, float* embedding, void* stream);

/* decision_recurrent_fn (414-432): afterstate [n][256], reward / discount [n] (support expectations the
 * reference appends to the afterstate), chance_logits [n][6], afterstate_value [n]. */
int muz_classic_nets_decision(const muz_classic_net_w* w, const int32_t* action, const float* embedding, int32_t n,
                              float* afterstate, float* reward, float* discount, float* chance_logits,
                              float* afterstate_value, void* stream);

/* chance_recurrent_fn (434-451): next_embedding [n][256], action_logits [n][4], value [n]. */
int muz_classic_nets_chance(const muz_classic_net_w* w, const int32_t* chance, const float* afterstate, int32_t n,
                            float* next_embedding, float* action_logits, float* value, void* stream);

/* mctx.stochastic_muzero_policy as called by run_stochastic_muzero_mcts (464-517). */
typedef struct muz_stoch_cfg {
  int32_t num_simulations;      /* S <= 100 */
  int32_t max_depth;            /* D <= 64 */
  float dirichlet_fraction;     /* 0.25 */
  float dirichlet_alpha;        /* 0.3 */
  float pb_c_init;              /* 1.25 */
  float pb_c_base;              /* 19652 */
  float temperature;
  int32_t turn;                 /* counter-RNG stream */
  uint64_t seed;
} muz_stoch_cfg;

int64_t muz_stochastic_workspace_bytes(int32_t n, int32_t num_simulations);

/* root: prior_logits [n][4], value [n], embedding [n][256] (muz_classic_nets_root); legal_bits bit a = pin a
 * legal.  dirichlet [n][4] / gumbel [n][4] are the root noise sample and the Gumbel draws of the final
 * categorical; null = the engine's counter RNG (Gamma(alpha) sampler / -log(-log U)).  The 1e-7
 * tie-break uniforms always come from the counter RNG (seed, game, turn, sim, depth, action).
 * Outputs: action [n], action_weights [n][4] (visit distribution), root_value [n] clipped to [-1, 1]. */
int muz_stochastic_search(const muz_classic_net_w* w, const muz_stoch_cfg* cfg, const float* root_logits,
                          const float* root_value, const float* root_embedding, const uint32_t* legal_bits,
                          const float* dirichlet, const float* gumbel, const int32_t* game_id, int32_t n,
                          void* workspace, int64_t workspace_bytes, int32_t* action, float* action_weights,
                          float* root_value_out, void* stream);

/* Chance records of the stochastic self-play buffers (game_agent_stochastic.py:165-172). */
typedef struct muz_traj_chance {
  int32_t* dice;      /* [n][T]     die of the turn (1..6) */
  float* dice_dist;   /* [n][T][6]  dice_probabilities of the state AFTER the turn (line 162) */
} muz_traj_chance;

int64_t muz_classic_selfplay_workspace_bytes(int32_t n, int32_t obs_channels, const muz_stoch_cfg* cfg /*host*/);

/* play_n_games_v3 + play_batch_of_games_jitted of MuZero_Classic_MADN/game_agent_stochastic.py:52-257:
 * reset n games, then per turn throw the die (counter RNG: uniform(seed, game, turn) through throw_die),
 * search games with a legal pin (run_stochastic_muzero_mcts with cfg; cfg->turn is set per turn), step or
 * no_step, and record obs / act / rew class / root value / visit policy [n][T][4] / mask / player / team /
 * discount class / dice / dice_dist until every game is done or max_steps turns ran. */
int muz_classic_selfplay(const muz_rules* rules /*host*/, const muz_classic_net_w* w /*host*/,
                         const muz_stoch_cfg* cfg /*host*/, muz_classic_soa state, muz_traj traj,
                         muz_traj_chance chance, int32_t n, void* workspace, int64_t workspace_bytes,
                         muz_sp_stats* stats /*host*/, void* stream);

/* muz_classic_selfplay streamed: num_games games through `lanes` refilled lanes (see
 * muz_detmadn_selfplay_stream); dice, Dirichlet, tie-break and final-action noise are keyed by game number
 * and the game's own step, so game k's record equals game k of a muz_classic_selfplay batch. */
int muz_classic_selfplay_stream(const muz_rules* rules /*host*/, const muz_classic_net_w* w /*host*/,
                                const muz_stoch_cfg* cfg /*host*/, muz_classic_soa state, muz_traj traj,
                                muz_traj_chance chance, int32_t num_games, int32_t lanes, void* workspace,
                                int64_t workspace_bytes, muz_sp_stats* stats /*host*/, void* stream);

/* ---- device replay ring (MuZero_det_MADN/vec_replay_buffer.py) ------------------------------
 * The reference's VectorizedReplayBuffer keeps [capacity][T] host NumPy arrays (obs fp32, 84 GB at
 * capacity 20000, T 550, C 34).  Here the ring lives in HBM, obs int8 (values 0..4, exact):
 * 21 GB at the same size.  save copies finished games device-to-device from the self-play
 * trajectory buffers; sample gathers a training batch and computes the value targets on device. */
typedef struct muz_ring {
  int8_t* obs;        /* [cap][T][C][56] */
  int32_t* act;       /* [cap][T] */
  int32_t* rew;       /* [cap][T] reward class */
  float* val;         /* [cap][T] root value */
  float* pol;         /* [cap][T][A] child visits (action weights) */
  float* mask;        /* [cap][T] */
  int32_t* player;    /* [cap][T] */
  int32_t* team;      /* [cap][T] */
  int32_t* discount;  /* [cap][T] discount class */
  int32_t* ep_len;    /* [cap] */
  int32_t capacity;
  int32_t max_steps;  /* T (= the trajectory buffers' max_steps) */
  int32_t obs_channels;
  int32_t num_actions;
  /* VectorizedReplayBufferStochastic (MuZero_Classic_MADN/vec_replay_buffer_stochastic.py): */
  int32_t won_if_positive;  /* 1: "game won" is final reward class > 0 (stochastic buffer, line 194), 0: == 2 */
  int32_t* dice;            /* [cap][T] or null (det) */
  float* dice_dist;         /* [cap][T][6] or null */
} muz_ring;

/* A training batch, sample_batch's return dict (vec_replay_buffer.py:256-264), K = unroll_steps + 1. */
typedef struct muz_sample {
  float* observations;        /* [B][C][56] */
  int32_t* actions;           /* [B][K-1] */
  int32_t* rewards;           /* [B][K-1] */
  float* policies;            /* [B][K][A] */
  float* values;              /* [B][K] */
  float* masks;               /* [B][K] */
  float* target_values;       /* [B][K] */
  int32_t* discount_targets;  /* [B][K-1] */
  int32_t* dice_outcomes;     /* [B][K-1] die - 1, 0 when padded (stochastic buffer); null = not produced */
  float* dice_probs;          /* [B][K-1][6] dice distribution, uniform when padded; null = not produced */
} muz_sample;

/* save_games_from_buffers (vec_replay_buffer.py:36-61): game i with traj.idx[i] > 0 goes to ring slot
 * (position + r_i) % capacity, r_i = number of such games before i (later games win a slot that wraps
 * twice, as in the sequential loop).  slot_out[i] (device int32[n], required) = its slot or -1;
 * count_out (device int32[1]) = number of games with idx > 0 (the host advances position / size). */
int muz_ring_save(muz_ring ring, muz_traj traj, const muz_traj_chance* chance /*host, null for det*/, int32_t n,
                  int32_t position, int32_t* slot_out, int32_t* count_out, void* stream);

/* sample_batch (vec_replay_buffer.py:63-264) for given episode / start indices (the reference draws them
 * with np.random; the host mirror draws them the same way).  gamma_pow (device double[max_steps + 1]) =
 * 0.997 ** n as NumPy computes it; targets are evaluated in double and rounded to float like the
 * reference (NumPy float64, then jnp.array). */
int muz_ring_sample(muz_ring ring, const int32_t* ep_idx, const int32_t* t_start, int32_t batch, int32_t unroll_steps,
                    int32_t td_steps, int32_t bootstrap_value_target, const double* gamma_pow, muz_sample out,
                    void* stream);

/* ---- TicTacToe (config (a): CPU plumbing; TicTacToe/TicTacToeV2.py, TicTacToe/mcts.py, eval.py) -------
 * Host code (no GPU).  The reference's jax keys are replaced by counter streams (csrc/tictactoe.cpp;
 * restated by oracle/tictactoe.py); tree arithmetic is double. */
typedef struct muz_ttt_state {
  int8_t board[9];        /* row-major 3x3: 0 empty, 1 / -1 players */
  int8_t current_player;  /* 1 or -1 */
  int8_t reward;
  uint8_t done;
  int8_t memory[6];       /* [player (1 -> row 0, -1 -> row 1)][last 3 moves, oldest first], -1 = none */
} muz_ttt_state;

typedef struct muz_ttt_policy_out {
  int32_t action;             /* categorical(log(action_weights) / temperature) */
  int32_t visits[9];          /* root children visit counts */
  double action_weights[9];   /* visit_probs */
  double value;               /* root node value */
} muz_ttt_policy_out;

/* env_reset (TicTacToeV2.py:37-44). */
int muz_ttt_reset(muz_ttt_state* state);
/* env_step (46-76) with its quirks (see oracle/tictactoe.py); action 0..8. */
int muz_ttt_step(muz_ttt_state* state, int32_t action, int8_t* reward, uint8_t* done);
/* policy_function (97-104) -> logits[9]. */
int muz_ttt_policy_logits(const muz_ttt_state* state, double* logits);
/* value_function / rollout (106-123) with the counter stream (seed, eval_id). */
int muz_ttt_rollout(const muz_ttt_state* state, uint64_t seed, uint32_t eval_id, double* value);
/* run_mcts (mcts.py:9-23): mctx.muzero_policy, rollout values, qtransform_by_min_max(-1, 1). */
int muz_ttt_muzero_policy(const muz_ttt_state* root, int32_t num_simulations, int32_t max_depth, double temperature,
                          uint64_t seed, int32_t turn, muz_ttt_policy_out* out);
/* eval.py:97-125 / 252-276: MCTS player (argmax of action_weights over empty cells) vs uniform random
 * player; result = winner * mcts_player, 0 at the ply limit. */
int muz_ttt_match(int32_t mcts_player, int32_t num_simulations, uint64_t seed, int32_t game, int32_t limit,
                  int32_t* result);

/* ---- trajectory transfer (actors -> learner; north star: RCCL gather into one learner rank) ------
 * The reference moves finished games device -> host with np.array and copies them slot by slot
 * (vec_replay_buffer.py:36-61).  Here an actor PACKS its games' [0, idx) steps into contiguous rows
 * (no padding to T), the packed rows travel rank -> learner over RCCL point-to-point, and the learner
 * writes them into its ring without unpacking.  Packed layout = a muz_traj whose arrays are indexed by
 * row (row_offset[g] + t) instead of g*T + t; idx = the game lengths. */

/* row_offset[g] = exclusive prefix sum of max(len, 0); total_rows[0] = sum (device int64). */
int muz_traj_offsets(const int32_t* len, int32_t n, int64_t* row_offset, int64_t* total_rows, void* stream);

/* Pack traj ([n][T] layout) into `packed` rows at row_offset (from muz_traj_offsets); packed.idx (may be
 * null) receives the lengths.  chance / packed_chance: both null or both set (classic dice fields). */
int muz_traj_pack(muz_traj traj, const muz_traj_chance* chance, const int64_t* row_offset, int32_t n,
                  int32_t obs_channels, int32_t num_actions, muz_traj packed, const muz_traj_chance* packed_chance,
                  void* stream);

/* muz_ring_save for packed rows: same slot rule, max_len = the longest game (bounds the grid). */
int muz_ring_save_packed(muz_ring ring, muz_traj packed, const muz_traj_chance* chance, const int64_t* row_offset,
                         int32_t n, int32_t max_len, int32_t position, int32_t* slot_out, int32_t* count_out,
                         void* stream);

/* ---- learner support (config (e); not a reference FFI entry point) --------------------------------
 * The Dense -> LayerNorm -> ReLU blocks of the unrolled MuZero loss (train_with_reward.py:24-141,
 * train_stochastic.py:34-181; Flax LayerNorm eps 1e-6, fast variance) as one fused epilogue after a
 * library GEMM, and its backward (csrc/learner_ln.hip).  y, res, out, z, dout, dz, dres: device float
 * [M][N] row-major; bias, gamma, beta, dgamma, dbeta, dbias: [N]; mean, rstd: [M]; N in {32, 64, 128, 256}.
 * mode 0: out = LN(y + bias); 1: relu(LN(y + bias)); 2: relu(res + LN(y + bias)) (res required exactly for
 * mode 2, and dres for its backward).  z, mean, rstd, out are the forward's saved values. */
int muz_ln_fwd(const float* y, const float* bias, const float* gamma, const float* beta, const float* res, int32_t M,
               int32_t N, int32_t mode, float* out, float* z, float* mean, float* rstd, void* stream);
/* muz_ln_fwd of y = the sum of `parts` [M][N] planes (consecutive in y), added in plane order: the epilogue of a
 * long-K GEMM run as a batched GEMM over K chunks (the learner's representation Dense_0, K = 3584). */
int muz_ln_fwd_parts(const float* y, int32_t parts, const float* bias, const float* gamma, const float* beta,
                     const float* res, int32_t M, int32_t N, int32_t mode, float* out, float* z, float* mean, float* rstd,
                     void* stream);
/* device float scratch muz_ln_bwd needs for M rows of width N (-1 for an unsupported N). */
int64_t muz_ln_bwd_scratch_floats(int32_t M, int32_t N);
/* The backward's two halves: muz_ln_bwd_rows writes dz (and dres) and the per-block column partials into
 * scratch (muz_ln_bwd_scratch_floats(M, N) floats = nblk x 3 x N); muz_ln_colsum reduces nblk partial blocks
 * (several calls' scratch laid end to end, e.g. one layer applied at every unroll step) in a fixed order. */
int muz_ln_bwd_rows(const float* dout, const float* out, const float* z, const float* mean, const float* rstd,
                    const float* gamma, int32_t M, int32_t N, int32_t mode, float* dz, float* dres, float* scratch,
                    void* stream);
/* muz_ln_bwd_rows with dout's rows ldd >= N floats apart (a column slice of a wider gradient, e.g. of a
 * concatenation's input: no copy to a contiguous block). */
int muz_ln_bwd_rows_ld(const float* dout, int32_t ldd, const float* out, const float* z, const float* mean,
                       const float* rstd, const float* gamma, int32_t M, int32_t N, int32_t mode, float* dz, float* dres,
                       float* scratch, void* stream);
int muz_ln_colsum(const float* scratch, int64_t nblk, int32_t N, float* dgamma, float* dbeta, float* dbias,
                  void* stream);
/* dz = d(y) (= the GEMM output's gradient); dgamma / dbeta / dbias: column sums (deterministic order). */
int muz_ln_bwd(const float* dout, const float* out, const float* z, const float* mean, const float* rstd,
               const float* gamma, int32_t M, int32_t N, int32_t mode, float* dz, float* dres, float* scratch,
               float* dgamma, float* dbeta, float* dbias, void* stream);
/* DynamicsNetwork4's action-only FiLM sub-graph over M learner rows (muzero_deterministic_madn.py:404-418; replaces
 * the reference's one_hot -> Dense_0 -> relu -> Dense_1 | Dense_2 of each unroll step, train_with_reward.py:98-105):
 * e = relu(b0 + W0[action]) ([M][64]; action outside [0, A) -> the all-zero one-hot row), scale = e W1 + b1,
 * shift = e W2 + b2 ([M][256]), optional scale1 = 1 + scale and optional float one-hot rows [M][A].  W0 [A][64],
 * W1 / W2 [64][256], row-major.  Backward: de = (dscale W1^T + dshift W2^T) * [e > 0] ([M][64]); the weight and
 * bias gradients are the caller's (e^T dscale, e^T dshift, one_hot^T de, column sums). */
int muz_film_fwd(const int32_t* action, int32_t M, int32_t A, const float* W0, const float* b0, const float* W1,
                 const float* b1, const float* W2, const float* b2, float* onehot, float* e, float* scale,
                 float* shift, float* scale1, void* stream);
/* The same over the M = B x K step-major rows of a [B][lda] action array (row k B + b reads action[b lda + k]): the
 * learner's batch["actions"][:, :K] without a transposed copy.  muz_film_fwd is B = M, K = 1, lda = 1. */
int muz_film_fwd_strided(const int32_t* action, int32_t B, int32_t K, int32_t lda, int32_t A, const float* W0,
                         const float* b0, const float* W1, const float* b1, const float* W2, const float* b2,
                         float* onehot, float* e, float* scale, float* shift, float* scale1, void* stream);
int muz_film_bwd(const float* dscale, const float* dshift, const float* e, const float* W1, const float* W2,
                 int32_t M, float* de, void* stream);
/* The FiLM input of a dynamics trunk (muzero_deterministic_madn.py:421-427; learner._TrunkChain): out = LayerNorm(x)
 * (Flax, eps 1e-6, no bias), film = shift + out * scale1 (scale1 = 1 + FiLM scale), saving z / mean / rstd like
 * muz_ln_fwd; and its backward half from d(film): dscale = d(film) * out and the LayerNorm row backward of
 * d(film) * scale1 (dz, column partials into scratch as muz_ln_bwd_rows, LN_PLAIN).  N = 256. */
int muz_ln_film_fwd(const float* x, const float* gamma, const float* beta, const float* scale1, const float* shift,
                    int32_t M, int32_t N, float* out, float* z, float* mean, float* rstd, float* film, void* stream);
int muz_ln_film_bwd_rows(const float* dfilm, const float* out, const float* z, const float* mean, const float* rstd,
                         const float* gamma, const float* scale1, int32_t M, int32_t N, float* dz, float* dscale,
                         float* scratch, void* stream);
/* The boundary of two dynamics-trunk applications (learner._TrunkChain) as one launch each way, N = 256:
 * muz_minmax_film_fwd = muz_minmax_fwd of application i (out, q, lohi, idx) followed by muz_ln_film_fwd of
 * application i + 1 on its output (ln_out, ln_z, ln_mean, ln_rstd, film); muz_film_minmax_bwd =
 * muz_ln_film_bwd_rows of application i + 1 (dscale, column partials into scratch) followed by muz_minmax_bwd of
 * application i with a = that LayerNorm input gradient (g, b, h, scale, scaled, q, lohi -> dq).  Bit-identical
 * to the separate calls. */
int muz_minmax_film_fwd(const float* x, const float* y, const float* bias, int32_t M, int32_t N, float* out, float* q,
                        float* lohi, int32_t* idx, const float* gamma, const float* beta, const float* scale1,
                        const float* shift, float* ln_out, float* ln_z, float* ln_mean, float* ln_rstd, float* film,
                        void* stream);
int muz_film_minmax_bwd(const float* dfilm, const float* out, const float* z, const float* mean, const float* rstd,
                        const float* gamma, const float* scale1, int32_t M, int32_t N, float* dscale, float* scratch,
                        const float* g, const float* b, const float* h, float scale, int32_t scaled, const float* q,
                        const float* lohi, float* dq, void* stream);
/* Min-max latent scaling closing a dynamics trunk (x = the trunk input; x null: q = y + bias, the
 * representation's last Dense, muzero_deterministic_madn.py:139-140), N = 256: q = x + (y + bias), out = (q - min) /
 * (max - min + 1e-8) per row; saves q [M][N], lohi [M][2] (min, max) and idx [M][2] (their columns, lowest on
 * ties).  Backward: dq from d = (g + (a + b)) x (scale if scaled) + h (a, b both null or both given; h
 * optional: a gradient that bypasses the latent scaling, e.g. the det reward / discount heads reading the
 * unscaled next latent, train_with_reward.py:49-105); the extremum gradient is split evenly over tied columns
 * (JAX's reduce_min / reduce_max rule). */
int muz_minmax_fwd(const float* x, const float* y, const float* bias, int32_t M, int32_t N, float* out, float* q,
                   float* lohi, int32_t* idx, void* stream);
int muz_minmax_bwd(const float* g, const float* a, const float* b, const float* h, float scale, int32_t scaled,
                   const float* q, const float* lohi, int32_t M, int32_t N, float* dq, void* stream);
/* Grouped learner gradients (csrc/learner_grad.hip): every weight gradient dW = X^T dZ of one backward, and every
 * bias / LayerNorm column sum, in two launches instead of one library call each.  Deterministic (fixed
 * reduction order).  muz_wgrad_grouped: out[K][N] = x[M][K]^T dz[M][N] (row strides ldx, lddz; overwrites out).
 * muz_colsum_grouped: kind 0 reduces muz_ln_bwd_rows partials (src = scratch, rows = blocks) into out0 = dgamma,
 * out1 = dbeta, out2 = dbias (any may be null); kind 1 sums the rows of src [rows][ld] into out0 [N]. */
typedef struct {
  const float* x;
  const float* dz;
  float* out;
  int32_t M, K, N, ldx, lddz;
} muz_wgrad_problem;
typedef struct {
  const float* src;
  float* out0;
  float* out1;
  float* out2;
  int32_t kind, rows, N, ld;
} muz_colsum_problem;
/* scratch: muz_wgrad_scratch_floats(problems, count) device floats (problems over muz_wgrad_segment_rows() rows
 * are split into segments of that many rows whose partials are added in segment order). */
int64_t muz_wgrad_scratch_floats(const muz_wgrad_problem* problems, int32_t count);
int32_t muz_wgrad_segment_rows(void);
int muz_wgrad_grouped(const muz_wgrad_problem* problems, int32_t count, float* scratch, int64_t scratch_floats,
                      void* stream);
int muz_colsum_grouped(const muz_colsum_problem* problems, int32_t count, void* stream);
/* The learner's losses and their gradients w.r.t. the network outputs in ONE launch (csrc/learner_loss.hip):
 * loss_fn (train_with_reward.py:24-141) and loss_fn_stochastic (train_stochastic.py:34-180) for all K + 1
 * unroll steps at once.  Rows are step-major (row k B + b = unroll step k of sample b).
 *   value:  l_v[k] = mean_b m[b][k] (tv[b][k] - value[row])^2                        (rows of K + 1 steps)
 *   policy: l_p[k] = mean_b m[b][k] * -(pol[b][k] . log_softmax(logits[row]))       (rows of K + 1 steps)
 *   term j (rows of the first K steps): ce = cross-entropy of logits_j against a class label labels[b][k]
 *     or a distribution probs[b][k][:]; "rare" rows: label == 1 (rare_not_one = 0), label != 1 (= 1), or a
 *     distribution not uniform (sum (p - 1/6)^2 > 1e-6); l_j[k] = w_rare S(m r ce) / n_r + w_common
 *     S(m (1 - r) ce) / n_c with n_r = max(S(m r), 1) and n_c = max(S(m) - S(m r), 1) (norm 0, det's
 *     _balanced_ce_steps) or max(S(m) - n_r, 1) (norm 1, train_stochastic.py:25-32).
 * total = scale_value S_k l_v + scale_policy S_k l_p + S_j scale_j S_k l_j.  parts: [total, S l_v, S l_p,
 * S l_0, S l_1, S l_2] (unused terms 0).  Every d* output receives d total / d input (overwritten).
 * Deterministic; one workgroup per unroll step. */
typedef struct {
  const float* logits;
  float* dlogits;
  const int32_t* labels;   /* [B][ld] (column k) -- or null with probs */
  const float* probs;      /* [B][ld][ncls] */
  int32_t ncls, ld, rare_not_one;
  float w_rare, w_common, scale;
} muz_loss_term;
typedef struct {
  int32_t K, B, A, T;      /* unroll steps (<= 64), batch, policy width (<= 1024: <= 32 a thread per row, wider a
                              wave per row -- the DOG learner's 806), time stride of masks / target_values / policies */
  int32_t nterms, norm;    /* CE terms (<= 3), n_common form */
  const float* masks;      /* [B][T] */
  const float* target_values;
  const float* policies;   /* [B][T][A] */
  const float* value;      /* [(K + 1) B] */
  const float* logits;     /* [(K + 1) B][A] */
  float* dvalue;
  float* dlogits;
  float scale_value, scale_policy;
  muz_loss_term term[3];
  float* parts;            /* [6] */
  float* total;            /* [1] (= parts[0]; a separate scalar for the autograd node's output) */
  float* partials;         /* scratch [(K + 1) * 5] */
  int32_t* ticket;         /* a device counter, 0 before the launch (the kernel leaves it 0 again) */
} muz_loss_args;
int muz_loss_heads(const muz_loss_args* args, void* stream);
/* The learner's output heads in one launch each way (csrc/learner_heads.hip): PredictionNetwork4's policy logits
 * Dense_2 and value head Dense_4 -> relu -> Dense_5 -> tanh over R rows of the policy / value hidden layers
 * (muzero_deterministic_madn.py:572-583), and DynamicsNetwork4's reward / discount heads Dense_6 | Dense_7 -> relu ->
 * reward_head | discount_head over Rk rows of [next latent, one_hot(action)] (lines 437-455).  Forward fills logits
 * [R][A], value [R], the saved relu outputs h4 [R][64], h6 / h7 [Rk][64], ri = [next latent, one_hot] [Rk][256 + A],
 * rl / dl [Rk][3].  Backward (g_* nullable = zero) fills the input gradients d_pol_h / d_v_h [R][128], d_head_in
 * [Rk][256] and the pre-activation gradients dz4 [R][64], dv5 [R], dz6 / dz7 [Rk][64] the weight gradients are
 * formed from.  Weights row-major [in][out]; A <= 32. */
typedef struct muz_heads_args {
  int32_t R, Rk, A;
  const float* pol_h; const float* v_h; const float* head_in; const float* onehot;
  const float* W2; const float* b2; const float* W4; const float* b4; const float* W5; const float* b5;
  const float* W6; const float* b6; const float* Wr; const float* br; const float* W7; const float* b7;
  const float* Wd; const float* bd;
  float* logits; float* value; float* h4; float* rl; float* dl; float* h6; float* h7; float* ri;
  const float* g_logits; const float* g_value; const float* g_rl; const float* g_dl;
  float* d_pol_h; float* d_v_h; float* d_head_in; float* dz4; float* dv5; float* dz6; float* dz7;
} muz_heads_args;
int muz_heads_fwd(const muz_heads_args* args, void* stream);
int muz_heads_bwd(const muz_heads_args* args, void* stream);
/* One launch per learner layer (csrc/learner_fused.hip): muz_dense_ln_fwd = muz_ln_fwd(x @ W, ...) with the GEMM
 * fused in (x [M][K], W [K][N] row-major, K <= 512, N in {32, 64, 128, 256}; same outputs out / z / mean / rstd);
 * muz_dense_ln_bwd = muz_ln_bwd_rows followed by dx = dz W^T (+ acc) (dx [M][K]; dx null: no input gradient),
 * column partials into scratch [ceil(M / 16)][3][N] (muz_dense_ln_bwd_scratch_floats; any muz_ln_colsum-style
 * reduction over its rows gives dgamma / dbeta / dbias). */
int muz_dense_ln_fwd(const float* x, int32_t M, int32_t K, const float* W, const float* WT, int32_t ldt,
                     const float* bias, const float* gamma, const float* beta, const float* res, int32_t N,
                     int32_t mode, float* out, float* z, float* mean, float* rstd, void* stream);
/* WT (optional, used instead of W when given): W^T as [N][ldt], ldt >= K rounded up to 16, a multiple of 4,
 * columns K .. ldt - 1 zero -- kept per layer by the learner and refreshed by muz_transpose_grouped, which
 * writes dst[n * ldt + k] = src[k * N + n] for k < K (one launch for all layers). */
typedef struct {
  const float* src;
  float* dst;
  int32_t K, N, ldt;
} muz_transpose_problem;
int muz_transpose_grouped(const muz_transpose_problem* problems, int32_t count, void* stream);
int64_t muz_dense_ln_bwd_scratch_floats(int32_t M, int32_t N);
int muz_dense_ln_bwd(const float* dout, const float* out, const float* z, const float* mean, const float* rstd,
                     const float* gamma, int32_t M, int32_t N, int32_t mode, const float* W, int32_t K,
                     const float* acc, float* dz, float* dres, float* dx, float* scratch, void* stream);
/* muz_dense_ln_bwd with dout's rows ldd floats apart (ldd >= N, a multiple of 4; dout 16-byte aligned). */
int muz_dense_ln_bwd_ld(const float* dout, int32_t ldd, const float* out, const float* z, const float* mean,
                        const float* rstd, const float* gamma, int32_t M, int32_t N, int32_t mode, const float* W,
                        int32_t K, const float* acc, float* dz, float* dres, float* dx, float* scratch, void* stream);
/* The unrolled dynamics chain of a learner step as ONE launch each way (csrc/learner_chain.hip; replaces
 * learner._TrunkChain's per-layer launch train of library GEMMs and row kernels; reference:
 * train_with_reward.py:98-107 (one trunk, K applications), train_stochastic.py:95-121 (act / chance trunks
 * alternating)).  Application i maps x_i -> x_{i+1} = minmax(x_i + proj(trunk(LN_0(x_i) * scale1_i + shift_i)))
 * with group app[i]'s weights, trunk = Dense + LN + ReLU twice, then two ResBlocks (Dense + LN + ReLU,
 * Dense + LN, + input, ReLU) -- DynamicsNetwork4 / StochasticDynamicsNetwork4's FiLM trunk
 * (muzero_deterministic_madn.py:391-457).  All widths 256.  One workgroup carries 16 rows through all T
 * applications (weights streamed from L2, the tile's activations in LDS).
 * Layer order of the 7-entry arrays: Dense "3", "4", ResBlock_0 Dense_0 / Dense_1, ResBlock_1 Dense_0 / Dense_1,
 * projection "5"; part[] has LayerNorm_0 first, then the 6 Dense + LayerNorm layers.
 * Forward writes out / q / lohi / idx (as muz_minmax_fwd, per application), ln0_out (LayerNorm_0 output), z / stats
 * (pre-LayerNorm y + bias of the 6 layers; mean, rstd of LayerNorm_0 then the 6 layers) and every weight layer's
 * input into the group's stack X[l] at row block slot[i].  Backward (reads everything the forward wrote) writes
 * each weight layer's output gradient into DZ[l] (same blocks), column partials [ceil(M / 16)][3][256] per
 * application into part[] (muz_ln_colsum layout), dscale / dshift [T][M][256] and dlatent0 [M][256]; the incoming
 * gradient of x_{i+1} is g[i] (+ the carried gradient), x grad_scale where scaled[i], + h[i] (h optional). */
#define MUZ_CHAIN_MAX_T 32
typedef struct {
  const float* ln0_gamma;
  const float* ln0_beta;
  const float* wf[7];      /* the weights [256][256] packed for the forward and the backward GEMM */
  const float* wb[7];      /* (muz_trunk_chain_pack) */
  const float* bias[7];
  const float* gamma[6];
  const float* beta[6];
  float* X[7];             /* [applications of the group][M][256] */
  float* DZ[7];
  float* part[7];          /* [applications of the group][ceil(M / 16)][3][256] */
} muz_chain_group;
typedef struct {
  int32_t T, M, ngroups;
  int32_t app[MUZ_CHAIN_MAX_T], slot[MUZ_CHAIN_MAX_T], scaled[MUZ_CHAIN_MAX_T];
  muz_chain_group group[2];
  const float* latent0;    /* [M][256] */
  const float* scale1;     /* [T][M][256] */
  const float* shift;      /* [T][M][256] */
  float* out;              /* [T][M][256] */
  float* q;                /* [T][M][256] */
  float* lohi;             /* [T][M][2] */
  int32_t* idx;            /* [T][M][2] */
  float* ln0_out;          /* [T][M][256] */
  float* z;                /* [T][6][M][256] */
  float* stats;            /* [T][7][2][M] */
  const float* g;          /* backward: [T][M][256] */
  const float* h;          /* optional [T][M][256] */
  float grad_scale;
  float* dscale;
  float* dshift;
  float* dlatent0;
  /* optional (null: unused) -- the learner's stacked-latent form, no copies around the chain: */
  float* out_twin;         /* forward: a second copy of out (the heads' unscaled-gradient input) */
  float* stack0;           /* forward: latent0 copied here (block 0 of a [T + 1][M][256] stack whose rest is out) */
  const float* g0;         /* backward: added to dlatent0 (the stack's block-0 gradient) */
} muz_chain_args;
/* wf / wb of count row-major [256][256] weights W[i] (y = x W): fwd + i * 65536 and bwd + i * 65536 hold them as
 * the MFMA A-operand stream of y = x W and of dx = dz W^T (one launch; call whenever the weights change). */
int muz_trunk_chain_pack(const float* const* W, int32_t count, float* fwd, float* bwd, void* stream);
int muz_trunk_chain_fwd(const muz_chain_args* args, void* stream);
int muz_trunk_chain_bwd(const muz_chain_args* args, void* stream);
/* A stack of nb ResBlocks (relu(x + LN(Dense_1(relu(LN(Dense_0(x))))))), muzero_deterministic_madn.py:12-24: the
 * representation's six and the prediction's two, as trained by train_with_reward.py) as ONE launch each way
 * (csrc/learner_chain.hip, the chain kernels' 16-row tiles and GEMM loop).  Weight layer l = 2 b + k (block b,
 * its Dense_k), all widths 256, weights packed by muz_trunk_chain_pack.  Forward writes X[l] (the input of weight
 * layer l; X[0] = x), out, z (pre-LayerNorm y + bias) and stats (mean, rstd).  Backward (reads what the forward
 * wrote) writes DZ[l] (the output gradient of weight layer l), the column partials part[l] [ceil(M / 16)][3][256]
 * (muz_ln_colsum layout) and dx. */
#define MUZ_RBSTACK_MAX 6
typedef struct {
  int32_t nb, M;
  const float* wf[2 * MUZ_RBSTACK_MAX];
  const float* wb[2 * MUZ_RBSTACK_MAX];
  const float* bias[2 * MUZ_RBSTACK_MAX];
  const float* gamma[2 * MUZ_RBSTACK_MAX];
  const float* beta[2 * MUZ_RBSTACK_MAX];
  const float* x;          /* [M][256] */
  float* X;                /* [2 nb][M][256] */
  float* out;              /* [M][256] */
  float* z;                /* [2 nb][M][256] */
  float* stats;            /* [2 nb][2][M] */
  const float* g;          /* backward: d out [M][256] */
  float* DZ;               /* [2 nb][M][256] */
  float* part;             /* [2 nb][ceil(M / 16)][3][256] */
  float* dx;               /* [M][256] */
} muz_rbstack_args;
int muz_rbstack_fwd(const muz_rbstack_args* args, void* stream);
int muz_rbstack_bwd(const muz_rbstack_args* args, void* stream);
/* 'SAME' Conv1D as a GEMM: the im2col matrix cols [B][W][K x Cin] of x [B][W][Cin] (zero outside each row;
 * tap d reads column w + d - (K - 1) / 2) and its backward dx = sum over taps (fixed order). */
int muz_im2col_fwd(const float* x, int32_t B, int32_t W, int32_t Cin, int32_t K, float* cols, void* stream);
/* muz_im2col_fwd of a strided view: x element (b, w, c) at x[b sb + w sw + c sc] (element strides). */
int muz_im2col_fwd_strided(const float* x, int32_t B, int32_t W, int32_t Cin, int32_t K, int64_t sb, int64_t sw,
                           int64_t sc, float* cols, void* stream);
int muz_im2col_bwd(const float* dcols, int32_t B, int32_t W, int32_t Cin, int32_t K, float* dx, void* stream);

/* One optimizer step over ntensors parameter tensors (csrc/learner_opt.hip): optax.chain(
 * clip_by_global_norm(max_norm), adamw(lr, b1, b2, eps, weight_decay)) with the piecewise-constant lr
 * lr0 x prod{factor_j : step - 1 >= iteration_j x steps_per_iteration} (train_with_reward.py:361-372,
 * train_stochastic.py:415-426).  params / grads / mu / nu: host arrays of device float pointers (a null
 * grad is a zero gradient), numel: host array; count: device double step counter (incremented); gnorm:
 * device float, receives the pre-clip global norm; scratch: muz_adamw_scratch_bytes(ntensors, numel) device
 * bytes; boundaries: host [nb][2] (iteration, factor), nb <= 4.  Deterministic (fixed-order reduction). */
int64_t muz_adamw_scratch_bytes(int32_t ntensors, const int64_t* numel);
int muz_adamw_step(float* const* params, const float* const* grads, float* const* mu, float* const* nu,
                   const int64_t* numel, int32_t ntensors, double* count, void* scratch, float* gnorm,
                   float max_norm, double b1, double b2, float eps, float weight_decay, double lr0,
                   double steps_per_iteration, const double* boundaries, int32_t nb, void* stream);
/* The same step in one launch per pass over a caller-owned device tensor table: muz_adamw_table_bytes(ntensors)
 * device bytes, filled by muz_adamw_table_write (eager only -- MUZ_E_INVALID under stream capture; returns once the
 * table is in device memory).  muz_adamw_step_table reads the table at run time, so a graph that captured it updates
 * whatever the table holds at replay: keep it unchanged while such a graph may replay. */
int64_t muz_adamw_table_bytes(int32_t ntensors);
int muz_adamw_table_write(void* table, float* const* params, const float* const* grads, float* const* mu,
                          float* const* nu, const int64_t* numel, int32_t ntensors, void* stream);
int muz_adamw_step_table(const void* table, const int64_t* numel, int32_t ntensors, double* count, void* scratch,
                         float* gnorm, float max_norm, double b1, double b2, float eps, float weight_decay, double lr0,
                         double steps_per_iteration, const double* boundaries, int32_t nb, void* stream);

/* ---- DOG MuZero slice (MuZero_DOG/muzero_dog.py, DOG/dog.py:1264-1272) -----------------------------------
 * The reference defines only the DOG RepresentationNetwork (muzero_dog.py:25-83: RepresentationNetwork2's trunk with
 * a LayerNorm after its last Dense instead of min-max); encode_board, the dynamics / prediction networks, the
 * inference functions and the self-play loop are `pass` (dog.py:1264-1272, muzero_dog.py:85-99, game_agent.py:52-57).
 * Following SURVEY 8(d) ("MCTS with the det-MADN-shaped nets at A=806") this slice defines them: a 34-channel
 * observation (oracle/dog_muzero.py encode_board), DynamicsNetwork4 / PredictionNetwork4 of the det file at A = 806,
 * and gumbel_muzero_policy at A = 806 as muzero_dog.py:101-137 calls it.  Parity unpinned beyond the env. */
#define MUZ_DOG_OBS_CHANNELS 34
typedef struct muz_dog_net_w {
  int32_t obs_channels;         /* 34 */
  int32_t num_actions;          /* 806 */
  muz_repr_w repr;              /* RepresentationNetwork (muzero_dog.py:25-83) up to Dense_4 */
  muz_ln repr_ln7;              /* its LayerNorm head (lines 80-81) */
  muz_dyn_w dyn;                /* DynamicsNetwork4 at A = 806 (film: [807][512]) */
  muz_pred_w pred;              /* PredictionNetwork4 at A = 806; pred.d2 == logits[0] */
  muz_dense logits[4];          /* Dense_2 (128 -> 806) as column chunks 0-255, 256-511, 512-767 (packed for 256
                                   columns) and 768-805 (packed for 38) */
} muz_dog_net_w;

/* dyn.film of a DOG weight set (muz_net_prepare's table at A = 806). */
int muz_dog_net_prepare(const muz_dog_net_w* w /*host*/, void* stream);

/* encode_board for n 4-player games (oracle/dog_muzero.py encode_board): obs [n][34][56] fp32. */
int muz_dog_encode(const muz_rules* rules /*host*/, muz_dog_soa state, float* obs, int32_t n, void* stream);

/* root_inference_fn: obs [n][34][56] -> prior_logits [n][806], value [n], embedding [n][256]; scratch as
 * muz_nets_root_scratch_bytes(n). */
int muz_dog_nets_root(const muz_dog_net_w* w /*host*/, const float* obs, int32_t n, void* scratch,
                      int64_t scratch_bytes, float* prior_logits, float* value, float* embedding, void* stream);

/* recurrent_inference_fn: (action [n], embedding [n][256]) -> reward, discount, prior_logits [n][806], value,
 * next_embedding. */
int muz_dog_nets_recurrent(const muz_dog_net_w* w /*host*/, const int32_t* action, const float* embedding, int32_t n,
                           float* reward, float* discount, float* prior_logits, float* value, float* next_embedding,
                           void* stream);

/* Workspace bytes of n DOG searches (children arrays [n][S+1][832] x 6 + node embeddings + the root noise + per-node
 * visited-child records [n][S+1][32] x 32 B and top-prior lists [n][S+1][8] x 8 B). */
int64_t muz_dog_search_workspace_bytes(int32_t n, const muz_search_cfg* cfg /*host*/);

/* run_muzero_mcts (muzero_dog.py:101-137): gumbel_muzero_policy at A = 806.  legal: muz_dog_legal's mask
 * [n][26] words (invalid = ~legal); gumbel [n][806] already scaled, or NULL for the device noise of
 * (cfg->seed, game, cfg->turn).  Outputs action [n] (-1 for a game without a legal action: the self-play loop's
 * no_step), action_weights [n][806], root_value [n].  Results do not depend on the two environment switches it
 * reads (tests use them): MUZ_DOG_EXACT_SELECT=1 runs every interior selection over all 806 exponentials instead of
 * the certified argmax; MUZ_DOG_TILE_ROWS=8|16 forces one / two games per wave (default: one up to n = 2048). */
/* Games per workgroup muz_dog_gumbel_search launches k_dog_search with for n games (reads the same environment
 * switches: MUZ_DOG_TILE_ROWS, MUZ_DOG_GPW): 6-8 in the one-game-per-wave form, 16 in the two-per-wave form. */
int32_t muz_dog_search_games_per_workgroup(int32_t n);
int muz_dog_gumbel_search(const muz_dog_net_w* w /*host*/, const muz_search_cfg* cfg /*host*/,
                          const float* root_logits, const float* root_value, const float* root_embedding,
                          const uint32_t* legal, const float* gumbel, int32_t n, void* workspace,
                          int64_t workspace_bytes, int32_t* action, float* action_weights, float* root_value_out,
                          void* stream);

/* The DOG MuZero self-play turn's bookkeeping (config (e) as MuZero_DOG/train.py:168-300 trains; its
 * play_batch_of_games_jitted, MuZero_DOG/game_agent.py:52-57, is `pass` -- the record is the det loop's,
 * MuZero_det_MADN/game_agent.py:64-141) fused with the step: for every lane g with lane_game[g] >= 0 writes the
 * turn's row idx[slot] of trajectory slot lane_game[g] (traj: [num_games][max_steps], obs int8 [34][56] from this
 * turn's muz_dog_encode `obs`, pol [806] = action_weights; zero obs / pol, act -1, value 0, mask 0, reward and
 * discount class 1 on a no-move turn, action[g] < 0), applies env_step / no_step (+ deal), and restarts a game that
 * ended (done, or its max_steps-th record) in place (deal counter continued), setting ended[g].  Lanes with
 * lane_game[g] < 0 are idle (untouched).  episodes[g] (nullable) counts finished games. */
int muz_dog_sp_record_step(const muz_rules* rules /*host*/, muz_dog_soa state, const float* obs, const int32_t* action,
                           const float* action_weights, const float* root_value, uint64_t seed, muz_traj traj,
                           int32_t* lane_game, int32_t* ended, uint32_t* episodes, int32_t n, void* stream);
/* After muz_dog_sp_record_step: lanes whose game ended take the next game numbers in lane order (deterministic):
 * counters (device int32[3]) = {next game number, num_games, out: lanes still holding a game}; a newly assigned
 * slot's traj_idx is zeroed; a lane past num_games goes idle (-1). */
int muz_dog_sp_assign(int32_t* lane_game, const int32_t* ended, int32_t* traj_idx, int32_t* counters, int32_t n,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MUZ_H_ */
