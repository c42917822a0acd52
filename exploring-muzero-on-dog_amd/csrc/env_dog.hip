// Batched DOG environment kernels + C ABI (include/muz.h).  One wavefront per game, 4 games per
// 256-thread workgroup; the game's state is staged in LDS (dog.hpp: DogG).
#include "dog.hpp"
#include "host_consts.hpp"

namespace muz {

constexpr int kDogGamesPerBlock = 4;   // wave-per-game kernels (reset, explicit-action step)
constexpr int kDogBlockThreads = 448;  // block-per-game kernels: 7 waves = 4 swap, 2 hot-7, 1 normal/-4 checks
// k_dog_play's workgroup: 4 waves, each running the checks of two of the 7 check waves above in turn.  At
// 1024 games per GPU (4 workgroups per CU) that is 4 waves per SIMD with 128 VGPRs each; with 7 waves per game
// the 8-wave budget left 64 VGPRs, and the kernel spilled 45 VGPRs (and 240 SGPRs through VGPR lanes) to
// scratch, which the serial part of every turn (lane 0's env_step) paid in memory latency.
#ifndef MUZ_DOG_PLAY_THREADS
#define MUZ_DOG_PLAY_THREADS 256
#endif
constexpr int kDogPlayThreads = MUZ_DOG_PLAY_THREADS;
constexpr int kDogPlayWPE = kDogPlayThreads == 448 ? 8 : 4;   // waves per SIMD the play kernel is budgeted for

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct WaveSync {   // one wavefront owns the game
  static constexpr int N = 64;
  __device__ __forceinline__ void operator()() const { wave_sync(); }
};
struct BlockSync {  // a whole workgroup owns the game
  static constexpr int N = kDogBlockThreads;
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};
struct PlaySync {   // k_dog_play's workgroup owns the game
  static constexpr int N = kDogPlayThreads;
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

// ---- SoA <-> LDS ---------------------------------------------------------------------------------
template <class Sync>
__device__ __forceinline__ void dog_load(const DetConsts& c, const muz_dog_soa& st, int g, DogG& s, int tid) {
  const int S = st.stride;
  for (int i = tid; i < kCells; i += Sync::N) s.board[i] = st.board[i * S + g];
  if (tid < 16) s.pins[tid] = tid < c.P * 4 ? st.pins[tid * S + g] : (int8_t)-1;
  for (int i = tid; i < 4 * kDogCards; i += Sync::N)
    s.hands[i / kDogCards][i % kDogCards] = i < c.P * kDogCards ? st.hands[i * S + g] : 0;
  if (tid < kDogCards) s.deck[tid] = st.deck[tid * S + g];
  if (tid < 4) s.swap_choices[tid] = st.swap_choices[tid * S + g];
  if (tid == 0) {
    s.cp = st.current_player[g];
    s.round_starter = st.round_starter[g];
    s.phase = st.phase[g];
    s.hand_size = st.hand_size[g];
    s.done = st.done[g] ? 1 : 0;
    s.reward = st.reward[g];
    s.deal = st.deal[g];
  }
  Sync()();
}

template <class Sync>
__device__ __forceinline__ void dog_store(const DetConsts& c, const muz_dog_soa& st, int g, const DogG& s, int tid) {
  Sync()();
  const int S = st.stride;
  for (int i = tid; i < kCells; i += Sync::N) st.board[i * S + g] = s.board[i];
  if (tid < c.P * 4) st.pins[tid * S + g] = s.pins[tid];
  for (int i = tid; i < c.P * kDogCards; i += Sync::N) st.hands[i * S + g] = s.hands[i / kDogCards][i % kDogCards];
  if (tid < kDogCards) st.deck[tid * S + g] = s.deck[tid];
  if (tid < 4) st.swap_choices[tid * S + g] = s.swap_choices[tid];
  if (tid == 0) {
    st.current_player[g] = (int8_t)s.cp;
    st.round_starter[g] = (int8_t)s.round_starter;
    st.phase[g] = (int8_t)s.phase;
    st.hand_size[g] = (int8_t)s.hand_size;
    st.done[g] = (uint8_t)s.done;
    st.reward[g] = (int8_t)s.reward;
    st.deal[g] = s.deal;
  }
}

// ---- distribute_cards (dog.py:201-298), all lanes ---------------------------------------------------
__device__ __forceinline__ float deal_key(unsigned long long seed, int gid, unsigned deal, int k) {
  return u24(mix64(game_key(seed ^ kDealStream, gid, (int)deal) ^ (unsigned long long)(k + 1) * 0xA24BAED4963EE407ull));
}

template <class Sync>
__device__ void dog_deal(const DetConsts& c, DogG& s, unsigned long long seed, int gid, int lane) {
  const int P = c.P;
  const int q = s.hand_size;
  const unsigned deal = s.deal;
  if (lane == 0) {
    int tot = 0;
    for (int k = 0; k < kDogCards; ++k) tot += s.deck[k];
    if (tot < q * P) {   // reset_deck (dog.py:188-191): card 0 gets 6 + 2 * (joker enabled)
      for (int k = 0; k < kDogCards; ++k) s.deck[k] = 8;
      s.deck[0] = 8;
    }
  }
  Sync()();
  // the pool in deck order (entry k: the card whose running count covers k; dummies past the deck) and its sort
  // keys, one entry per lane (lane 0 filled it serially before: ~120 dependent LDS writes per deal)
  for (int k = lane; k < kMaxPool; k += Sync::N) {
    int acc = 0, card = kDogCards;
    for (int d = 0; d < kDogCards; ++d) {
      const int n = s.deck[d];
      if (card == kDogCards && k < acc + n) card = d;
      acc += n;
    }
    s.pool[k] = (int8_t)card;
    s.key[k] = card == kDogCards ? 2.0f : deal_key(seed, gid, deal, k);
  }
  Sync()();
  // stable argsort: rank = #smaller keys + #equal keys at a lower index
  for (int k = lane; k < kMaxPool; k += Sync::N) {
    const float kk = s.key[k];
    int r = 0;
    for (int j = 0; j < kMaxPool; ++j) {
      const float kj = s.key[j];
      r += (kj < kk) || (kj == kk && j < k);
    }
    s.shuffled[r] = s.pool[k];
  }
  Sync()();
  // player p takes shuffled[p q .. p q + q): counted per (player, card) and per card in parallel (the same sums as
  // the serial hand-by-hand increments)
  const int qq = q < 6 ? q : 6;
  for (int t = lane; t < P * kDogCards; t += Sync::N) {
    const int p = t / kDogCards, card = t % kDogCards;
    int n = 0;
    for (int sl = 0; sl < qq; ++sl) n += s.shuffled[p * q + sl] == card;
    s.hands[p][card] = (int8_t)(s.hands[p][card] + n);
  }
  for (int card = lane; card < kDogCards; card += Sync::N) {
    int n = 0;
    for (int p = 0; p < P; ++p)
      for (int sl = 0; sl < qq; ++sl) n += s.shuffled[p * q + sl] == card;
    s.deck[card] = (int8_t)(s.deck[card] - n);
  }
  if (lane == 0) {
    const int rs = s.round_starter == -1 ? s.cp : (s.round_starter + 1) % P;
    s.cp = rs;
    s.round_starter = rs;
    for (int i = 0; i < 4; ++i) s.swap_choices[i] = -1;
    s.phase = (has(c.flags, R_TEAMS) && P == 4) ? 1 : 0;
    s.hand_size = q == 2 ? 6 : q - 1;
    s.deal = deal + 1;
  }
  Sync()();
}

// ---- transitions (lane 0) ---------------------------------------------------------------------------
__device__ __forceinline__ void dog_rebuild(const DetConsts& c, DogG& s) {
  for (int i = 0; i < kCells; ++i) s.board[i] = -1;
  for (int p = 0; p < c.P; ++p)
    for (int k = 0; k < 4; ++k) {
      const int pos = s.pins[p * 4 + k];
      if (pos >= 0 && pos < kCells) s.board[pos] = (int8_t)p;
    }
}

// winner / reward / done of a step_* function (dog.py:782-786 ...)
__device__ __forceinline__ void dog_finish(const DetConsts& c, const DogG& s, int cp, bool invalid, int& reward,
                                           int& done) {
  const uint32_t w = dog_winners(c, s.board);
  done = (s.done || w) ? 1 : 0;
  reward = s.done ? 0 : (invalid ? -1 : (int)((w >> cp) & 1u));
}

// `legal`: the caller drew the action from the legal mask of this very state, so the step function's own
// validity check (the same predicate) is skipped.
__device__ void dog_step_swap(const DetConsts& c, DogG& s, int cp, int pin, int pos, int& reward, int& done,
                              bool legal = false) {
  const bool invalid = !legal && !dog_val_swap(c, s, cp, pin, pos);
  if (!invalid) {
    const int sp = s.board[pos];
    const int pp = s.pins[cp * 4 + pin];
    s.board[pos] = (int8_t)cp;
    s.board[pp] = (int8_t)sp;
    s.pins[cp * 4 + pin] = (int8_t)pos;
    for (int k = 0; k < 4; ++k)
      if (s.pins[sp * 4 + k] == pos) s.pins[sp * 4 + k] = (int8_t)pp;
  }
  dog_finish(c, s, cp, invalid, reward, done);
}

// `legal` (k_dog_play): the board equals set_pins_on_board(pins) before the move (every transition ends
// with a rebuild or the equivalent swap update), the mover is on the board or at home and npos is a cell,
// so the rebuild reduces to clearing the mover's old cell and writing its new one: the captured pin sat
// on npos, which the mover now takes.
__device__ void dog_capture_move(const DetConsts& c, DogG& s, int cp, int pin, int npos, bool invalid, int& reward,
                                 int& done, bool legal = false) {
  if (!invalid) {
    const int at = s.board[jidx(npos, kCells)];
    if (at != -1 && (at != cp || has(c.flags, R_FRIENDLY)))
      for (int k = 0; k < 4; ++k)
        if (s.pins[at * 4 + k] == npos) s.pins[at * 4 + k] = -1;
    const int cur = s.pins[cp * 4 + pin];
    s.pins[cp * 4 + pin] = (int8_t)npos;
    if (legal && npos >= 0 && npos < kCells) {   // incremental board update (a validated move)
      if (cur >= 0 && cur < kCells) s.board[cur] = -1;
      s.board[npos] = (int8_t)cp;
    } else {
      dog_rebuild(c, s);
    }
  }
  dog_finish(c, s, cp, invalid, reward, done);
}

__device__ void dog_step_normal(const DetConsts& c, DogG& s, int cp, int pin, int move, int& reward, int& done,
                                bool legal = false) {
  const uint32_t F = c.flags;
  const bool invalid = !legal && !dog_val_normal(c, s, cp, pin, move);
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = dcst(c.target, cp);
  const int g0 = dgoal(c, cp, 0);
  const int cur = s.pins[cp * 4 + pin];
  const int moved = cur + move;
  const int fitted = fmodp(moved, kTrack);
  const int x = moved - tgt - mt;
  const bool ing = in_goal_p(c, cp, cur);
  const bool a = ing ? dog_goal_free(c, s.board, cp, cur - g0, moved - g0 + 1) : dog_goal_free(c, s.board, cp, -1, x);
  const int gx = dgoal(c, cp, jidx(x - 1, 4));
  const bool A = (s.board[gx] != cp) && (has(F, R_JUMP_GOAL) || a);
  int npos;
  if (cur == -1)
    npos = dcst(c.start, cp);
  else if (ing)
    npos = moved;
  else if (4 >= x && x > 0 && A && cur <= tgt)
    npos = gx;
  else
    npos = fitted;
  dog_capture_move(c, s, cp, pin, npos, invalid, reward, done, legal);
}

__device__ void dog_step_neg(const DetConsts& c, DogG& s, int cp, int pin, int& reward, int& done, int move = -4,
                             bool legal = false) {
  const bool invalid = !legal && !dog_val_neg(c, s, cp, pin, move);
  dog_capture_move(c, s, cp, pin, fmodp(s.pins[cp * 4 + pin] + move, kTrack), invalid, reward, done, legal);
}

// path bits [si, ei] (wrap when si > ei) inside [0, N); empty for a pin at home or not moving
__device__ __forceinline__ unsigned long long path_bits(int si, int ei, int N, bool same_area) {
  if (si == -1 || ei == -1 || (same_area && si == ei)) return 0ull;
  const unsigned long long full = N >= 64 ? ~0ull : ((1ull << N) - 1ull);
  auto ge = [&](int a) { return a <= 0 ? full : (a >= N ? 0ull : (full & ~((1ull << a) - 1ull))); };   // idx >= a
  auto le = [&](int b) { return b < 0 ? 0ull : (b >= N - 1 ? full : ((1ull << (b + 1)) - 1ull)); };    // idx <= b
  return si <= ei ? (ge(si) & le(ei)) : (ge(si) | le(ei));
}

__device__ void dog_step_hot7(const DetConsts& c, DogG& s, int cp, const int (&d)[4], int& reward, int& done,
                              bool legal = false) {
  const uint32_t F = c.flags;
  const bool invalid = !legal && !dog_val7(c, s, cp, d);
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = dcst(c.target, cp);
  int cur[4], moved[4], npos[4];
  bool ing[4];
  for (int k = 0; k < 4; ++k) {
    cur[k] = s.pins[cp * 4 + k];
    moved[k] = cur[k] + d[k];
    ing[k] = in_goal_p(c, cp, cur[k]);
  }
  bool occ[4];
  for (int g = 0; g < 4; ++g) {
    bool o = false;
    for (int k = 0; k < 4; ++k) o |= (ing[k] ? moved[k] : cur[k]) == dgoal(c, cp, g);
    occ[g] = o;
  }
  for (int k = 0; k < 4; ++k) {
    const int x = moved[k] - tgt - mt;
    bool a = true;
    if (!ing[k])
      for (int g = 0; g < 4; ++g)
        if (-1 < g && g < x) a &= !occ[g];
    const bool A = has(F, R_JUMP_GOAL) || a;
    if (cur[k] == -1)
      npos[k] = -1;
    else if (ing[k])
      npos[k] = moved[k];
    else if (4 >= x && x > 0 && A && cur[k] <= tgt)
      npos[k] = dgoal(c, cp, jidx(x - 1, 4));
    else
      npos[k] = fmodp(moved[k], kTrack);
  }
  // get_path_matrix (utils 237-303), rows as 56-bit masks
  unsigned long long row[4];
  bool cross = false;
  const int g0 = dgoal(c, cp, 0);
  for (int k = 0; k < 4; ++k) {
    const bool A0 = in_goal_p(c, cp, cur[k]), B0 = in_goal_p(c, cp, npos[k]);
    cross |= A0 != B0;
    row[k] = (A0 == B0) ? path_bits(cur[k], npos[k], kTrack, true)
                        : (path_bits(cur[k], tgt, kTrack, false) | path_bits(g0, npos[k], kCells, false));
  }
  if (cross)
    for (int k = 0; k < 4; ++k) row[k] |= 1ull << dcst(c.start, cp);
  const unsigned long long anyp = row[0] | row[1] | row[2] | row[3];
  if (!invalid) {
    uint32_t hit = 0;   // bit p*4+k
    for (int j = 0; j < c.P * 4; ++j) hit |= (uint32_t)((anyp >> jidx(s.pins[j], kCells)) & 1ull) << j;
    hit &= ~(0xFu << (4 * cp));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unsigned long long other = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j != k) other |= row[j];
      const bool h = ((other >> jidx(cur[k], kCells)) & 1ull) && ((other >> jidx(npos[k], kCells)) & 1ull);
      hit |= (uint32_t)h << (4 * cp + k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s.pins[cp * 4 + k] = (int8_t)npos[k];
    for (int j = 0; j < c.P * 4; ++j)
      if ((hit >> j) & 1u) s.pins[j] = -1;
    dog_rebuild(c, s);
  }
  dog_finish(c, s, cp, invalid, reward, done);
}

// Cards in each player's hand: the 56 hand bytes as 7 eight-byte LDS reads (memcpy, no type pun), summed
// 4 bytes at a time.  Counts can go negative (the swap phase decrements without a check, dog.py:1084), so
// each dword's byte sum is v_sad_u8's unsigned sum minus 256 per byte with the sign bit set.  Player p owns
// bytes [14p, 14p + 14).  (Round 1 blamed this function for k_dog_play's run-to-run differences; the cause
// was the unordered s.done read in the turn loop, see k_dog_play.)
__device__ __forceinline__ void dog_hand_counts(const DogG& s, int (&h)[4]) {
  static_assert(__builtin_offsetof(DogG, hands) % 8 == 0, "hands must be 8-byte aligned");
  uint32_t d[14];
  __builtin_memcpy(d, &s.hands[0][0], sizeof(d));
  auto ssum = [](uint32_t x) { return (int)__builtin_amdgcn_sad_u8(x, 0u, 0u) - 256 * __popc(x & 0x80808080u); };
  h[0] = ssum(d[0]) + ssum(d[1]) + ssum(d[2]) + ssum(d[3] & 0xFFFFu);
  h[1] = ssum(d[3] >> 16) + ssum(d[4]) + ssum(d[5]) + ssum(d[6]);
  h[2] = ssum(d[7]) + ssum(d[8]) + ssum(d[9]) + ssum(d[10] & 0xFFFFu);
  h[3] = ssum(d[10] >> 16) + ssum(d[11]) + ssum(d[12]) + ssum(d[13]);
}

// next player holding cards after the UNSUBSTITUTED current player (fori_loop of dog.py:1042-1046)
__device__ __forceinline__ int dog_next_with_cards(const DetConsts& c, const DogG& s, int& total) {
  int h[4];
  dog_hand_counts(s, h);
  int nxt = -1;
  total = 0;
  for (int p = 0; p < c.P; ++p) total += h[p];
  for (int i = 0; i < c.P; ++i) {
    const int cand = (s.cp + i + 1) % c.P;
    const int hc = cand == 0 ? h[0] : cand == 1 ? h[1] : cand == 2 ? h[2] : h[3];
    if (nxt == -1 && hc > 0) nxt = cand;
  }
  return nxt;
}

// env_step (dog.py:1117-1131) on lane 0; returns 1 when a deal must follow.
__device__ int dog_env_step(const DetConsts& c, DogG& s, int action, int& reward, int& done, bool legal = false) {
  if (s.phase == 1) {   // env_step_swap_phase (1077-1114): no validity check
    const int card = action - kDogPlay;
    const int cp0 = s.cp;
    const int ci = card < 0 ? card + kDogCards : card;   // .at[cp, card].add(-1): normalise once, drop OOB
    if (ci >= 0 && ci < kDogCards) s.hands[cp0][ci] = (int8_t)(s.hands[cp0][ci] - 1);
    s.swap_choices[cp0] = (int8_t)card;                   // jnp.int8(card_idx) wraps
    const int nxt = (cp0 + 1) % c.P;
    if (nxt == s.round_starter) {
      for (int p = 0; p < c.P; ++p) {   // execute_team_swap: partner of p is (p + 2) % 4
        const int rc = s.swap_choices[(p + 2) & 3];
        if (rc >= 0 && rc < kDogCards) s.hands[p][rc] = (int8_t)(s.hands[p][rc] + 1);
      }
      for (int i = 0; i < 4; ++i) s.swap_choices[i] = -1;
      s.phase = 0;
      s.cp = s.round_starter;
    } else {
      s.cp = nxt;
    }
    s.reward = 0;
    reward = 0;
    done = s.done;
    return 0;
  }
  // env_step_play_phase (986-1062)
  const int cp = dog_sub(c, s);
  const bool joker = action < kDogBase;
  const int act = ((action % kDogBase) + kDogBase) % kDogBase;
  const int card = joker ? 0 : dog_base_card(act);
  if (s.hands[cp][card] <= 0) {
    reward = -1;
    done = s.done;
  } else if (act < kDogSwaps) {
    dog_step_swap(c, s, cp, act / kCells, act % kCells, reward, done, legal);
  } else if (act < kDogNormalBase) {
    int d[4];
    for (int k = 0; k < 4; ++k) d[k] = c_dists7[act - kDogSwaps][k];
    dog_step_hot7(c, s, cp, d, reward, done, legal);
  } else if (act < kDogNegBase) {
    const int na = act - kDogNormalBase;
    int mv = na % 12 + 1;
    mv += mv >= 7 ? 1 : 0;
    dog_step_normal(c, s, cp, na / 12, mv, reward, done, legal);
  } else {
    dog_step_neg(c, s, cp, act - kDogNegBase, reward, done, -4, legal);
  }
  if (reward != -1) s.hands[cp][card] = (int8_t)(s.hands[cp][card] - 1);
  int total;
  const int nxt = dog_next_with_cards(c, s, total);
  s.cp = done ? cp : nxt;
  s.reward = reward;
  s.done = done;
  (void)total;   // all(hand_cards == 0) implies nxt == -1 (dog.py:1059); per-player, not summed
  return (nxt == -1 && !done) ? 1 : 0;
}

// ---- play-phase env_step on one whole wave (k_dog_play) -------------------------------------------------------
// The same transition as dog_env_step(.., legal = true), with the game's state spread over the 64 lanes instead of
// re-read from LDS by one lane: lane i < 56 holds board[i], lane j < 16 pins[j], lane 16p + k (k < 14) hands[p][k].
// The scalar logic runs redundantly on every lane with wave-uniform values, so a board / pin lookup is a readlane
// (a few cycles) instead of a dependent LDS round trip; the board rebuild, the occupancy tests of the winner check
// and the hand sums of the next-player search are per-lane work plus a ballot or a 16-lane row sum.  Round 3 measured
// lane 0's LDS-bound env_step at 30 % of a DOG turn (profiles/r3_dog_stamps.log).
struct DogWave {
  int lane;
  int cell;   // board[lane] (lane < kCells)
  int pin;    // pins[lane] (lane < 16)
  int hand;   // hands[lane >> 4][lane & 15] (lane & 15 < kDogCards; 0 otherwise)
  __device__ __forceinline__ int board(int x) const { return __builtin_amdgcn_readlane(cell, x); }
  __device__ __forceinline__ void set_board(int x, int v) { cell = lane == x ? v : cell; }
  __device__ __forceinline__ int pins(int j) const { return __builtin_amdgcn_readlane(pin, j); }
  __device__ __forceinline__ void set_pin(int j, int v) { pin = lane == j ? v : pin; }
  // goal cells of every player as 56-bit masks (kernel constants)
  __device__ __forceinline__ static unsigned long long goal_mask(const DetConsts& c, int p) {
    unsigned long long m = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) m |= 1ull << dgoal(c, p, g);
    return m;
  }
  __device__ __forceinline__ unsigned long long occupied() const { return __ballot(lane < kCells && cell >= 0); }
  __device__ __forceinline__ static bool player_done(const DetConsts& c, unsigned long long occ, int p) {
    const unsigned long long gm = goal_mask(c, p);
    return p < c.P && (occ & gm) == gm;
  }
  // dog_winners over the occupancy mask
  __device__ __forceinline__ uint32_t winners(const DetConsts& c) const {
    const unsigned long long occ = occupied();
    uint32_t d = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) d |= player_done(c, occ, p) ? (1u << p) : 0u;
    if (!has(c.flags, R_TEAMS)) return d;
    const bool t0 = (d & 1u) && (d & 4u), t1 = (d & 2u) && (d & 8u);
    if ((t0 && t1) || !(t0 || t1)) return 0u;
    return t0 ? 0x5u : 0xAu;
  }
  // set_pins_on_board: every cell cleared, then each pin's owner written in (p, k) order
  __device__ __forceinline__ void rebuild(const DetConsts& c) {
    int v = -1;
    for (int j = 0; j < c.P * 4; ++j) {
      const int pos = pins(j);
      v = (pos == lane) ? (j >> 2) : v;   // pos in [0, 56) whenever it matches a board lane
    }
    cell = v;
  }
  __device__ __forceinline__ bool goal_free(const DetConsts& c, int cp, int lo, int hi) const {
    bool ok = true;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (lo < g && g < hi) ok &= board(dgoal(c, cp, g)) != cp;
    return ok;
  }
};

__device__ __forceinline__ void wv_finish(const DetConsts& c, const DogWave& W, int sdone, int cp, int& reward,
                                          int& done) {
  const uint32_t w = W.winners(c);
  done = (sdone || w) ? 1 : 0;
  reward = sdone ? 0 : (int)((w >> cp) & 1u);
}

__device__ __forceinline__ void wv_capture_move(const DetConsts& c, DogWave& W, int sdone, int cp, int pin, int npos,
                                                int& reward, int& done) {
  const int at = W.board(jidx(npos, kCells));
  if (at != -1 && (at != cp || has(c.flags, R_FRIENDLY)))
    for (int k = 0; k < 4; ++k)
      if (W.pins(at * 4 + k) == npos) W.set_pin(at * 4 + k, -1);
  const int cur = W.pins(cp * 4 + pin);
  W.set_pin(cp * 4 + pin, npos);
  if (npos >= 0 && npos < kCells) {
    if (cur >= 0 && cur < kCells) W.set_board(cur, -1);
    W.set_board(npos, cp);
  } else {
    W.rebuild(c);
  }
  wv_finish(c, W, sdone, cp, reward, done);
}

__device__ __forceinline__ void wv_step_normal(const DetConsts& c, DogWave& W, int sdone, int cp, int pin, int move,
                                               int& reward, int& done) {
  const uint32_t F = c.flags;
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = dcst(c.target, cp);
  const int g0 = dgoal(c, cp, 0);
  const int cur = W.pins(cp * 4 + pin);
  const int moved = cur + move;
  const int fitted = fmodp(moved, kTrack);
  const int x = moved - tgt - mt;
  const bool ing = in_goal_p(c, cp, cur);
  const bool a = ing ? W.goal_free(c, cp, cur - g0, moved - g0 + 1) : W.goal_free(c, cp, -1, x);
  const int gx = dgoal(c, cp, jidx(x - 1, 4));
  const bool A = (W.board(gx) != cp) && (has(F, R_JUMP_GOAL) || a);
  int npos;
  if (cur == -1)
    npos = dcst(c.start, cp);
  else if (ing)
    npos = moved;
  else if (4 >= x && x > 0 && A && cur <= tgt)
    npos = gx;
  else
    npos = fitted;
  wv_capture_move(c, W, sdone, cp, pin, npos, reward, done);
}

__device__ __forceinline__ void wv_step_swap(const DetConsts& c, DogWave& W, int sdone, int cp, int pin, int pos,
                                             int& reward, int& done) {
  const int sp = W.board(pos);
  const int pp = W.pins(cp * 4 + pin);
  W.set_board(pos, cp);
  W.set_board(pp, sp);
  W.set_pin(cp * 4 + pin, pos);
  for (int k = 0; k < 4; ++k)
    if (W.pins(sp * 4 + k) == pos) W.set_pin(sp * 4 + k, pp);
  wv_finish(c, W, sdone, cp, reward, done);
}

__device__ __forceinline__ void wv_step_hot7(const DetConsts& c, DogWave& W, int sdone, int cp, const int (&d)[4],
                                             int& reward, int& done) {
  const uint32_t F = c.flags;
  const int mt = has(F, R_MUST_TRAVERSE) ? 1 : 0;
  const int tgt = dcst(c.target, cp);
  int cur[4], moved[4], npos[4];
  bool ing[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    cur[k] = W.pins(cp * 4 + k);
    moved[k] = cur[k] + d[k];
    ing[k] = in_goal_p(c, cp, cur[k]);
  }
  bool occ[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bool o = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) o |= (ing[k] ? moved[k] : cur[k]) == dgoal(c, cp, g);
    occ[g] = o;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = moved[k] - tgt - mt;
    bool a = true;
    if (!ing[k])
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (-1 < g && g < x) a &= !occ[g];
    const bool A = has(F, R_JUMP_GOAL) || a;
    if (cur[k] == -1)
      npos[k] = -1;
    else if (ing[k])
      npos[k] = moved[k];
    else if (4 >= x && x > 0 && A && cur[k] <= tgt)
      npos[k] = dgoal(c, cp, jidx(x - 1, 4));
    else
      npos[k] = fmodp(moved[k], kTrack);
  }
  unsigned long long row[4];
  bool cross = false;
  const int g0 = dgoal(c, cp, 0);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool A0 = in_goal_p(c, cp, cur[k]), B0 = in_goal_p(c, cp, npos[k]);
    cross |= A0 != B0;
    row[k] = (A0 == B0) ? path_bits(cur[k], npos[k], kTrack, true)
                        : (path_bits(cur[k], tgt, kTrack, false) | path_bits(g0, npos[k], kCells, false));
  }
  if (cross)
#pragma unroll
    for (int k = 0; k < 4; ++k) row[k] |= 1ull << dcst(c.start, cp);
  const unsigned long long anyp = row[0] | row[1] | row[2] | row[3];
  // pins hit: lane j tests its own pin (one ballot instead of 16 lookups)
  const bool hj = W.lane < c.P * 4 && ((anyp >> jidx(W.pin, kCells)) & 1ull);
  uint32_t hit = (uint32_t)__ballot(hj);
  hit &= ~(0xFu << (4 * cp));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    unsigned long long other = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j != k) other |= row[j];
    const bool h = ((other >> jidx(cur[k], kCells)) & 1ull) && ((other >> jidx(npos[k], kCells)) & 1ull);
    hit |= (uint32_t)h << (4 * cp + k);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) W.set_pin(cp * 4 + k, npos[k]);
  if (W.lane < 16 && ((hit >> W.lane) & 1u)) W.pin = -1;
  W.rebuild(c);
  wv_finish(c, W, sdone, cp, reward, done);
}

// play-phase env_step for an action drawn from the legal mask, all 64 lanes of one wave (lane = tid); returns 1 when
// a deal must follow (wave-uniform) and writes the state back to LDS
__device__ int dog_env_step_play_wave(const DetConsts& c, DogG& s, int action, int lane, int& reward, int& done) {
  DogWave W;
  W.lane = lane;
  W.cell = lane < kCells ? s.board[lane] : -1;
  W.pin = lane < 16 ? s.pins[lane] : -1;
  const int hp = lane >> 4, hk = lane & 15;
  W.hand = hk < kDogCards ? s.hands[hp][hk] : 0;
  const int scp = s.cp, sdone = s.done;
  const int cp = (has(c.flags, R_TEAMS) && DogWave::player_done(c, W.occupied(), scp)) ? (scp + 2) % 4 : scp;
  const bool joker = action < kDogBase;
  const int act = ((action % kDogBase) + kDogBase) % kDogBase;
  const int card = joker ? 0 : dog_base_card(act);
  if (__builtin_amdgcn_readlane(W.hand, cp * 16 + card) <= 0) {
    reward = -1;
    done = sdone;
  } else if (act < kDogSwaps) {
    wv_step_swap(c, W, sdone, cp, act / kCells, act % kCells, reward, done);
  } else if (act < kDogNormalBase) {
    int d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = c_dists7[act - kDogSwaps][k];
    wv_step_hot7(c, W, sdone, cp, d, reward, done);
  } else if (act < kDogNegBase) {
    const int na = act - kDogNormalBase;
    int mv = na % 12 + 1;
    mv += mv >= 7 ? 1 : 0;
    wv_step_normal(c, W, sdone, cp, na / 12, mv, reward, done);
  } else {
    wv_capture_move(c, W, sdone, cp, act - kDogNegBase, fmodp(W.pins(cp * 4 + act - kDogNegBase) - 4, kTrack), reward,
                    done);
  }
  if (reward != -1 && lane == cp * 16 + card) W.hand -= 1;
  // next player holding cards after the unsubstituted current player: per-player hand sums as 16-lane row sums
  int h = W.hand;
  h += __builtin_amdgcn_update_dpp(0, h, 0xB1, 0xF, 0xF, false);    // quad_perm xor 1
  h += __builtin_amdgcn_update_dpp(0, h, 0x4E, 0xF, 0xF, false);    // quad_perm xor 2
  h += __builtin_amdgcn_update_dpp(0, h, 0x141, 0xF, 0xF, false);   // row_half_mirror
  h += __builtin_amdgcn_update_dpp(0, h, 0x140, 0xF, 0xF, false);   // row_mirror
  int nxt = -1;
  for (int i = 0; i < c.P; ++i) {
    const int cand = (scp + i + 1) % c.P;
    if (nxt == -1 && __builtin_amdgcn_readlane(h, cand * 16) > 0) nxt = cand;
  }
  // write back
  if (lane < kCells) s.board[lane] = (int8_t)W.cell;
  if (lane < 16) s.pins[lane] = (int8_t)W.pin;
  if (hk < kDogCards) s.hands[hp][hk] = (int8_t)W.hand;
  if (lane == 0) {
    s.cp = done ? cp : nxt;
    s.reward = reward;
    s.done = done;
  }
  return (nxt == -1 && !done) ? 1 : 0;
}

// no_step (dog.py:713-752) on lane 0; returns 1 when a deal must follow.
__device__ int dog_no_step(const DetConsts& c, DogG& s) {
  for (int k = 0; k < kDogCards; ++k) s.hands[s.cp][k] = 0;
  int total;
  const int nxt = dog_next_with_cards(c, s, total);
  (void)total;   // any(hand_cards > 0) <=> nxt != -1 (dog.py:752)
  if (nxt != -1) {
    s.cp = nxt;
    return 0;
  }
  return 1;
}

// ---- kernels ----------------------------------------------------------------------------------------
// env_reset (dog.py:83-186) of the game in LDS, first deal included.  `deal` is the deal counter to
// continue from (0 for a fresh batch; the running count when a finished game is restarted in place, so
// that the new episode draws new shuffle keys).
template <class Sync>
__device__ void dog_reset_lds(const DetConsts& c, DogG& s, unsigned long long seed, int g, unsigned deal, int tid) {
  const bool fp = has(c.flags, R_FREE_PIN);
  if (tid < 16) {
    const int p = tid / 4, k = tid % 4;
    s.pins[tid] = (int8_t)((p < c.P) ? ((fp && k == 0) ? c.start[p] : -1) : -1);
  }
  for (int i = tid; i < 4 * kDogCards; i += Sync::N) s.hands[i / kDogCards][i % kDogCards] = 0;
  if (tid < kDogCards) s.deck[tid] = tid == 0 ? 6 : 8;   // env_reset: joker 6, others 8 (dog.py:143-145)
  if (tid < 4) s.swap_choices[tid] = -1;
  if (tid == 0) {
    s.cp = c.starting_player >= 0 ? c.starting_player : start_seat(game_key(seed, g, (int)deal), c.P);
    s.round_starter = -1;
    s.phase = 0;
    s.hand_size = 6;
    s.done = 0;
    s.reward = 0;
    s.deal = deal;
  }
  Sync()();
  if (tid == 0) dog_rebuild(c, s);
  Sync()();
  dog_deal<Sync>(c, s, seed, g, tid);
}

__global__ __launch_bounds__(256) void k_dog_reset(DetConsts c, muz_dog_soa st, unsigned long long seed, int n) {
  __shared__ DogG sg[kDogGamesPerBlock];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = blockIdx.x * kDogGamesPerBlock + w;
  if (g >= n) return;
  DogG& s = sg[w];
  dog_reset_lds<WaveSync>(c, s, seed, g, 0u, lane);
  dog_store<WaveSync>(c, st, g, s, lane);
}

// ---- block-per-game legality -----------------------------------------------------------------------
// Thread t of the 448 checks one base action: waves 0-3 the 224 swaps, waves 4-5 the 120 hot-7 splits,
// wave 6 the 48 normal moves and 4 "-4" moves, so every wave runs one kind of check (no divergence
// between kinds).  The result bit of base action i sits at slot dog_slot(i) of s.wb.
__device__ __forceinline__ int dog_check_of(int tid) {
  const int w = tid >> 6, l = tid & 63;
  if (w < 4) return w * 64 + l < kDogSwaps ? w * 64 + l : -1;
  if (w < 6) return kDogSwaps + (w - 4) * 64 + l < kDogNormalBase ? kDogSwaps + (w - 4) * 64 + l : -1;
  return l < kDogBase - kDogNormalBase ? kDogNormalBase + l : -1;
}
__device__ __forceinline__ int dog_slot(int i) {
  return i < kDogSwaps ? i : (i < kDogNormalBase ? 256 + i - kDogSwaps : 384 + i - kDogNormalBase);
}

// Base checks of the game in LDS into s.wb (all threads; ends with a block barrier).  Checks run only for
// actions whose joker or real card is in the (substituted) player's hand: the others are masked anyway.
__device__ __forceinline__ void dog_checks_block(const DetConsts& c, DogG& s, int tid) {
  if (s.phase == 0) {
    const int cp = dog_sub(c, s);
    const int i = dog_check_of(tid);
    const bool v = i >= 0 && (s.hands[cp][0] > 0 || s.hands[cp][dog_base_card(i)] > 0) && dog_base_valid(c, s, cp, i);
    const unsigned long long b = __ballot(v);
    if ((tid & 63) == 0) s.wb[tid >> 6] = b;
  }
  __syncthreads();
}

// k_dog_play's checks: as dog_checks_block, but the joker and real-card copies of each base action are
// gated by the hand right here (two ballots), so the legal set is 14 slot-ordered words (wj then wr) in
// LDS instead of the 806-bit mask.  Slot order is base order, so the k-th set bit over wj[0..6], wr[0..6]
// is the k-th legal action in action order (joker copies [0, 396) before real copies [396, 792)).
// (thread t of an NTH-thread workgroup takes check threads t, t + NTH, ... of the 448; NTH a multiple of 64, so
// each pass is whole waves and the ballots stay per check wave)
#ifndef MUZ_DOG_D7_LDS
#define MUZ_DOG_D7_LDS 1        // the hot-7 distribution table in LDS for the lean checks (0: __constant__ loads)
#endif
#ifndef MUZ_DOG_LEAN_CHECKS
#define MUZ_DOG_LEAN_CHECKS 1   // k_dog_play's checks on dog.hpp's lean predicates (0: dog_base_valid, A/B)
#endif
#ifndef MUZ_DOG_PAIRING
#define MUZ_DOG_PAIRING 0       // 1: k_dog_play pairs the hot-7 check waves with the normal wave / nothing (A/B: 0.4 % slower)
#endif
#ifdef MUZ_DOG_STAMPS
// diagnostic: per physical wave w, cycles of its check pass p (slot 8 + 4 p + w) and the number of passes that ran
// a check (slot 16 + 4 p + w), of the phase's setup before the passes (slot w: context build, its barrier, hoisted
// loads) and of the wait at the closing barrier (slot 4 + w), lane 0 of every wave; summed in LDS over the launch, added to the global totals once
// per workgroup at its end (per-pass global atomics from every workgroup serialised and distorted the turn)
__device__ unsigned long long g_dog_wave_stamps[24];
__device__ __forceinline__ unsigned long long* dog_wave_acc() {
  __shared__ unsigned long long acc[24];
  return acc;
}
#endif
template <int NTH = kDogBlockThreads>
__device__ __forceinline__ void dog_checks_play(const DetConsts& c, DogG& s, int tid, const uint32_t* d7 = nullptr,
                                                DogCtx* ctx = nullptr) {
  if (s.phase == 0) {
#ifdef MUZ_DOG_STAMPS
    const unsigned long long tp = __builtin_amdgcn_s_memtime();
#endif
#if MUZ_DOG_LEAN_CHECKS
    if (tid < 64) dog_ctx_turn(s, tid, ctx);   // the mover's uniform facts, once per check phase, in LDS
    __syncthreads();
    const DogCtx& x = *ctx;
    const int cp = x.cp;
#else
    const int cp = dog_sub(c, s);
#endif
    const bool hj = s.hands[cp][0] > 0;
#ifdef MUZ_DOG_STAMPS
    if ((tid & 63) == 0) dog_wave_acc()[tid >> 6] += __builtin_amdgcn_s_memtime() - tp;   // slots 0-3: setup
#endif
    // check wave of (physical wave w, pass p): NTH = 256 pairs the two hot-7 waves (the costliest pass, ~5.5 k
    // cycles when a 7 or joker is in hand) with the normal / -4 wave and nothing, and the four swap waves two by two,
    // so the longest physical wave of a joker turn is hot-7 + normal (~7.5 k) rather than swap + hot-7 (~8.8 k,
    // profiles/r5v_dog_play_stamps_lean.log); otherwise wave w takes check waves w, w + NTH / 64, ...
    for (int pass = 0; pass * NTH < kDogBlockThreads; ++pass) {
      const int pw = tid >> 6;
      int cw = (pass * NTH + tid) >> 6;
      if (NTH == 256 && MUZ_DOG_PAIRING) cw = pass == 0 ? (pw < 2 ? pw : pw + 2) : (pw < 2 ? pw + 2 : (pw == 2 ? 6 : 7));
      if (cw * 64 >= kDogBlockThreads) continue;   // (wave-uniform)
      const int vt = cw * 64 + (tid & 63);
#ifdef MUZ_DOG_STAMPS
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
      const int i = dog_check_of(vt);
      const bool hr = i >= 0 && s.hands[cp][dog_base_card(i)] > 0;
#if MUZ_DOG_LEAN_CHECKS
      const bool v = i >= 0 && (hj || hr) && dog_base_valid_lean(x, s, i, d7);
#else
      const bool v = i >= 0 && (hj || hr) && dog_base_valid(c, s, cp, i);
#endif
      const unsigned long long bj = __ballot(v && hj), br = __ballot(v && hr);
      if ((vt & 63) == 0) {
        s.wj[vt >> 6] = bj;
        s.wr[vt >> 6] = br;
      }
#ifdef MUZ_DOG_STAMPS
      const bool ran = __ballot(i >= 0 && (hj || hr)) != 0ull;
      if ((tid & 63) == 0 && pass < 2) {
        dog_wave_acc()[8 + 4 * pass + (tid >> 6)] += __builtin_amdgcn_s_memtime() - t0;
        if (ran) dog_wave_acc()[16 + 4 * pass + (tid >> 6)] += 1ull;
      }
#endif
    }
#ifdef MUZ_DOG_STAMPS
    const unsigned long long te = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if ((tid & 63) == 0) dog_wave_acc()[4 + (tid >> 6)] += __builtin_amdgcn_s_memtime() - te;   // slots 4-7: wait
#endif
  }
  __syncthreads();
}

__device__ __forceinline__ int dog_base_of_slot(int sl) {
  return sl < 256 ? sl : (sl < 384 ? kDogSwaps + sl - 256 : kDogNormalBase + sl - 384);
}

// The k-th legal action, k = floor(u * count) (kth_legal over dog_mask_words, same result), from the
// slot words of dog_checks_play (play phase) or the current player's cards (swap phase); -1 when nothing
// is legal.  One full wave; the bit inside the chosen word is found by a ballot over per-lane prefix counts.
__device__ __forceinline__ int dog_pick(const DogG& s, float u, int lane, int* count = nullptr) {
  unsigned long long w[14];
  if (s.phase == 0) {
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      w[r] = s.wj[r];
      w[7 + r] = s.wr[r];
    }
  } else {
    w[0] = __ballot(lane < kDogCards && s.hands[s.cp][lane < kDogCards ? lane : 0] > 0);
#pragma unroll
    for (int r = 1; r < 14; ++r) w[r] = 0ull;
  }
  int tot = 0;
#pragma unroll
  for (int r = 0; r < 14; ++r) tot += __popcll(w[r]);
  if (count) *count = tot;
  if (tot == 0) return -1;
  int k = (int)(u * (float)tot);
  k = k >= tot ? tot - 1 : k;
  int word = -1, kk = 0;
  unsigned long long x = 0;
#pragma unroll
  for (int r = 0; r < 14; ++r) {   // the word holding the k-th bit, without indexing w[] dynamically
    const int pc = __popcll(w[r]);
    if (word < 0) {
      if (k < pc) {
        word = r;
        x = w[r];
        kk = k;
      } else {
        k -= pc;
      }
    }
  }
  const bool set = (x >> lane) & 1ull;
  const int before = __popcll(x & ((1ull << lane) - 1ull));
  const int b = __ffsll((long long)__ballot(set && before == kk)) - 1;
  if (s.phase != 0) return kDogPlay + b;
  const int base = dog_base_of_slot((word % 7) * 64 + b);
  return word < 7 ? base : kDogBase + base;
}

// valid_actions (dog.py:693-711) from s.wb as 13 wave-uniform words (bit a of word a/64); one wave.
__device__ __forceinline__ void dog_mask_words(const DetConsts& c, const DogG& s, int lane, unsigned long long (&m)[13]) {
  const int cp = dog_sub(c, s);
#pragma unroll
  for (int r = 0; r < 13; ++r) {
    const int a = r * 64 + lane;
    bool v = false;
    if (a < kDogActions) {
      if (s.phase == 0) {
        if (a < kDogPlay) {
          const int i = a % kDogBase;
          const int sl = dog_slot(i);
          const bool bv = (s.wb[sl >> 6] >> (sl & 63)) & 1ull;
          v = bv && (a < kDogBase ? s.hands[cp][0] > 0 : s.hands[cp][dog_base_card(i)] > 0);
        }
      } else if (a >= kDogPlay) {
        v = s.hands[s.cp][a - kDogPlay] > 0;
      }
    }
    m[r] = __ballot(v);
  }
}

__global__ __launch_bounds__(kDogBlockThreads) void k_dog_legal(DetConsts c, muz_dog_soa st, uint32_t* mask, int n) {
  __shared__ DogG s;
  const int tid = threadIdx.x, g = blockIdx.x;
  dog_load<BlockSync>(c, st, g, s, tid);
  dog_checks_block(c, s, tid);
  if (tid >= 64) return;
  unsigned long long m[13];
  dog_mask_words(c, s, tid, m);
  uint32_t* out = mask + (size_t)g * kDogWords;
  if (tid < kDogWords) {
    unsigned long long x = m[0];
#pragma unroll
    for (int r = 1; r < 13; ++r)
      if ((tid >> 1) == r) x = m[r];
    out[tid] = (tid & 1) ? (uint32_t)(x >> 32) : (uint32_t)x;
  }
}

constexpr unsigned long long kRandomActionStream = 0x52A4D0DA11ull;

__device__ __forceinline__ float random_action_uniform(unsigned long long seed, int g, int turn) {
  return u24(mix64(game_key(seed ^ kRandomActionStream, g, turn)));
}

// The k-th set bit of a 13-word mask (wave-uniform inputs), -1 when empty; k = floor(u * count).
__device__ __forceinline__ int kth_legal(const unsigned long long (&m)[13], float u) {
  int tot = 0;
#pragma unroll
  for (int r = 0; r < 13; ++r) tot += __popcll(m[r]);
  if (tot == 0) return -1;
  int k = (int)(u * (float)tot);
  k = k >= tot ? tot - 1 : k;
  int word = -1, kk = 0;
  unsigned long long x = 0;
#pragma unroll
  for (int r = 0; r < 13; ++r) {   // the word holding the k-th bit, without indexing m[] dynamically
    const int pc = __popcll(m[r]);
    if (word < 0) {
      if (k < pc) {
        word = r;
        x = m[r];
        kk = k;
      } else {
        k -= pc;
      }
    }
  }
  for (int j = 0; j < kk; ++j) x &= x - 1;   // drop the kk lowest set bits
  return word * 64 + __ffsll((long long)x) - 1;
}

// Diagnostic build only (EXTRA=-DMUZ_DOG_STAMPS): per-phase shader-clock totals of k_dog_play, thread 0.
#ifdef MUZ_DOG_STAMPS
__device__ unsigned long long g_dog_stamps[8];
#define DOG_STAMP_INIT()                                                           \
  unsigned long long ds_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ds_last = __builtin_amdgcn_s_memtime(); \
  if (tid < 24) dog_wave_acc()[tid] = 0ull;                                          \
  __syncthreads()
#define DOG_STAMP(i)                                          \
  do {                                                        \
    if (tid == 0) {                                           \
      const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
      ds_acc[i] += _t - ds_last;                              \
      ds_last = _t;                                           \
    }                                                         \
  } while (0)
#define DOG_STAMP_END()                                                       \
  do {                                                                        \
    if (tid == 0)                                                             \
      for (int i = 0; i < 8; ++i) atomicAdd(&g_dog_stamps[i], ds_acc[i]);    \
    __syncthreads();                                                          \
    if (tid < 24) atomicAdd(&g_dog_wave_stamps[tid], dog_wave_acc()[tid]); \
  } while (0)
#else
#define DOG_STAMP_INIT() do {} while (0)
#define DOG_STAMP(i) do {} while (0)
#define DOG_STAMP_END() do {} while (0)
#endif

// Config (d)'s actor: `nturns` turns of one game per workgroup with the state resident in LDS --
// valid_actions -> uniform random legal action (turn0 + t) -> env_step, or no_step when nothing is legal
// -> deal if needed.  A finished game stops (action -2), or with `auto_reset` restarts in place
// (dog_reset_lds, deal counter continued) and keeps playing.  env_steps[g] (optional) accumulates the
// turns played and episodes[g] (optional) the games finished; action / reward / done (optional) are
// those of the last turn.
#ifndef MUZ_DOG_PRIO
#define MUZ_DOG_PRIO 1
#endif
#ifndef MUZ_DOG_WAVE_STEP
#define MUZ_DOG_WAVE_STEP 1   // the play-phase env_step on wave 0's 64 lanes (dog_env_step_play_wave)
#endif

struct DogPlayArgs {
  DetConsts c;
  muz_dog_soa st;
  unsigned long long seed;
  int turn0, nturns, auto_reset;
  int32_t* action_out;   // optional outputs of the last turn
  int8_t* reward;
  uint8_t* done;
  uint32_t* env_steps;   // optional accumulators
  uint32_t* episodes;
  muz_dog_traj rec;      // optional per-turn records (rec.act == null: none)
};

// All arguments come in one struct that the kernel reads through the kernarg segment (kernarg0: scalar
// loads, the pointer laundered at each use), so the rule constants and the SoA pointers are reloaded where
// they are needed instead of being held live across the turn loop -- at the 64-VGPR budget that kept
// state spilled SGPRs into VGPR lanes and VGPRs into scratch.
__global__ __launch_bounds__(kDogPlayThreads) __attribute__((amdgpu_waves_per_eu(kDogPlayWPE))) void k_dog_play(
    DogPlayArgs args) {
  (void)args;
  __shared__ DogG s;
  const int tid = threadIdx.x, g = blockIdx.x;
  auto A = []() -> const DogPlayArgs& { return *(const DogPlayArgs*)kernarg0<DogPlayArgs>(); };
  if (A().st.done[g] && !A().auto_reset) {
    if (tid == 0) {
      if (A().action_out) A().action_out[g] = -2;
      if (A().reward) A().reward[g] = 0;
      if (A().done) A().done[g] = 1;
    }
    return;
  }
  dog_load<PlaySync>(A().c, A().st, g, s, tid);
#if MUZ_DOG_LEAN_CHECKS && MUZ_DOG_D7_LDS
  // the hot-7 distributions packed into LDS once per launch (the checks read them per lane every turn)
  __shared__ uint32_t s_d7[kDogHot];
  for (int i = tid; i < kDogHot; i += kDogPlayThreads)
    s_d7[i] = (uint32_t)(uint8_t)c_dists7[i][0] | ((uint32_t)(uint8_t)c_dists7[i][1] << 8) |
              ((uint32_t)(uint8_t)c_dists7[i][2] << 16) | ((uint32_t)(uint8_t)c_dists7[i][3] << 24);
  __syncthreads();
  const uint32_t* d7 = s_d7;
#else
  const uint32_t* d7 = nullptr;
#endif
#if MUZ_DOG_LEAN_CHECKS
  __shared__ DogCtx s_ctx;
  DogCtx* ctx = &s_ctx;
  if (tid == 0) dog_ctx_static(A().c, ctx);   // ordered before the first turn's reads by dog_checks_play's barrier
#else
  DogCtx* ctx = nullptr;
#endif
  const int nturns = A().nturns;
  int played = 0, finished = 0, a = -2, r = 0;
  DOG_STAMP_INIT();
  for (int t = 0; t < nturns; ++t) {
    const DogPlayArgs& P = A();
    const DetConsts& c = P.c;
    // s.done is block-uniform: its last writer (lane 0's env_step) is ordered before these reads by the
    // turn-end barrier.  When the game ended, the barrier below keeps dog_reset_lds's s.done = 0 (tid 0,
    // before its first barrier) from overtaking a wave that has not read s.done yet -- without it, such a
    // wave read 0, skipped the reset, and its barriers paired with the wrong ones of the other waves
    // (the run-to-run differences of round 1).
    if (s.done) {
      if (!P.auto_reset) break;
      const unsigned deal = s.deal;
      __syncthreads();
      dog_reset_lds<PlaySync>(c, s, P.seed, g, deal, tid);
    }
    DOG_STAMP(0);   // reset
    dog_checks_play<kDogPlayThreads>(c, s, tid, d7, ctx);
    DOG_STAMP(1);   // base checks (+ barrier)
    if (tid < 64) {
      // the turn's serial part (choice, lane 0's env_step) runs at raised wave priority: the CU's other
      // workgroups are in their VALU-heavy check phases meanwhile, and without it this wave got a small share
      // of the SIMD's issue slots
      if (MUZ_DOG_PRIO) __builtin_amdgcn_s_setprio(2);
      int nleg = 0;
      a = dog_pick(s, random_action_uniform(P.seed, g, P.turn0 + t), tid, &nleg);
      DOG_STAMP(2);   // action choice
      const int mover = s.cp;
      int need = 0;
      if (MUZ_DOG_WAVE_STEP && a >= 0 && s.phase == 0) {   // wave-uniform: the play phase on all 64 lanes
        int d = 0;
        need = dog_env_step_play_wave(c, s, a, tid, r, d);
      } else if (tid == 0) {                              // no_step and the swap phase: lane 0
        int d = s.done;
        r = 0;
        need = a < 0 ? dog_no_step(c, s) : dog_env_step(c, s, a, r, d, true);
      }
      if (tid == 0) {
        s.need_deal = need;
        if (P.rec.act) {   // the turn's record row (game lane g, row idx[g] + turns recorded this launch)
          const int row = P.rec.idx[g] + played;
          if (row < P.rec.max_steps) {
            const size_t o = (size_t)g * P.rec.max_steps + row;
            P.rec.act[o] = a;
            P.rec.player[o] = mover;
            P.rec.reward[o] = r;
            P.rec.legal[o] = nleg;
            P.rec.done[o] = (uint8_t)s.done;
          }
        }
      }
      DOG_STAMP(3);   // env_step / no_step (lane 0)
      if (MUZ_DOG_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    ++played;
    __syncthreads();
    DOG_STAMP(4);   // barrier
    if (s.need_deal) dog_deal<PlaySync>(c, s, P.seed, g, tid);
    DOG_STAMP(5);   // deal
    finished += s.done;
  }
  DOG_STAMP_END();
  const DogPlayArgs& P = A();
  dog_store<PlaySync>(P.c, P.st, g, s, tid);
  if (tid == 0) {
    if (P.action_out) P.action_out[g] = a;
    if (P.reward) P.reward[g] = (int8_t)r;
    if (P.done) P.done[g] = (uint8_t)s.done;
    if (P.env_steps) P.env_steps[g] += (uint32_t)played;
    if (P.episodes) P.episodes[g] += (uint32_t)finished;
    if (P.rec.act) P.rec.idx[g] = min(P.rec.max_steps, P.rec.idx[g] + played);
  }
}

// mode 0: env_step(action[g]); mode 1: no_step.  action < 0 with mode 0 = no_step as well.
// restart != 0 (the MuZero self-play loop, muz_dog_step_restart): a game the step finished restarts in place after
// it (dog_reset_lds with the deal counter continued, as k_dog_play's auto reset) and episodes[g] counts it.
__global__ __launch_bounds__(256) void k_dog_step(DetConsts c, muz_dog_soa st, const int32_t* action, int mode,
                                                  unsigned long long seed, int8_t* reward, uint8_t* done, int n,
                                                  int restart = 0, uint32_t* episodes = nullptr) {
  __shared__ DogG sg[kDogGamesPerBlock];
  __shared__ int need_deal[kDogGamesPerBlock];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = blockIdx.x * kDogGamesPerBlock + w;
  if (g >= n) return;
  DogG& s = sg[w];
  dog_load<WaveSync>(c, st, g, s, lane);
  if (lane == 0) {
    int r = 0, d = s.done;
    int deal;
    if (mode == 1 || action[g] < 0) {
      deal = dog_no_step(c, s);
      r = 0;
      d = s.done;
    } else {
      deal = dog_env_step(c, s, action[g], r, d);
    }
    need_deal[w] = deal;
    if (reward) reward[g] = (int8_t)r;
    if (done) done[g] = (uint8_t)d;
  }
  wave_sync();
  if (need_deal[w]) dog_deal<WaveSync>(c, s, seed, g, lane);
  if (restart && s.done) {   // (one wave: every lane has read s.done before dog_reset_lds clears it)
    if (episodes && lane == 0) episodes[g] += 1u;
    dog_reset_lds<WaveSync>(c, s, seed, g, s.deal, lane);
  }
  dog_store<WaveSync>(c, st, g, s, lane);
}

// ---- DOG MuZero self-play records (config (e) as MuZero_DOG/train.py trains: play_n_games_v3's buffer dict) ------
// MuZero_DOG/game_agent.py:52-57 is `pass`; the det loop it copies (MuZero_det_MADN/game_agent.py:64-141) defines the
// record of a turn: obs (zeros on a no-move turn), action (-1), reward class {0: -1, 1: 0, 2: +1} of a game-ending
// step, root value, the search's action weights (zeros), mask (1 search turn, 0 no-move turn), the player and team
// BEFORE the move, and the discount class (1 terminal or no-move turn, 2 same team moves next, 0 the other team).
// One wave per lane (game in flight): the turn's record goes to row idx[slot] of the lane's trajectory slot
// (lane_game[g]; < 0: an idle lane, left untouched), then env_step / no_step as k_dog_step; a game that ended (done,
// or its max_steps-th record) restarts in place (deal counter continued) and sets ended[g] for k_dog_sp_assign.
constexpr int kDogObsBytes = 34 * kCells;   // (dog_nets.hpp kDogC x 56)

struct DogSpArgs {
  DetConsts c;
  muz_dog_soa st;
  const float* obs;         // [n][34][56] this turn's encode_board (the networks' input)
  const int32_t* action;    // [n] (-1: no legal action -> no_step)
  const float* weights;     // [n][806]
  const float* root_value;  // [n]
  unsigned long long seed;
  muz_traj traj;            // [num_games][T], obs int8 [34][56], pol [806]
  int32_t* lane_game;       // [n] trajectory slot of the lane's game, -1 idle
  int32_t* ended;           // [n] out: 1 when the lane's game ended this turn
  uint32_t* episodes;       // [n] nullable: finished (done) games per lane
  int n;
};

__global__ __launch_bounds__(256) void k_dog_sp_record_step(DogSpArgs P) {
  __shared__ DogG sg[kDogGamesPerBlock];
  __shared__ int sh_deal[kDogGamesPerBlock], sh_end[kDogGamesPerBlock];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = blockIdx.x * kDogGamesPerBlock + w;
  if (g >= P.n) return;
  const int slot = P.lane_game[g];
  if (slot < 0) {
    if (lane == 0) P.ended[g] = 0;
    return;
  }
  const DetConsts& c = P.c;
  DogG& s = sg[w];
  dog_load<WaveSync>(c, P.st, g, s, lane);
  const int T = P.traj.max_steps;
  const int t = P.traj.idx[slot];
  const int a = P.action[g];
  const int cp0 = s.cp;
  const size_t row = (size_t)slot * T + t;
  {   // the observation (int8, exact: values 0..110) and the policy of the turn
    const float* src = P.obs + (size_t)g * kDogObsBytes;
    int8_t* o = P.traj.obs + row * kDogObsBytes;
    for (int i = lane; i < kDogObsBytes; i += 64) o[i] = a >= 0 ? (int8_t)src[i] : (int8_t)0;
    const float* ws = P.weights + (size_t)g * kDogActions;
    float* pp = P.traj.pol + row * kDogActions;
    for (int i = lane; i < kDogActions; i += 64) pp[i] = a >= 0 ? ws[i] : 0.f;
  }
  int r = 0, d = 0;
  if (lane == 0) {
    int deal;
    if (a < 0) {
      deal = dog_no_step(c, s);
      d = s.done;
    } else {
      deal = dog_env_step(c, s, a, r, d);
    }
    sh_deal[w] = deal;
  }
  wave_sync();
  if (sh_deal[w]) dog_deal<WaveSync>(c, s, P.seed, g, lane);
  if (lane == 0) {
    const int cp1 = s.cp;     // next_env.current_player (after the step's deal)
    const bool teams = has(c.flags, R_TEAMS);
    const muz_traj& tr = P.traj;
    int rew = 1, disc = 1;
    if (a >= 0) {
      rew = (d && r > 0) ? 2 : ((d && r < 0) ? 0 : 1);
      disc = d ? 1 : ((teams ? (cp0 & 1) == (cp1 & 1) : cp0 == cp1) ? 2 : 0);
    }
    tr.act[row] = a >= 0 ? a : -1;
    tr.rew[row] = rew;
    tr.val[row] = a >= 0 ? P.root_value[g] : 0.f;
    tr.mask[row] = a >= 0 ? 1.f : 0.f;
    tr.player[row] = cp0;
    tr.team[row] = teams ? (cp0 & 1) : -1;
    tr.discount[row] = disc;
    tr.idx[slot] = t + 1;
    const int end = (d || t + 1 >= T) ? 1 : 0;
    P.ended[g] = end;
    sh_end[w] = end;
    if (P.episodes && d) P.episodes[g] += 1u;
  }
  wave_sync();
  if (sh_end[w]) dog_reset_lds<WaveSync>(c, s, P.seed, g, s.deal, lane);   // (every lane has read s.done / cp)
  dog_store<WaveSync>(c, P.st, g, s, lane);
}

// The lanes whose game ended take the next game numbers in lane order (one workgroup, deterministic): ctr[0] = next
// game number, ctr[1] = num_games, ctr[2] (out) = lanes still holding a game.  A lane past num_games goes idle.
__global__ __launch_bounds__(1024) void k_dog_sp_assign(int32_t* lane_game, const int32_t* ended, int32_t* idx,
                                                        int32_t* ctr, int n) {
  __shared__ int wsum[16];
  __shared__ int base_s, active_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) base_s = ctr[0], active_s = 0;
  __syncthreads();
  const int ng = ctr[1];
  for (int l0 = 0; l0 < n; l0 += 1024) {
    const int l = l0 + tid;
    const bool fin = l < n && lane_game[l] >= 0 && ended[l];
    const unsigned long long b = __ballot(fin);
    const int pre = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(b);
    __syncthreads();
    int off = base_s;
    for (int k = 0; k < w; ++k) off += wsum[k];
    if (fin) {
      const int slot = off + pre;
      lane_game[l] = slot < ng ? slot : -1;
      if (slot < ng) idx[slot] = 0;
    }
    const int act = (l < n && lane_game[l] >= 0) ? 1 : 0;
    const int wa = __popcll(__ballot(act));
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int k = 0; k < 16; ++k) tot += wsum[k];
      base_s += tot;
    }
    if (lane == 0 && wa) atomicAdd(&active_s, wa);
    __syncthreads();
  }
  if (tid == 0) {
    ctr[0] = base_s;
    ctr[2] = active_s;
  }
}

// One step_* function of dog.py on its own (the form DOG/test.py calls): kind 0 step_swap(pin, pos),
// 1 step_normal_move(pin, move), 2 step_neg_move(pin, move), 3 step_hot_7(d0..d3).  Board and pins change;
// hands, turn and the state's reward / done fields do not (the reference returns them separately).
__global__ __launch_bounds__(256) void k_dog_step_move(DetConsts c, muz_dog_soa st, const int32_t* kind,
                                                       const int32_t* args, int8_t* reward, uint8_t* done, int n) {
  __shared__ DogG sg[kDogGamesPerBlock];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = blockIdx.x * kDogGamesPerBlock + w;
  if (g >= n) return;
  DogG& s = sg[w];
  dog_load<WaveSync>(c, st, g, s, lane);
  if (lane == 0) {
    const int cp = dog_sub(c, s);
    const int k = kind[g];
    const int a0 = args[4 * g], a1 = args[4 * g + 1];
    int r = 0, d = s.done;
    if (k == 0) {
      dog_step_swap(c, s, cp, a0 < 0 ? 0 : (a0 > 3 ? 3 : a0), a1 < 0 ? 0 : (a1 > kCells - 1 ? kCells - 1 : a1), r, d);
    } else if (k == 1) {
      dog_step_normal(c, s, cp, a0 & 3, a1, r, d);
    } else if (k == 2) {
      dog_step_neg(c, s, cp, a0 & 3, r, d, a1);
    } else {
      const int dd[4] = {args[4 * g], args[4 * g + 1], args[4 * g + 2], args[4 * g + 3]};
      dog_step_hot7(c, s, cp, dd, r, d);
    }
    if (reward) reward[g] = (int8_t)r;
    if (done) done[g] = (uint8_t)d;
  }
  dog_store<WaveSync>(c, st, g, s, lane);
}

// Uniform random legal action (config (d)'s policy): the k-th set bit, k = floor(u * popcount); -1 if none.
__global__ __launch_bounds__(256) void k_dog_random_action(const uint32_t* mask, const float* uniform,
                                                           unsigned long long seed, int turn, int32_t* action, int n) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const uint32_t* m = mask + (size_t)g * kDogWords;
  int tot = 0;
  for (int i = 0; i < kDogWords; ++i) tot += __popc(m[i]);
  if (tot == 0) {
    action[g] = -1;
    return;
  }
  const float u = uniform ? uniform[g] : random_action_uniform(seed, g, turn);
  int k = (int)(u * (float)tot);
  k = k >= tot ? tot - 1 : k;
  int a = -1;
  for (int i = 0; i < kDogWords && a < 0; ++i) {
    const int pc = __popc(m[i]);
    if (k < pc) {
      uint32_t x = m[i];
      for (int j = 0; j < k; ++j) x &= x - 1;   // drop the k lowest set bits
      a = i * 32 + __ffs(x) - 1;
    } else {
      k -= pc;
    }
  }
  action[g] = a;
}

static int dog_consts(const muz_rules* rules, DetConsts* c) {
  int rc = make_det_consts(rules, c, true);   // every DOG reset has its seed (muz_dog_reset, the in-place restarts)
  if (rc) return rc;
  if (rules->disable_swapping || rules->disable_hot_seven || rules->disable_joker) return MUZ_E_UNSUPPORTED;
  return MUZ_OK;
}

static int dog_tables_ready() {
  static bool done = false;
  if (done) return MUZ_OK;
  int8_t t[kDogHot][4];
  int i = 0;
  for (int a = 0; a <= 7; ++a)
    for (int b = 0; b <= 7; ++b)
      for (int cc = 0; cc <= 7; ++cc) {
        const int d = 7 - a - b - cc;
        if (d >= 0) {
          t[i][0] = (int8_t)a;
          t[i][1] = (int8_t)b;
          t[i][2] = (int8_t)cc;
          t[i][3] = (int8_t)d;
          ++i;
        }
      }
  MUZ_HIP_RET(hipMemcpyToSymbol(HIP_SYMBOL(c_dists7), t, sizeof(t)));
  done = true;
  return MUZ_OK;
}

}  // namespace muz

using namespace muz;

static inline unsigned dog_blocks(int n) { return (unsigned)((n + kDogGamesPerBlock - 1) / kDogGamesPerBlock); }

#define DOG_PROLOGUE(extra)                           \
  DetConsts c;                                        \
  int rc = dog_consts(rules, &c);                     \
  if (rc) return rc;                                  \
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && extra);  \
  if ((rc = dog_tables_ready())) return rc;           \
  if (n == 0) return MUZ_OK;

extern "C" {

#ifdef MUZ_DOG_STAMPS
int muz_diag_dog_stamps(unsigned long long* host_out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_dog_stamps), sizeof(unsigned long long) * 8);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_dog_stamps), z, sizeof(z));
  }
  return (int)e;
}
// per-wave check passes (dog_checks_play): host_out[24] (slot layout at g_dog_wave_stamps)
int muz_diag_dog_wave_stamps(unsigned long long* host_out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_dog_wave_stamps), sizeof(unsigned long long) * 24);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[24] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_dog_wave_stamps), z, sizeof(z));
  }
  return (int)e;
}
#endif

int muz_dog_reset(const muz_rules* rules, muz_dog_soa st, uint64_t seed, int32_t n, void* stream) {
  DOG_PROLOGUE(true)
  k_dog_reset<<<dog_blocks(n), 256, 0, (hipStream_t)stream>>>(c, st, seed, n);
  return muz_last_launch_error();
}

int muz_dog_legal(const muz_rules* rules, muz_dog_soa st, uint32_t* mask, int32_t n, void* stream) {
  DOG_PROLOGUE(mask != nullptr)
  k_dog_legal<<<n, kDogBlockThreads, 0, (hipStream_t)stream>>>(c, st, mask, n);
  return muz_last_launch_error();
}

int muz_dog_step(const muz_rules* rules, muz_dog_soa st, const int32_t* action, uint64_t seed, int8_t* reward,
                 uint8_t* done, int32_t n, void* stream) {
  DOG_PROLOGUE(action != nullptr)
  k_dog_step<<<dog_blocks(n), 256, 0, (hipStream_t)stream>>>(c, st, action, 0, seed, reward, done, n);
  return muz_last_launch_error();
}

int muz_dog_step_restart(const muz_rules* rules, muz_dog_soa st, const int32_t* action, uint64_t seed, int8_t* reward,
                         uint8_t* done, uint32_t* episodes, int32_t n, void* stream) {
  DOG_PROLOGUE(action != nullptr)
  k_dog_step<<<dog_blocks(n), 256, 0, (hipStream_t)stream>>>(c, st, action, 0, seed, reward, done, n, 1, episodes);
  return muz_last_launch_error();
}

int muz_dog_sp_record_step(const muz_rules* rules, muz_dog_soa st, const float* obs, const int32_t* action,
                           const float* action_weights, const float* root_value, uint64_t seed, muz_traj traj,
                           int32_t* lane_game, int32_t* ended, uint32_t* episodes, int32_t n, void* stream) {
  DOG_PROLOGUE(obs && action && action_weights && root_value && lane_game && ended)
  MUZ_HOST_CHECK(c.P == 4 && traj.max_steps > 0 && traj.obs && traj.act && traj.rew && traj.val && traj.pol &&
                 traj.mask && traj.player && traj.team && traj.discount && traj.idx);
  k_dog_sp_record_step<<<dog_blocks(n), 256, 0, (hipStream_t)stream>>>(
      DogSpArgs{c, st, obs, action, action_weights, root_value, seed, traj, lane_game, ended, episodes, n});
  return muz_last_launch_error();
}

int muz_dog_sp_assign(int32_t* lane_game, const int32_t* ended, int32_t* traj_idx, int32_t* counters, int32_t n,
                      void* stream) {
  MUZ_HOST_CHECK(n >= 0 && lane_game && ended && traj_idx && counters);
  k_dog_sp_assign<<<1, 1024, 0, (hipStream_t)stream>>>(lane_game, ended, traj_idx, counters, n);
  return muz_last_launch_error();
}

int muz_dog_nostep(const muz_rules* rules, muz_dog_soa st, uint64_t seed, int8_t* reward, uint8_t* done, int32_t n,
                   void* stream) {
  DOG_PROLOGUE(true)
  k_dog_step<<<dog_blocks(n), 256, 0, (hipStream_t)stream>>>(c, st, nullptr, 1, seed, reward, done, n);
  return muz_last_launch_error();
}

int muz_dog_step_move(const muz_rules* rules, muz_dog_soa st, const int32_t* kind, const int32_t* args,
                      int8_t* reward, uint8_t* done, int32_t n, void* stream) {
  DOG_PROLOGUE(kind != nullptr && args != nullptr)
  k_dog_step_move<<<dog_blocks(n), 256, 0, (hipStream_t)stream>>>(c, st, kind, args, reward, done, n);
  return muz_last_launch_error();
}

int muz_dog_random_turn(const muz_rules* rules, muz_dog_soa st, uint64_t seed, int32_t turn, int32_t* action,
                        int8_t* reward, uint8_t* done, int32_t n, void* stream) {
  DOG_PROLOGUE(true)
  k_dog_play<<<n, kDogPlayThreads, 0, (hipStream_t)stream>>>(
      DogPlayArgs{c, st, seed, turn, 1, 0, action, reward, done, nullptr, nullptr});
  return muz_last_launch_error();
}

int muz_dog_random_play(const muz_rules* rules, muz_dog_soa st, uint64_t seed, int32_t turn0, int32_t nturns,
                        int32_t auto_reset, uint32_t* env_steps, uint32_t* episodes, int32_t n, void* stream) {
  DOG_PROLOGUE(nturns >= 0)
  if (nturns == 0) return MUZ_OK;
  k_dog_play<<<n, kDogPlayThreads, 0, (hipStream_t)stream>>>(
      DogPlayArgs{c, st, seed, turn0, nturns, auto_reset ? 1 : 0, nullptr, nullptr, nullptr, env_steps, episodes,
                  muz_dog_traj{}});
  return muz_last_launch_error();
}

int muz_dog_random_play_record(const muz_rules* rules, muz_dog_soa st, uint64_t seed, int32_t turn0, int32_t nturns,
                               int32_t auto_reset, uint32_t* env_steps, uint32_t* episodes, muz_dog_traj rec, int32_t n,
                               void* stream) {
  DOG_PROLOGUE(nturns >= 0)
  MUZ_HOST_CHECK(rec.act && rec.player && rec.reward && rec.legal && rec.done && rec.idx && rec.max_steps > 0);
  if (nturns == 0) return MUZ_OK;
  k_dog_play<<<n, kDogPlayThreads, 0, (hipStream_t)stream>>>(
      DogPlayArgs{c, st, seed, turn0, nturns, auto_reset ? 1 : 0, nullptr, nullptr, nullptr, env_steps, episodes, rec});
  return muz_last_launch_error();
}

int muz_dog_random_action(const uint32_t* mask, const float* uniform, uint64_t seed, int32_t turn, int32_t* action,
                          int32_t n, void* stream) {
  MUZ_HOST_CHECK(n >= 0 && mask && action);
  if (n == 0) return MUZ_OK;
  k_dog_random_action<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(mask, uniform, seed, turn, action, n);
  return muz_last_launch_error();
}

}  // extern "C"
