// Counter-based random numbers of the engine (splitmix64 finaliser over (seed, game, turn, ...)).
// The reference draws with jax threefry, which is not restated: every stream here is documented in
// include/muz.h and restated bit-exactly by the test oracles (oracle/selfplay.py, oracle/mctx_stochastic.py).
#pragma once
#include "common.hpp"

namespace muz {

constexpr float kTinyF = 1.1754943508222875e-38f;   // jnp.finfo(float32).tiny

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ unsigned long long game_key(unsigned long long seed, int gid, int turn) {
  return seed ^ mix64(((unsigned long long)(unsigned)gid << 32) | (unsigned)turn);
}
// U[0, 1) on a 24-bit grid
__device__ __forceinline__ float u24(unsigned long long h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

// env_reset's random starting player (deterministic_madn.py:60-62, classic_madn.py:70-72, dog.py:102-104: jax
// randint(split(PRNGKey(seed))[1], (), 0, P); threefry is not restated): seat floor(U * P) of the counter RNG of the
// reset's key (det / classic: the game's seed; DOG: game_key(seed, game, deal counter)).
constexpr unsigned long long kStartStream = 0x57A27C0DE5ull;
__device__ __forceinline__ int start_seat(unsigned long long key, int P) {
  const int s = (int)(u24(mix64(key ^ kStartStream)) * (float)P);
  return s < P ? s : P - 1;
}

// jax.random.gumbel semantics on the counter RNG: -log(-log(U[tiny, 1)))
__device__ __forceinline__ float gumbel_noise(unsigned long long seed, int gid, int turn, int a) {
  const unsigned long long h = mix64(game_key(seed, gid, turn) ^ (unsigned long long)(a + 1) * 0xD6E8FEB86659FD93ull);
  const float u = fmaxf(u24(h), kTinyF);
  return -logf(-logf(u));
}

// The 1e-7 tie-break uniform of mctx muzero_action_selection, per (sim, depth, action).
__device__ __forceinline__ float tiebreak_uniform(unsigned long long seed, int gid, int turn, int sim, int depth,
                                                  int a) {
  const unsigned long long h =
      mix64(game_key(seed, gid, turn) ^ mix64(((unsigned long long)(sim & 0xFFFF) << 16) | (unsigned)(depth & 0xFFFF)) ^
            (unsigned long long)(a + 1) * 0x9E6C63D0676A9A99ull);
  return u24(h);
}

// Gamma(alpha) by Marsaglia-Tsang (alpha < 1 boosted through alpha + 1), uniforms from stream `key`.
// Bounded loops: acceptance is > 95 % per round, 32 rounds fail with probability < 1e-40.
__device__ __forceinline__ float gamma_sample(float alpha, unsigned long long key) {
  const float a = alpha < 1.f ? alpha + 1.f : alpha;
  const float d = a - 1.f / 3.f, c = 1.f / sqrtf(9.f * d);
  float g = d;
  for (int it = 0; it < 32; ++it) {
    const float u1 = fmaxf(u24(mix64(key ^ (4ull * it + 1))), kTinyF);
    const float u2 = u24(mix64(key ^ (4ull * it + 2)));
    const float x = sqrtf(-2.f * logf(u1)) * cosf(6.2831853071795865f * u2);
    float v = 1.f + c * x;
    if (v <= 0.f) continue;
    v = v * v * v;
    const float u = fmaxf(u24(mix64(key ^ (4ull * it + 3))), kTinyF);
    if (logf(u) < 0.5f * x * x + d - d * v + d * logf(v)) {
      g = d * v;
      break;
    }
  }
  if (alpha < 1.f) g *= powf(fmaxf(u24(mix64(key ^ 0xA5A5A5A5ull)), kTinyF), 1.f / alpha);
  return g;
}

// The evaluation agents' sampling (jax.random.categorical as argmax(logits + Gumbel)): the Gumbel draw of action a
// from key = game_key(seed ^ kPolicyStream, game, turn) (det and classic agents, oracle/evaluate.py policy_gumbel)
constexpr unsigned long long kPolicyStream = 0x9011C7A6E47ull;
__device__ __forceinline__ float policy_gumbel(unsigned long long key, int a) {
  const float u = fmaxf(u24(mix64(key ^ (unsigned long long)(a + 1) * 0xD6E8FEB86659FD93ull)), kTinyF);
  return -logf(-logf(u));
}

}  // namespace muz
