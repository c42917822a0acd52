// Shared pieces of the C++ CPU restatements (oracle/cpu_selfplay.cpp: det MuZero self-play,
// oracle/cpu_classic.cpp: classic Stochastic MuZero self-play, oracle/cpu_dog.cpp: DOG random play).
// TEST INFRASTRUCTURE / CPU BASELINE ONLY (see cpu_selfplay.cpp).  Everything is in an anonymous namespace:
// each translation unit gets its own copy.
#pragma once
#pragma GCC diagnostic ignored "-Wunused-function"   // not every TU uses every shared piece
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include <immintrin.h>
#include <omp.h>

namespace {

constexpr int kCells = 56;
constexpr int kA = 24;
constexpr int kLat = 256;
constexpr float kTiny = std::numeric_limits<float>::min();
constexpr float kFMin = -std::numeric_limits<float>::max();
constexpr float kInf = std::numeric_limits<float>::infinity();

enum : uint32_t {
  R_TEAMS = 1, R_FREE_PIN = 2, R_CIRCULAR = 4, R_START_BLOCK = 8, R_JUMP_GOAL = 16, R_FRIENDLY = 32,
  R_START_ON_1 = 64, R_BONUS_6 = 128, R_MUST_TRAVERSE = 256, R_DICE_RETHROW = 512
};

inline long long pymod(long long a, long long n) { long long r = a % n; return r < 0 ? r + n : r; }
inline long long floordiv(long long a, long long n) { long long q = a / n; return (a % n != 0 && ((a < 0) != (n < 0))) ? q - 1 : q; }
// jax gather: normalise a negative index once, then clamp into [0, n)
inline long long gidx(long long i, long long n) { if (i < 0) i += n; return i < 0 ? 0 : (i >= n ? n - 1 : i); }

// ------------------------------------------------------------------------------------------- networks
struct Net {
  std::map<std::string, std::vector<float>> p;
  int C = 0, A = 24;   // observation channels, policy width (det 24, classic 4)
  const float* w(const std::string& k) const {
    auto it = p.find(k);
    if (it == p.end()) return nullptr;
    return it->second.data();
  }
  size_t n(const std::string& k) const { return p.at(k).size(); }
};

// out[R rows][N] = in[R][K] @ W[K][N] + b with the accumulators in AVX2 registers: 4 rows x 16 columns per
// block, k innermost (each output is the k-ordered fma chain starting from its bias).
template <int R>
void dense_rows(const float* in, int K, int N, const float* W, const float* b, float* out) {
  int j = 0;
  for (; j + 16 <= N; j += 16) {
    __m256 acc[R][2];
    for (int r = 0; r < R; ++r) {
      acc[r][0] = _mm256_loadu_ps(b + j);
      acc[r][1] = _mm256_loadu_ps(b + j + 8);
    }
    for (int k = 0; k < K; ++k) {
      const __m256 w0 = _mm256_loadu_ps(W + (size_t)k * N + j), w1 = _mm256_loadu_ps(W + (size_t)k * N + j + 8);
      for (int r = 0; r < R; ++r) {
        const __m256 a = _mm256_broadcast_ss(in + (size_t)r * K + k);
        acc[r][0] = _mm256_fmadd_ps(a, w0, acc[r][0]);
        acc[r][1] = _mm256_fmadd_ps(a, w1, acc[r][1]);
      }
    }
    for (int r = 0; r < R; ++r) {
      _mm256_storeu_ps(out + (size_t)r * N + j, acc[r][0]);
      _mm256_storeu_ps(out + (size_t)r * N + j + 8, acc[r][1]);
    }
  }
  for (; j + 8 <= N; j += 8) {
    __m256 acc[R];
    for (int r = 0; r < R; ++r) acc[r] = _mm256_loadu_ps(b + j);
    for (int k = 0; k < K; ++k) {
      const __m256 w0 = _mm256_loadu_ps(W + (size_t)k * N + j);
      for (int r = 0; r < R; ++r) acc[r] = _mm256_fmadd_ps(_mm256_broadcast_ss(in + (size_t)r * K + k), w0, acc[r]);
    }
    for (int r = 0; r < R; ++r) _mm256_storeu_ps(out + (size_t)r * N + j, acc[r]);
  }
  for (; j < N; ++j)
    for (int r = 0; r < R; ++r) {
      float a = b[j];
      for (int k = 0; k < K; ++k) a = std::fma(in[(size_t)r * K + k], W[(size_t)k * N + j], a);
      out[(size_t)r * N + j] = a;
    }
}

void dense_raw(const float* W, const float* b, const float* in, int B, int K, int N, float* out) {
  int r = 0;
  for (; r + 8 <= B; r += 8) dense_rows<8>(in + (size_t)r * K, K, N, W, b, out + (size_t)r * N);
  for (; r + 4 <= B; r += 4) dense_rows<4>(in + (size_t)r * K, K, N, W, b, out + (size_t)r * N);
  for (; r < B; ++r) dense_rows<1>(in + (size_t)r * K, K, N, W, b, out + (size_t)r * N);
}

void dense(const Net& net, const std::string& name, const float* in, int B, int K, int N, float* out) {
  dense_raw(net.w(name + "/kernel"), net.w(name + "/bias"), in, B, K, N, out);
}

void layer_norm(const Net& net, const std::string& name, float* x, int B, int N, bool relu) {
  const float* sc = net.w(name + "/scale");
  const float* sh = net.w(name + "/bias");
  for (int r = 0; r < B; ++r) {
    float* v = x + (size_t)r * N;
    float s = 0.f, s2 = 0.f;
    for (int j = 0; j < N; ++j) {
      s += v[j];
      s2 += v[j] * v[j];
    }
    const float mean = s / (float)N, mean2 = s2 / (float)N;
    const float var = std::max(0.f, mean2 - mean * mean);
    const float inv = 1.0f / std::sqrt(var + 1e-6f);
    for (int j = 0; j < N; ++j) {
      const float y = (v[j] - mean) * (inv * sc[j]) + sh[j];
      v[j] = relu ? std::max(y, 0.f) : y;
    }
  }
}

void relu_(float* x, size_t n) { for (size_t i = 0; i < n; ++i) x[i] = std::max(x[i], 0.f); }

void minmax(float* x, int B, int N) {
  for (int r = 0; r < B; ++r) {
    float* v = x + (size_t)r * N;
    float lo = kInf, hi = -kInf;
    for (int j = 0; j < N; ++j) {
      lo = std::min(lo, v[j]);
      hi = std::max(hi, v[j]);
    }
    const float den = hi - lo + 1e-8f;
    for (int j = 0; j < N; ++j) v[j] = (v[j] - lo) / den;
  }
}

// ResBlock (12-24) in place on x [B][256]
void resblock(const Net& net, const std::string& pre, float* x, int B, std::vector<float>& t1, std::vector<float>& t2) {
  t1.resize((size_t)B * kLat);
  t2.resize((size_t)B * kLat);
  dense(net, pre + "/Dense_0", x, B, kLat, kLat, t1.data());
  layer_norm(net, pre + "/LayerNorm_0", t1.data(), B, kLat, true);
  dense(net, pre + "/Dense_1", t1.data(), B, kLat, kLat, t2.data());
  layer_norm(net, pre + "/LayerNorm_1", t2.data(), B, kLat, false);
  for (size_t i = 0; i < (size_t)B * kLat; ++i) x[i] = std::max(x[i] + t2[i], 0.f);
}

struct Scratch {
  std::vector<float> a, b, c, d, t1, t2;
};

// Conv 1-D 'SAME' (Flax), as im2col + dense: in [B][56][Cin] -> out [B][56][Cout]
void conv1d(const Net& net, const std::string& name, const float* in, int B, int Cin, int Cout, int K, float* out) {
  const int pl = (K - 1) / 2;
  std::vector<float> cols((size_t)B * kCells * K * Cin, 0.f);
  for (int r = 0; r < B; ++r)
    for (int w = 0; w < kCells; ++w)
      for (int d = 0; d < K; ++d) {
        const int src = w + d - pl;
        if (src < 0 || src >= kCells) continue;
        std::memcpy(&cols[(((size_t)r * kCells + w) * K + d) * Cin], in + ((size_t)r * kCells + src) * Cin,
                    sizeof(float) * Cin);
      }
  dense(net, name, cols.data(), B * kCells, K * Cin, Cout, out);   // kernel [K][Cin][Cout] = [K*Cin][Cout]
}

// RepresentationNetwork2 (75-141): obs [B][C][56] -> latent [B][256]; with representation/LayerNorm_7 the DOG
// RepresentationNetwork (MuZero_DOG/muzero_dog.py:25-83: LayerNorm instead of min-max after Dense_4)
void representation(const Net& net, const float* obs, int B, float* lat, Scratch& s) {
  const int C = net.C;
  const std::string r = "representation/";
  s.a.assign((size_t)B * kCells * 6, 0.f);
  for (int b = 0; b < B; ++b)
    for (int w = 0; w < kCells; ++w)
      for (int c = 0; c < 6; ++c) s.a[((size_t)b * kCells + w) * 6 + c] = obs[((size_t)b * C + c) * kCells + w];
  s.b.resize((size_t)B * kCells * 64);
  s.c.resize((size_t)B * kCells * 64);
  conv1d(net, r + "Conv_0", s.a.data(), B, 6, 32, 3, s.b.data());
  layer_norm(net, r + "LayerNorm_0", s.b.data(), B * kCells, 32, true);
  conv1d(net, r + "Conv_1", s.b.data(), B, 32, 64, 3, s.c.data());
  layer_norm(net, r + "LayerNorm_1", s.c.data(), B * kCells, 64, true);
  conv1d(net, r + "Conv_2", s.c.data(), B, 64, 64, 5, s.b.data());
  layer_norm(net, r + "LayerNorm_2", s.b.data(), B * kCells, 64, true);
  std::vector<float> cat((size_t)B * 320);
  std::vector<float> flat((size_t)B * kLat);
  dense(net, r + "Dense_0", s.b.data(), B, kCells * 64, kLat, flat.data());
  layer_norm(net, r + "LayerNorm_3", flat.data(), B, kLat, true);
  std::vector<float> g((size_t)B * (C - 6)), g1((size_t)B * 64), g2((size_t)B * 64);
  for (int b = 0; b < B; ++b)
    for (int c = 6; c < C; ++c) g[(size_t)b * (C - 6) + c - 6] = obs[((size_t)b * C + c) * kCells];
  dense(net, r + "Dense_1", g.data(), B, C - 6, 64, g1.data());
  layer_norm(net, r + "LayerNorm_4", g1.data(), B, 64, true);
  dense(net, r + "Dense_2", g1.data(), B, 64, 64, g2.data());
  layer_norm(net, r + "LayerNorm_5", g2.data(), B, 64, true);
  for (int b = 0; b < B; ++b) {
    std::memcpy(&cat[(size_t)b * 320], &flat[(size_t)b * kLat], sizeof(float) * kLat);
    std::memcpy(&cat[(size_t)b * 320 + kLat], &g2[(size_t)b * 64], sizeof(float) * 64);
  }
  std::vector<float> h((size_t)B * kLat);
  dense(net, r + "Dense_3", cat.data(), B, 320, kLat, h.data());
  layer_norm(net, r + "LayerNorm_6", h.data(), B, kLat, true);
  for (int i = 0; i < 6; ++i) resblock(net, r + "ResBlock_" + std::to_string(i), h.data(), B, s.t1, s.t2);
  dense(net, r + "Dense_4", h.data(), B, kLat, kLat, lat);
  if (net.w(r + "LayerNorm_7/scale")) layer_norm(net, r + "LayerNorm_7", lat, B, kLat, false);   // DOG head (80-81)
  else minmax(lat, B, kLat);
}

// PredictionNetwork4 (549-583): latent [B][256] -> logits [B][A], value [B]
void prediction(const Net& net, const float* lat, int B, float* logits, float* value, Scratch& s) {
  const std::string p = "prediction/";
  std::vector<float> x(lat, lat + (size_t)B * kLat);
  layer_norm(net, p + "LayerNorm_0", x.data(), B, kLat, false);
  for (int i = 0; i < 2; ++i) resblock(net, p + "ResBlock_" + std::to_string(i), x.data(), B, s.t1, s.t2);
  std::vector<float> h0((size_t)B * kLat), h1((size_t)B * 128), v0((size_t)B * 128), v1((size_t)B * 64);
  dense(net, p + "Dense_0", x.data(), B, kLat, kLat, h0.data());
  layer_norm(net, p + "LayerNorm_1", h0.data(), B, kLat, true);
  dense(net, p + "Dense_1", h0.data(), B, kLat, 128, h1.data());
  layer_norm(net, p + "LayerNorm_2", h1.data(), B, 128, true);
  dense(net, p + "Dense_2", h1.data(), B, 128, net.A, logits);
  dense(net, p + "Dense_3", x.data(), B, kLat, 128, v0.data());
  layer_norm(net, p + "LayerNorm_3", v0.data(), B, 128, true);
  dense(net, p + "Dense_4", v0.data(), B, 128, 64, v1.data());
  relu_(v1.data(), v1.size());
  std::vector<float> v2(B);
  dense(net, p + "Dense_5", v1.data(), B, 64, 1, v2.data());
  for (int b = 0; b < B; ++b) value[b] = std::tanh(v2[b]);
}

float support3(const float* l) {   // sum(softmax(l) * [-1, 0, 1])
  const float m = std::max(std::max(l[0], l[1]), l[2]);
  const float e0 = std::exp(l[0] - m), e1 = std::exp(l[1] - m), e2 = std::exp(l[2] - m);
  const float z = e0 + e1 + e2;
  return (e0 / z) * -1.0f + (e1 / z) * 0.0f + (e2 / z) * 1.0f;
}

void softmax(const float* x, float* out, int n) {
  float m = -kInf;
  for (int i = 0; i < n; ++i) m = std::max(m, x[i]);
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += (out[i] = std::exp(x[i] - m));
  for (int i = 0; i < n; ++i) out[i] /= s;
}

int argmax(const float* x, int n) {
  int bi = 0;
  for (int i = 1; i < n; ++i)
    if (x[i] > x[bi]) bi = i;
  return bi;
}

// counter-based hash of the engine (csrc/rng.hpp)
inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

}  // namespace
