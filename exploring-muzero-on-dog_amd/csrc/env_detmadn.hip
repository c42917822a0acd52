// Batched deterministic-MADN environment kernels + their C ABI (include/muz.h).
// One board per lane; 256-lane workgroups; the lane's board is staged in LDS.
#include "detmadn.hpp"
#include "host_consts.hpp"

namespace muz {

constexpr int kEnvBlock = 256;

__global__ __launch_bounds__(kEnvBlock) void k_det_reset(DetConsts c, muz_detmadn_soa st, int n) {
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const bool fp = has(c.flags, R_FREE_PIN);
  for (int cell = 0; cell < kCells; ++cell) st.board[cell * S + g] = -1;
  for (int p = 0; p < c.P; ++p) {
    for (int k = 0; k < 4; ++k) st.pins[(p * 4 + k) * S + g] = (int8_t)((fp && k == 0) ? c.start[p] : -1);
    for (int m = 0; m < 6; ++m) st.action_set[(p * 6 + m) * S + g] = 4;
    if (fp) st.board[c.start[p] * S + g] = (int8_t)p;
  }
  st.current_player[g] = (int8_t)c.starting_player;
  st.reward[g] = 0;
  st.done[g] = 0;
}

__global__ __launch_bounds__(kEnvBlock) void k_det_legal(DetConsts c, muz_detmadn_soa st, uint32_t* legal, int n) {
  __shared__ int8_t sboard[kCells * kEnvBlock];
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  BoardView b{sboard + threadIdx.x, kEnvBlock};
  DetLane s;
  det_load(c, st, g, s, b);
  legal[g] = det_legal(c, s, b);
}

// mode 0: action index (map_action), mode 1: explicit (pin, move)
__global__ __launch_bounds__(kEnvBlock) void k_det_step(DetConsts c, muz_detmadn_soa st, const int32_t* a0,
                                                        const int32_t* a1, int mode, int8_t* reward, uint8_t* done,
                                                        uint32_t* next_legal, int n) {
  __shared__ int8_t sboard[kCells * kEnvBlock];
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  BoardView b{sboard + threadIdx.x, kEnvBlock};
  DetLane s;
  det_load(c, st, g, s, b);
  int pin, move;
  if (mode == 0) {
    const int a = a0[g];
    pin = fdiv(a, 6);
    move = fmodp(a, 6) + 1;
  } else {
    pin = a0[g];
    move = a1[g];
  }
  const int r = det_step(c, s, b, pin, move);
  det_store(c, st, g, s, b, true);
  if (reward) reward[g] = (int8_t)r;
  if (done) done[g] = (uint8_t)s.done;
  if (next_legal) next_legal[g] = det_legal(c, s, b);
}

__global__ __launch_bounds__(kEnvBlock) void k_det_nostep(DetConsts c, muz_detmadn_soa st, int8_t* reward,
                                                          uint8_t* done, int n) {
  const int g = blockIdx.x * kEnvBlock + threadIdx.x;
  if (g >= n) return;
  const int S = st.stride;
  const int cp = st.current_player[g];
  for (int m = 0; m < 6; ++m) st.action_set[(cp * 6 + m) * S + g] = 4;
  st.current_player[g] = (int8_t)((cp + 1) % c.P);
  if (reward) reward[g] = 0;
  if (done) done[g] = st.done[g];
}

// One thread per (game, cell): coalesced obs writes along the cell axis.
template <typename T>
__global__ __launch_bounds__(64) void k_det_encode(DetConsts c, muz_detmadn_soa st, T* obs, int n) {
  const int g = blockIdx.x;
  const int w = threadIdx.x;
  if (g >= n || w >= kCells) return;
  const int S = st.stride;
  DetLane s;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = st.pins[min(j, c.P * 4 - 1) * S + g];
    s.pins[j] = (j < c.P * 4) ? v : -1;
  }
#pragma unroll
  for (int j = 0; j < 24; ++j) {
    const int v = st.action_set[min(j, c.P * 6 - 1) * S + g];
    s.aset[j] = (j < c.P * 6) ? v : 0;
  }
  s.cp = st.current_player[g];
  const int C = 8 * c.P + 2;
  T* out = obs + (size_t)g * C * kCells;
  auto owner = [&](int cell) { return (int)st.board[cell * S + g]; };
  for (int ch = 0; ch < C; ++ch) out[ch * kCells + w] = (T)det_encode_value(c, s, ch, w, owner);
}

}  // namespace muz

using namespace muz;

static inline unsigned nblocks(int n, int b) { return (unsigned)((n + b - 1) / b); }

extern "C" {

int muz_detmadn_reset(const muz_rules* rules, muz_detmadn_soa st, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n);
  if (n == 0) return MUZ_OK;
  k_det_reset<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, n);
  return muz_last_launch_error();
}

int muz_detmadn_legal(const muz_rules* rules, muz_detmadn_soa st, uint32_t* legal, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && legal);
  if (n == 0) return MUZ_OK;
  k_det_legal<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, legal, n);
  return muz_last_launch_error();
}

int muz_detmadn_step(const muz_rules* rules, muz_detmadn_soa st, const int32_t* action, int8_t* reward,
                     uint8_t* done, uint32_t* next_legal, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && action);
  if (n == 0) return MUZ_OK;
  k_det_step<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, action, nullptr, 0, reward, done,
                                                                            next_legal, n);
  return muz_last_launch_error();
}

int muz_detmadn_step_pin_move(const muz_rules* rules, muz_detmadn_soa st, const int32_t* pin, const int32_t* move,
                              int8_t* reward, uint8_t* done, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && pin && move);
  if (n == 0) return MUZ_OK;
  k_det_step<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, pin, move, 1, reward, done,
                                                                            nullptr, n);
  return muz_last_launch_error();
}

int muz_detmadn_nostep(const muz_rules* rules, muz_detmadn_soa st, int8_t* reward, uint8_t* done, int32_t n,
                       void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n);
  if (n == 0) return MUZ_OK;
  k_det_nostep<<<nblocks(n, kEnvBlock), kEnvBlock, 0, (hipStream_t)stream>>>(c, st, reward, done, n);
  return muz_last_launch_error();
}

int muz_detmadn_encode_f32(const muz_rules* rules, muz_detmadn_soa st, float* obs, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && obs);
  if (n == 0) return MUZ_OK;
  k_det_encode<float><<<n, 64, 0, (hipStream_t)stream>>>(c, st, obs, n);
  return muz_last_launch_error();
}

int muz_detmadn_encode_i8(const muz_rules* rules, muz_detmadn_soa st, int8_t* obs, int32_t n, void* stream) {
  DetConsts c;
  int rc = make_det_consts(rules, &c);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && st.stride >= n && obs);
  if (n == 0) return MUZ_OK;
  k_det_encode<int8_t><<<n, 64, 0, (hipStream_t)stream>>>(c, st, obs, n);
  return muz_last_launch_error();
}

}  // extern "C"
