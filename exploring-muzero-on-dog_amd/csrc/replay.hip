// Device replay ring: save_games_from_buffers + sample_batch of MuZero_det_MADN/vec_replay_buffer.py.
//
// The ring lives in HBM (include/muz.h muz_ring).  Saving is a device-to-device copy of each finished
// game's [0, len) slice from the self-play trajectory buffers (HBM-bound byte moves: one workgroup per
// (game, 16-step chunk), 8-byte words along the contiguous obs rows).  Sampling gathers the
// K-step windows of a training batch and computes the value targets (perspective flip, gamma^n,
// bootstrap) in double precision, the way the reference's NumPy code does, then rounds to float.
#include "common.hpp"

namespace muz {

constexpr int kRingScan = 1024;
constexpr int kCopySteps = 16;   // trajectory steps per copy workgroup

// Slot of every game: rank among games with idx > 0 (deterministic single-workgroup scan).
__global__ __launch_bounds__(kRingScan) void k_ring_slots(const int32_t* idx, int n, int position, int cap,
                                                          int32_t* slot, int32_t* count) {
  __shared__ int part[kRingScan];
  const int t = threadIdx.x;
  const int chunk = (n + kRingScan - 1) / kRingScan;
  const int lo = min(n, t * chunk), hi = min(n, lo + chunk);
  int cnt = 0;
  for (int g = lo; g < hi; ++g) cnt += idx[g] > 0;
  part[t] = cnt;
  __syncthreads();
  for (int off = 1; off < kRingScan; off <<= 1) {
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int total = part[kRingScan - 1];
  int r = part[t] - cnt;
  for (int g = lo; g < hi; ++g) {
    if (idx[g] > 0) {
      // the sequential loop overwrites a slot when more than `cap` games are saved in one call:
      // only the last `cap` of them survive
      slot[g] = (total - r > cap) ? -1 : (int)(((long long)position + r) % cap);
      ++r;
    } else {
      slot[g] = -1;
    }
  }
  if (t == 0) count[0] = total;
}

// The per-step fields of a trajectory store (self-play buffers, packed transfer rows, or the ring).
struct Rows {
  int8_t* obs;
  int32_t *act, *rew;
  float *val, *pol, *mask;
  int32_t *player, *team, *discount, *dice;
  float* dice_dist;
};
__host__ __device__ inline Rows rows_of(const muz_traj& t, const muz_traj_chance& c) {
  return Rows{t.obs, t.act, t.rew, t.val, t.pol, t.mask, t.player, t.team, t.discount, c.dice, c.dice_dist};
}
__host__ __device__ inline Rows rows_of(const muz_ring& r) {
  return Rows{r.obs, r.act, r.rew, r.val, r.pol, r.mask, r.player, r.team, r.discount, r.dice, r.dice_dist};
}

// Copy game g's steps [0, len[g]) from row src_row(g) to row dst_row(g), one workgroup per (game, chunk
// of kCopySteps steps).  Rows are laid out [row][field]; obs rows are C*56 bytes (a multiple of 8) and
// move as 8-byte words.  src_row = src_off ? src_off[g] : g*src_T; dst_row = dst_off ? dst_off[g] :
// slot[g]*dst_T (slot < 0: not copied).  dice / dice_dist move when both sides have them.
__global__ __launch_bounds__(256) void k_rows_copy(Rows src, Rows dst, const int32_t* len, const int64_t* src_off,
                                                   int src_T, const int64_t* dst_off, const int32_t* slot, int dst_T,
                                                   int C, int A, int32_t* ep_len) {
  const int g = blockIdx.y;
  const int s = slot ? slot[g] : 0;
  if (s < 0) return;
  const int L = len[g];
  const int t0 = blockIdx.x * kCopySteps;
  if (t0 >= L) return;
  const int t1 = min(L, t0 + kCopySteps);
  const size_t src_row = src_off ? (size_t)src_off[g] : (size_t)g * src_T;
  const size_t dst_row = dst_off ? (size_t)dst_off[g] : (size_t)s * dst_T;
  const size_t ob = (size_t)C * 56;
  const size_t nw = (size_t)(t1 - t0) * ob / 8;
  const AS1 uint64_t* so = reinterpret_cast<const AS1 uint64_t*>(gp(src.obs) + (src_row + t0) * ob);
  AS1 uint64_t* dob = reinterpret_cast<AS1 uint64_t*>(gpw(dst.obs) + (dst_row + t0) * ob);
  for (size_t i = threadIdx.x; i < nw; i += blockDim.x) dob[i] = so[i];
  const int np = (t1 - t0) * A;
  for (int i = threadIdx.x; i < np; i += blockDim.x) gpw(dst.pol)[(dst_row + t0) * A + i] = gp(src.pol)[(src_row + t0) * A + i];
  const bool chance = dst.dice && src.dice;
  for (int t = t0 + (int)threadIdx.x; t < t1; t += blockDim.x) {
    dst.act[dst_row + t] = src.act[src_row + t];
    dst.rew[dst_row + t] = src.rew[src_row + t];
    dst.val[dst_row + t] = src.val[src_row + t];
    dst.mask[dst_row + t] = src.mask[src_row + t];
    dst.player[dst_row + t] = src.player[src_row + t];
    dst.team[dst_row + t] = src.team[src_row + t];
    dst.discount[dst_row + t] = src.discount[src_row + t];
    if (chance) dst.dice[dst_row + t] = src.dice[src_row + t];
  }
  if (chance)
    for (int i = threadIdx.x; i < (t1 - t0) * 6; i += blockDim.x)
      dst.dice_dist[(dst_row + t0) * 6 + i] = src.dice_dist[(src_row + t0) * 6 + i];
  if (ep_len && blockIdx.x == 0 && threadIdx.x == 0) ep_len[s] = L;
}

// Exclusive scan of the game lengths (int64 row offsets of the packed layout) + total rows.
__global__ __launch_bounds__(kRingScan) void k_len_scan(const int32_t* len, int n, int64_t* off, int64_t* total) {
  __shared__ long long part[kRingScan];
  const int t = threadIdx.x;
  const int chunk = (n + kRingScan - 1) / kRingScan;
  const int lo = min(n, t * chunk), hi = min(n, lo + chunk);
  long long cnt = 0;
  for (int g = lo; g < hi; ++g) cnt += max(len[g], 0);
  part[t] = cnt;
  __syncthreads();
  for (int o = 1; o < kRingScan; o <<= 1) {
    const long long v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  long long r = part[t] - cnt;
  for (int g = lo; g < hi; ++g) {
    off[g] = r;
    r += max(len[g], 0);
  }
  if (t == kRingScan - 1) total[0] = part[t];
}

// sample_batch for one batch element per workgroup (vec_replay_buffer.py:101-264).
__global__ __launch_bounds__(256) void k_ring_sample(muz_ring ring, const int32_t* ep_idx, const int32_t* t_start,
                                                     int K, int TD, int boot_flag, const double* gpow, muz_sample o) {
  const int b = blockIdx.x;
  const int T = ring.max_steps, A = ring.num_actions, C = ring.obs_channels;
  // indices come from the host; clamp so a bad one reads a wrong slot instead of faulting
  const int e = min(max(ep_idx[b], 0), ring.capacity - 1);
  const int L = min(max(ring.ep_len[e], 1), T);
  const int t0 = min(max(t_start[b], 0), L - 1);
  const size_t row = (size_t)e * T;
  // root observation (int8 -> float)
  const int8_t* so = ring.obs + (row + t0) * (size_t)C * 56;
  for (int i = threadIdx.x; i < C * 56; i += blockDim.x) o.observations[(size_t)b * C * 56 + i] = (float)so[i];
  const int fin = L - 1;
  const int f_rew = ring.rew[row + fin], f_pl = ring.player[row + fin], f_tm = ring.team[row + fin];
  // policies [K][A]
  for (int i = threadIdx.x; i < K * A; i += blockDim.x) {
    const int k = i / A, a = i % A;
    const int sq = t0 + k;
    const int sc = min(sq, L - 1);
    o.policies[((size_t)b * K + k) * A + a] = sq < L ? ring.pol[(row + sc) * A + a] : 0.f;
  }
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const int sq = t0 + k;
    const bool valid = sq < L;
    const int sc = min(sq, L - 1);
    const int pl = ring.player[row + sc], tm = ring.team[row + sc];
    o.values[(size_t)b * K + k] = valid ? ring.val[row + sc] : 0.f;
    o.masks[(size_t)b * K + k] = valid ? ring.mask[row + sc] : 0.f;
    if (k < K - 1) {
      o.actions[(size_t)b * (K - 1) + k] = valid ? ring.act[row + sc] : 0;
      o.rewards[(size_t)b * (K - 1) + k] = valid ? ring.rew[row + sc] : 1;
      o.discount_targets[(size_t)b * (K - 1) + k] = valid ? ring.discount[row + sc] : 1;
      if (o.dice_outcomes && ring.dice)   // dice index 0..5; padding 0 (vec_replay_buffer_stochastic.py:266, 280)
        o.dice_outcomes[(size_t)b * (K - 1) + k] = valid ? max(ring.dice[row + sc] - 1, 0) : 0;
      if (o.dice_probs && ring.dice_dist)
        for (int i = 0; i < 6; ++i)
          o.dice_probs[((size_t)b * (K - 1) + k) * 6 + i] = valid ? ring.dice_dist[(row + sc) * 6 + i] : 1.0f / 6.0f;
    }
    // value target (7.3 - 7.7)
    double z = 0.0;
    if (ring.won_if_positive ? f_rew > 0 : f_rew == 2) z = (tm == -1) ? (f_pl == pl ? 1.0 : -1.0) : (f_tm == tm ? 1.0 : -1.0);
    const int steps = L - 1 - sq;
    const bool boot_from_value = steps >= TD;
    const int bi = min(sq + TD, L - 1);
    const float braw = ring.val[row + bi];
    const bool same = (tm != -1) ? (tm == ring.team[row + bi]) : (pl == ring.player[row + bi]);
    const double boot = same ? (double)braw : -(double)braw;
    z = z * gpow[max(steps, 0)];
    const int be = min(TD, steps);
    const double tv = (z == 0.0 || (boot_from_value && boot_flag)) ? boot * gpow[max(be, 0)] : z;
    const double cl = tv < -1.0 ? -1.0 : (tv > 1.0 ? 1.0 : tv);
    o.target_values[(size_t)b * K + k] = valid ? (float)cl : 0.f;
  }
}

}  // namespace muz

using namespace muz;

extern "C" {

int muz_ring_save(muz_ring ring, muz_traj traj, const muz_traj_chance* chance, int32_t n, int32_t position,
                  int32_t* slot_out, int32_t* count_out, void* stream) {
  MUZ_HOST_CHECK(n >= 0 && slot_out && count_out && traj.idx && traj.obs && ring.obs && ring.ep_len);
  MUZ_HOST_CHECK((ring.dice == nullptr) == (ring.dice_dist == nullptr));
  MUZ_HOST_CHECK(!ring.dice || (chance && chance->dice && chance->dice_dist));
  const muz_traj_chance ch = chance ? *chance : muz_traj_chance{nullptr, nullptr};
  MUZ_HOST_CHECK(ring.capacity > 0 && position >= 0 && position < ring.capacity);
  MUZ_HOST_CHECK(traj.max_steps > 0 && traj.max_steps <= ring.max_steps);
  MUZ_HOST_CHECK(ring.obs_channels > 0 && ring.num_actions > 0);
  hipStream_t s = (hipStream_t)stream;
  k_ring_slots<<<1, kRingScan, 0, s>>>(traj.idx, n, position, ring.capacity, slot_out, count_out);
  int rc = muz_last_launch_error();
  if (rc || n == 0) return rc;
  dim3 grid((traj.max_steps + kCopySteps - 1) / kCopySteps, n);
  k_rows_copy<<<grid, 256, 0, s>>>(rows_of(traj, ch), rows_of(ring), traj.idx, nullptr, traj.max_steps, nullptr,
                                   slot_out, ring.max_steps, ring.obs_channels, ring.num_actions, ring.ep_len);
  return muz_last_launch_error();
}

int muz_traj_offsets(const int32_t* len, int32_t n, int64_t* row_offset, int64_t* total_rows, void* stream) {
  MUZ_HOST_CHECK(n >= 0 && len && row_offset && total_rows);
  k_len_scan<<<1, kRingScan, 0, (hipStream_t)stream>>>(len, n, row_offset, total_rows);
  return muz_last_launch_error();
}

int muz_traj_pack(muz_traj traj, const muz_traj_chance* chance, const int64_t* row_offset, int32_t n,
                  int32_t obs_channels, int32_t num_actions, muz_traj packed, const muz_traj_chance* packed_chance,
                  void* stream) {
  MUZ_HOST_CHECK(n >= 0 && traj.idx && traj.obs && packed.obs && row_offset && traj.max_steps > 0);
  MUZ_HOST_CHECK(obs_channels > 0 && num_actions > 0);
  MUZ_HOST_CHECK((chance == nullptr) == (packed_chance == nullptr));
  const muz_traj_chance ch = chance ? *chance : muz_traj_chance{nullptr, nullptr};
  const muz_traj_chance pch = packed_chance ? *packed_chance : muz_traj_chance{nullptr, nullptr};
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return MUZ_OK;
  if (packed.idx && packed.idx != traj.idx)
    MUZ_HIP_RET(hipMemcpyAsync(packed.idx, traj.idx, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
  dim3 grid((traj.max_steps + kCopySteps - 1) / kCopySteps, n);
  k_rows_copy<<<grid, 256, 0, s>>>(rows_of(traj, ch), rows_of(packed, pch), traj.idx, nullptr, traj.max_steps,
                                   row_offset, nullptr, 0, obs_channels, num_actions, nullptr);
  return muz_last_launch_error();
}

int muz_ring_save_packed(muz_ring ring, muz_traj packed, const muz_traj_chance* chance, const int64_t* row_offset,
                         int32_t n, int32_t max_len, int32_t position, int32_t* slot_out, int32_t* count_out,
                         void* stream) {
  MUZ_HOST_CHECK(n >= 0 && slot_out && count_out && packed.idx && packed.obs && row_offset && ring.obs && ring.ep_len);
  MUZ_HOST_CHECK((ring.dice == nullptr) == (ring.dice_dist == nullptr));
  MUZ_HOST_CHECK(!ring.dice || (chance && chance->dice && chance->dice_dist));
  MUZ_HOST_CHECK(ring.capacity > 0 && position >= 0 && position < ring.capacity);
  MUZ_HOST_CHECK(max_len >= 0 && max_len <= ring.max_steps);
  const muz_traj_chance ch = chance ? *chance : muz_traj_chance{nullptr, nullptr};
  hipStream_t s = (hipStream_t)stream;
  k_ring_slots<<<1, kRingScan, 0, s>>>(packed.idx, n, position, ring.capacity, slot_out, count_out);
  int rc = muz_last_launch_error();
  if (rc || n == 0 || max_len == 0) return rc;
  dim3 grid((max_len + kCopySteps - 1) / kCopySteps, n);
  k_rows_copy<<<grid, 256, 0, s>>>(rows_of(packed, ch), rows_of(ring), packed.idx, row_offset, 0, nullptr, slot_out,
                                   ring.max_steps, ring.obs_channels, ring.num_actions, ring.ep_len);
  return muz_last_launch_error();
}

int muz_ring_sample(muz_ring ring, const int32_t* ep_idx, const int32_t* t_start, int32_t batch, int32_t unroll_steps,
                    int32_t td_steps, int32_t bootstrap_value_target, const double* gamma_pow, muz_sample out,
                    void* stream) {
  MUZ_HOST_CHECK(batch >= 0 && ep_idx && t_start && gamma_pow && unroll_steps >= 1 && td_steps >= 0);
  MUZ_HOST_CHECK(td_steps <= ring.max_steps && ring.capacity > 0 && ring.obs && ring.ep_len);
  MUZ_HOST_CHECK(out.observations && out.actions && out.rewards && out.policies && out.values && out.masks &&
                 out.target_values && out.discount_targets);
  if (batch == 0) return MUZ_OK;
  k_ring_sample<<<batch, 256, 0, (hipStream_t)stream>>>(ring, ep_idx, t_start, unroll_steps + 1, td_steps,
                                                        bootstrap_value_target, gamma_pow, out);
  return muz_last_launch_error();
}

}  // extern "C"
