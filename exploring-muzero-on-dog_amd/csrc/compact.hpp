// Deterministic single-workgroup compaction of the games that search this turn, shared by the
// self-play drivers (internal linkage: each translation unit launches its own copy).
#pragma once
#include "common.hpp"

namespace muz {

// One workgroup: exclusive scan of "searches this turn" -> list (slot -> game) and slot (game -> slot).
constexpr int kScanThreads = 1024;
static __global__ __launch_bounds__(kScanThreads) void k_sp_compact(const int32_t* flag, int n, int32_t* list, int32_t* slot,
                                                             int32_t* counts) {
  __shared__ int part[kScanThreads];
  __shared__ int act[kScanThreads];
  const int t = threadIdx.x;
  const int chunk = (n + kScanThreads - 1) / kScanThreads;
  const int lo = min(n, t * chunk), hi = min(n, lo + chunk);
  int cnt = 0, a = 0;
  for (int g = lo; g < hi; ++g) {
    const int f = flag[g];
    cnt += f == 1;
    a += f != 0;
  }
  part[t] = cnt;
  act[t] = a;
  __syncthreads();
  for (int off = 1; off < kScanThreads; off <<= 1) {
    const int v = t >= off ? part[t - off] : 0;
    const int w = t >= off ? act[t - off] : 0;
    __syncthreads();
    part[t] += v;
    act[t] += w;
    __syncthreads();
  }
  int pos = part[t] - cnt;   // exclusive prefix
  for (int g = lo; g < hi; ++g) {
    if (flag[g] == 1) {
      list[pos] = g;
      slot[g] = pos;
      ++pos;
    } else {
      slot[g] = -1;
    }
  }
  if (t == kScanThreads - 1) {
    counts[0] = part[t];
    counts[1] = act[t];
  }
}

}  // namespace muz
