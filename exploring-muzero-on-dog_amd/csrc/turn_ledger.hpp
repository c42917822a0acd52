// Host-side bookkeeping of the native self-play turn loops (selfplay.hip, selfplay_classic.hip).
//
// Each turn copies its counts (games searching, games active at the start) into a small pinned ring and
// records an event; the host reads a turn's counts kLag turns late, so the GPU queue never drains.  The
// search launch of every turn is bracketed by a ring of timing events, read one turn later still (a turn's
// search has completed once the NEXT turn's count event has).  Nothing is allocated per turn.  Turns are
// retired in order and the first turn whose start found no active game ends the count (the reference's
// while loop stops there); the at most kLag turns launched after it record nothing.
#pragma once
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace muz {

class TurnLedger {
 public:
  static constexpr int kLag = 2, kRing = 4;
  static_assert(kRing >= kLag + 2, "event ring too small");

  TurnLedger(hipStream_t s, bool timing) : s_(s), timing_(timing) {}
  ~TurnLedger() {
    for (int i = 0; i < kRing; ++i) {
      if (ev_[i]) (void)hipEventDestroy(ev_[i]);
      if (tev_[i][0]) (void)hipEventDestroy(tev_[i][0]);
      if (tev_[i][1]) (void)hipEventDestroy(tev_[i][1]);
    }
    if (t0_) (void)hipEventDestroy(t0_);
    if (t1_) (void)hipEventDestroy(t1_);
    if (host_) (void)hipHostFree(host_);
  }
  int begin() {
    hipError_t e = hipHostMalloc((void**)&host_, (size_t)kRing * 2 * sizeof(int32_t), hipHostMallocMapped);
    if (e != hipSuccess) return (int)e;
    if (hipHostGetDevicePointer((void**)&dev_, host_, 0) != hipSuccess) dev_ = nullptr;
    // every create is checked; on a failure the events made so far (and the pinned ring) are released by the
    // destructor, which only touches handles that were created (nullptr-initialised members)
    for (int i = 0; i < kRing; ++i) {
      if ((e = hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming)) != hipSuccess) return (int)e;
      if (timing_) {
        if ((e = hipEventCreate(&tev_[i][0])) != hipSuccess) return (int)e;
        if ((e = hipEventCreate(&tev_[i][1])) != hipSuccess) return (int)e;
      }
    }
    if ((e = hipEventCreate(&t0_)) != hipSuccess) return (int)e;
    if ((e = hipEventCreate(&t1_)) != hipSuccess) return (int)e;
    if ((e = hipEventRecord(t0_, s_)) != hipSuccess) return (int)e;
    ok_ = true;
    return MUZ_OK;
  }
  // top of turn `turn`: false when the loop must stop (a retired turn found no active game)
  bool proceed(int turn) {
    if (turn < kLag) return true;
    const int u = turn - kLag;
    (void)hipEventSynchronize(ev_[u % kRing]);
    if (u >= 1) time_turn(u - 1);
    retire(u);
    return !stopped_;
  }
  // the device-visible address of `turn`'s pinned counts slot, for a kernel that writes the counts there itself
  // (then counts_written instead of counts); null when the ring has no device mapping
  int32_t* device_slot(int turn) const { return dev_ ? dev_ + 2 * (turn % kRing) : nullptr; }
  void counts_written(int turn) { (void)hipEventRecord(ev_[turn % kRing], s_); }
  // after the counts of `turn` are final on the device (2 int32: searching, active)
  void counts(int turn, const int32_t* dev_counts) {
    (void)hipMemcpyAsync(host_ + 2 * (turn % kRing), dev_counts, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s_);
    (void)hipEventRecord(ev_[turn % kRing], s_);
  }
  void search_begin(int turn) {
    if (timing_) (void)hipEventRecord(tev_[turn % kRing][0], s_);
  }
  void search_end(int turn) {
    if (timing_) (void)hipEventRecord(tev_[turn % kRing][1], s_);
  }
  // after the loop: `turns` = turns launched
  void finish(int turns, muz_sp_stats* stats) {
    (void)hipEventRecord(t1_, s_);
    (void)hipStreamSynchronize(s_);
    for (int u = retired_; u < turns && !stopped_; ++u) retire(u);
    for (int u = timed_; u < turns; ++u) time_turn(u);
    if (stats) {
      float tot = 0.f;
      (void)hipEventElapsedTime(&tot, t0_, t1_);
      stats->turns = active_;
      stats->searches = searches_;
      stats->search_ms = search_ms_;
      stats->total_ms = tot;
    }
  }

 private:
  void retire(int u) {
    const int32_t* hc = host_ + 2 * (u % kRing);
    if (!stopped_ && hc[1] == 0) stopped_ = true;
    if (!stopped_) {
      ++active_;
      searches_ += hc[0];
    }
    retired_ = u + 1;
  }
  void time_turn(int u) {
    if (timing_ && u < active_) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, tev_[u % kRing][0], tev_[u % kRing][1]);
      search_ms_ += ms;
    }
    timed_ = u + 1;
  }

  hipStream_t s_;
  bool timing_, ok_ = false, stopped_ = false;
  int32_t* host_ = nullptr;
  int32_t* dev_ = nullptr;   // host_ as the device sees it (mapped pinned memory)
  hipEvent_t ev_[kRing] = {}, tev_[kRing][2] = {}, t0_ = nullptr, t1_ = nullptr;
  int retired_ = 0, timed_ = 0, active_ = 0;
  long long searches_ = 0;
  double search_ms_ = 0.0;
};

}  // namespace muz
