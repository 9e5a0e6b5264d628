// Host-side input movement shared by the block pipeline (pipeline.cpp) and the
// multi-device scanner (multi.cpp): the parallel, fault-reporting host copy
// into pinned memory, the per-device "lane" that scans its window of a block,
// and the shard / window bounds of SURVEY.md §8e (yara_amd/dist.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/yara_amd.h"

namespace yamd {

// The caller-supplied copy (yr_amd_pipeline_set_copy / yr_amd_multi_set_copy)
// or memcpy.  A libyara caller passes one that runs memcpy inside YR_TRYCATCH
// (exception.h:150-185) on whichever thread calls it, so a block that faults
// (a truncated file mapping) is reported as a failed copy -- never a SIGBUS
// on a helper thread -- and surfaces as YR_AMD_COULD_NOT_MAP_FILE, as the
// reference's walk does at scanner.c:493-496.
struct CopyFn {
  yr_amd_copy_fn fn = nullptr;
  void* user = nullptr;
  bool operator()(void* dst, const void* src, size_t n) const {
    if (n == 0) return true;
    if (fn == nullptr) {
      memcpy(dst, src, n);
      return true;
    }
    return fn(user, dst, src, n) == 0;
  }
};

// A parallel copy: persistent helper threads plus the calling thread claim
// 4 MiB chunks of one job.  A claim is a compare-and-swap on a ticket that
// carries the job's generation, so a helper that wakes late (or is still
// looking for work when the next job starts) can never take a chunk of a job
// it did not snapshot; the caller returns once every chunk of its job has
// been copied (or has failed) -- a chunk counts as done only after its copy.
class CopyPool {
 public:
  static constexpr size_t kChunk = 4u << 20;

  // first_gen: the generation the first job follows (tests start it next to
  // the ticket's wrap point)
  explicit CopyPool(unsigned helpers, uint64_t first_gen = 0) : gen_(first_gen) {
    for (unsigned i = 0; i < helpers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;

  // false: some chunk's copy failed (every other chunk was still attempted)
  bool copy(uint8_t* dst, const uint8_t* src, size_t size, const CopyFn& fn) {
    if (size < 2 * kChunk || th_.empty()) return fn(dst, src, size);
    Job j;
    {
      std::lock_guard<std::mutex> lk(mu_);
      // the ticket keeps 64 - kGenShift bits of the generation: the job's
      // generation is stored and compared in that width, so it wraps with the
      // ticket (a full-width generation stopped matching its own
      // ticket after 2^24 jobs and every claim loop returned at once)
      job_ = Job{dst, src, size, fn, ++gen_ & kGenMask};
      j = job_;
      done_ = 0;
      failed_ = false;
      ticket_.store(j.gen << kGenShift);
    }
    cv_.notify_all();
    work(j);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return done_ == size; });
    return !failed_;
  }

 private:
  // ticket = generation << kGenShift | next chunk index
  static constexpr unsigned kGenShift = 40;
  static constexpr uint64_t kGenMask = (1ull << (64 - kGenShift)) - 1;
  struct Job {
    uint8_t* dst = nullptr;
    const uint8_t* src = nullptr;
    size_t size = 0;
    CopyFn fn;
    uint64_t gen = 0;
  };
  void work(const Job& j) {
    const uint64_t n_chunks = (j.size + kChunk - 1) / kChunk;
    for (;;) {
      uint64_t t = ticket_.load();
      uint64_t c;
      do {
        if ((t >> kGenShift) != j.gen) return;        // another job's ticket
        c = t & ((1ull << kGenShift) - 1);
        if (c >= n_chunks) return;                    // all claimed
      } while (!ticket_.compare_exchange_weak(t, t + 1));
      const size_t off = c * kChunk, n = std::min(kChunk, j.size - off);
      const bool ok = j.fn(j.dst + off, j.src + off, n);
      std::lock_guard<std::mutex> lk(mu_);
      if (!ok) failed_ = true;
      done_ += n;
      if (done_ == j.size) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const Job j = job_;   // snapshot under the lock
      lk.unlock();
      work(j);
      lk.lock();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  Job job_;
  uint64_t gen_ = 0;   // full width (the helpers' wake-up test); jobs use gen_ & kGenMask
  size_t done_ = 0;
  bool failed_ = false;
  bool stop_ = false;
  std::atomic<uint64_t> ticket_{0};
};

// Helper threads for a CopyPool: half the machine's threads, at most 7.
inline unsigned copy_helpers() {
  const unsigned hw = std::thread::hardware_concurrency();
  return std::min(7u, hw > 1 ? hw / 2 : 0u);
}

constexpr uint64_t kShardAlign = 1u << 20;   // dist.py shard_bounds

// [begin, end) of device k of n in a block of `size` bytes (dist.py shard_bounds).
inline void shard_of(uint64_t size, uint32_t n, uint32_t k, uint64_t& begin, uint64_t& end) {
  const uint64_t per = (size / n) / kShardAlign * kShardAlign;
  begin = (uint64_t)k * per;
  end = k == n - 1 ? size : begin + per;
}

// [lo, hi): the bytes a device holds for [begin, end) (dist.py shard_window).
inline void window_of(uint64_t size, uint64_t begin, uint64_t end, uint64_t before, uint64_t after,
                      uint64_t& lo, uint64_t& hi) {
  before = std::max<uint64_t>(before, YR_AMD_MAX_ATOM_LENGTH);
  lo = (begin - std::min(begin, before)) / 16 * 16;
  hi = std::min(size, end + after);
}

// One device's share of a block: its scanner, stream and window buffer, and
// the records of its last scan.
struct Lane {
  yr_amd_tables* tables = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;   // the scanner's stream; H2D copies go on it too
  yr_amd_scanner* scanner = nullptr;
  uint8_t* d_win = nullptr;
  size_t d_win_cap = 0;
  std::vector<yr_amd_verify_rec> recs;
  uint64_t candidates = 0;        // of its last scan (the rebase of candidate indices)
  int status = YR_AMD_SUCCESS;
  // the lane's range of the current block: positions (begin, end], window [lo, hi)
  uint64_t begin = 0, end = 0, lo = 0, hi = 0;
  bool active = false;            // owns positions of the current block
};

// Create / destroy a lane's stream and scanner on its tables' device.
int lane_open(Lane& L, yr_amd_tables* tables);
void lane_close(Lane& L);
// Room for the window on the device (L.hi - L.lo bytes).
int lane_reserve(Lane& L);
// Scan the window (already in L.d_win) and pre-verify its candidates; the
// records land in L.recs (block-global offsets, candidate indices of this lane).
int lane_scan(Lane& L, uint64_t size, uint64_t data_base);
// Concatenate the lanes' records in order, rebasing candidate indices onto the
// whole block's candidate stream (mod 2^32, as a single scan's).
void lanes_concat(const std::vector<Lane>& lanes, std::vector<yr_amd_verify_rec>& out);
// Set each lane's range and window for a block of `size` bytes split over the
// n lanes (n = 1: the whole block, no halos); `whole` >= 0: the whole block
// goes to that lane alone.
void lanes_split(std::vector<Lane>& lanes, uint64_t size, uint64_t halo_before, uint64_t halo_after,
                 int whole);

}  // namespace yamd
