// Block pipeline (include/yara_amd.h, yr_amd_pipeline_*): SURVEY.md §8f row 2.
//
// libyara's block driver (yr_scanner_scan_mem_blocks, scanner.c:417-583)
// handles one YR_MEMORY_BLOCK at a time: fetch, walk, verify, next.  On the
// GPU the per-block cost is H2D + scan + pre-verify on the device and the
// replay of the surviving calls on the host; the pipeline overlaps them: while
// the host replays block k, blocks k+1 .. k+depth are copied and scanned.
//
// Each slot owns a scanner (its own HIP stream and device workspace), a host
// copy of its block and a worker thread that runs
// yr_amd_scan_block_verified for it.  Results are handed back strictly in
// submission order, so the replay order is the reference's block order.
//
// Two ways in.  yr_amd_pipeline_submit copies the block with memcpy in the
// caller's thread (a fault on an mmap'ed block unwinds through the caller's
// YR_TRYCATCH), then the worker's H2D reads that copy: two host passes over
// every byte (the memcpy and the runtime's pageable staging), ~23 GB/s.
// yr_amd_pipeline_submit_dma instead copies the caller's bytes into the slot's
// PINNED host buffer with several threads at once (the caller's thread and a
// small pool: one host pass at the machine's memory bandwidth, not one
// core's), returns -- the caller's buffer is free again -- and the worker moves
// the pinned copy to the device with a plain DMA (no runtime staging), then
// scans it; the pinned copy is what the replay reads.  Helper threads cannot
// unwind a fault through the caller's YR_TRYCATCH, so the caller must have
// made every page of the block readable first (the shim touches each page
// inside its YR_TRYCATCH, as for its direct blocks).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/yara_amd.h"

namespace {

enum SlotState { kIdle, kSubmitted, kDone, kHeld };

struct Slot {
  yr_amd_scanner* scanner = nullptr;
  uint8_t* buf = nullptr;       // host copy of the block (pageable: the H2D
                                // path of the runtime is faster than a host
                                // memcpy into pinned memory)
  size_t cap = 0;
  size_t size = 0;
  uint64_t base = 0;
  SlotState state = kIdle;
  int rc = 0;
  const yr_amd_verify_rec* recs = nullptr;
  uint64_t count = 0;
  std::thread worker;
  // submit_dma: the block on the device, its host copy in pinned memory, the
  // records fetched by the worker
  bool dma = false;
  int device = 0;
  hipStream_t copy_stream = nullptr;
  uint8_t* d_buf = nullptr;
  size_t d_cap = 0;
  uint8_t* h_pinned = nullptr;
  size_t h_cap = 0;
  std::vector<yr_amd_verify_rec> h_recs;
};

// A parallel memcpy: persistent helper threads plus the calling thread take
// 4 MiB chunks of one copy job from an atomic counter.
class CopyPool {
 public:
  explicit CopyPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  void copy(uint8_t* dst, const uint8_t* src, size_t size) {
    if (size < 2 * kChunk || th_.empty()) {
      memcpy(dst, src, size);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      dst_ = dst;
      src_ = src;
      size_ = size;
      next_.store(0);
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return done_ == size_; });
  }

 private:
  static constexpr size_t kChunk = 4u << 20;
  void work() {   // take chunks until the job is exhausted
    for (;;) {
      const size_t off = next_.fetch_add(kChunk);
      if (off >= size_) return;
      const size_t n = std::min(kChunk, size_ - off);
      memcpy(dst_ + off, src_ + off, n);
      std::lock_guard<std::mutex> lk(mu_);
      done_ += n;
      if (done_ == size_) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      lk.unlock();
      work();
      lk.lock();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  size_t size_ = 0, done_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

struct yr_amd_pipeline {
  std::vector<Slot> slots;       // depth + 1: one may be held by the caller
  uint32_t depth = 0;
  uint32_t head = 0;             // oldest submitted (not yet returned) slot
  uint32_t in_flight = 0;        // submitted, not yet returned
  int held = -1;                 // slot returned by the last pipeline_next
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv;
  CopyPool* copier = nullptr;   // submit_dma's parallel host copy (created on first use)
};

namespace {

// A submit_dma block on the worker: the pinned host copy goes to the device
// by DMA, then the block is scanned and pre-verified there.
int run_dma(Slot& s, const yr_amd_verify_rec** recs, uint64_t* n) {
  *recs = nullptr;
  *n = 0;
  if (hipSetDevice(s.device) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR;
  if (s.size > 0 && (hipMemcpyAsync(s.d_buf, s.h_pinned, s.size, hipMemcpyHostToDevice,
                                    s.copy_stream) != hipSuccess ||
                     hipStreamSynchronize(s.copy_stream) != hipSuccess))
    return YR_AMD_COULD_NOT_MAP_FILE;
  int r = yr_amd_scan_device(s.scanner, s.d_buf, s.size, 0, s.size);
  if (!r) r = yr_amd_scan_device_result(s.scanner, nullptr, nullptr, nullptr);
  const yr_amd_verify_rec* d_rec = nullptr;
  uint64_t cnt = 0;
  if (!r) r = yr_amd_verify_device(s.scanner, s.base, &d_rec, &cnt);
  if (!r) {
    s.h_recs.resize(cnt);
    if (cnt > 0 && hipMemcpy(s.h_recs.data(), d_rec, cnt * sizeof(yr_amd_verify_rec),
                             hipMemcpyDeviceToHost) != hipSuccess)
      r = YR_AMD_INTERNAL_FATAL_ERROR;
  }
  if (r) return r;
  *recs = s.h_recs.data();
  *n = cnt;
  return YR_AMD_SUCCESS;
}

void worker_main(yr_amd_pipeline* p, uint32_t idx) {
  Slot& s = p->slots[idx];
  std::unique_lock<std::mutex> lk(p->mu);
  for (;;) {
    p->cv.wait(lk, [&] { return p->stop || s.state == kSubmitted; });
    if (p->stop) return;
    lk.unlock();
    const yr_amd_verify_rec* recs = nullptr;
    uint64_t n = 0;
    const int rc = s.dma ? run_dma(s, &recs, &n)
                         : yr_amd_scan_block_verified(s.scanner, s.buf, s.size, s.base, &recs, &n);
    lk.lock();
    s.rc = rc;
    s.recs = recs;
    s.count = n;
    s.state = kDone;
    p->cv.notify_all();
  }
}

void release_held(yr_amd_pipeline* p) {
  if (p->held >= 0) {
    p->slots[p->held].state = kIdle;
    p->held = -1;
  }
}

}  // namespace

extern "C" {

int yr_amd_pipeline_destroy(yr_amd_pipeline* p) {
  if (p == nullptr) return YR_AMD_SUCCESS;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    p->stop = true;
  }
  p->cv.notify_all();
  for (Slot& s : p->slots) {
    if (s.worker.joinable()) s.worker.join();
    if (s.scanner) yr_amd_scanner_destroy(s.scanner);
    free(s.buf);
    if (s.copy_stream) {
      (void)hipSetDevice(s.device);
      (void)hipStreamSynchronize(s.copy_stream);
      (void)hipStreamDestroy(s.copy_stream);
    }
    if (s.d_buf) (void)hipFree(s.d_buf);
    if (s.h_pinned) (void)hipHostFree(s.h_pinned);
  }
  delete p->copier;
  delete p;
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_create(yr_amd_tables* tables, uint32_t depth, yr_amd_pipeline** out) {
  if (tables == nullptr || out == nullptr || depth == 0 || depth > 8) return YR_AMD_INVALID_ARGUMENT;
  *out = nullptr;
  yr_amd_pipeline* p = new (std::nothrow) yr_amd_pipeline();
  if (p == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
  p->depth = depth;
  p->slots = std::vector<Slot>(depth + 1);
  const int device = yr_amd_tables_device(tables);
  for (Slot& s : p->slots) {
    s.device = device;
    const int r = yr_amd_scanner_create(tables, nullptr, &s.scanner);
    if (r != YR_AMD_SUCCESS) {
      yr_amd_pipeline_destroy(p);
      return r;
    }
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&s.copy_stream, hipStreamNonBlocking) != hipSuccess) {
      s.copy_stream = nullptr;
      yr_amd_pipeline_destroy(p);
      return YR_AMD_INTERNAL_FATAL_ERROR;
    }
  }
  for (uint32_t i = 0; i <= depth; ++i) p->slots[i].worker = std::thread(worker_main, p, i);
  *out = p;
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_submit(yr_amd_pipeline* p, const uint8_t* data, size_t size, uint64_t base) {
  if (p == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  uint32_t idx;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->in_flight >= p->depth) return YR_AMD_INVALID_ARGUMENT;   // call pipeline_next first
    idx = (p->head + p->in_flight) % (p->depth + 1);
    if ((int)idx == p->held) release_held(p);
    if (p->slots[idx].state != kIdle) return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  Slot& s = p->slots[idx];
  if (size > s.cap) {
    free(s.buf);
    s.cap = 0;
    s.buf = (uint8_t*)malloc(size);
    if (s.buf == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
    s.cap = size;
  }
  // The copy runs in the caller's thread with no lock held: a fault on an
  // mmap'ed block unwinds through the caller's YR_TRYCATCH (exception.h)
  // exactly as the reference's in-walk read would (scanner.c:493-496).
  if (size > 0) memcpy(s.buf, data, size);
  {
    std::lock_guard<std::mutex> lk(p->mu);
    s.dma = false;
    s.size = size;
    s.base = base;
    s.state = kSubmitted;
    ++p->in_flight;
  }
  p->cv.notify_all();
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_submit_dma(yr_amd_pipeline* p, const uint8_t* data, size_t size,
                               uint64_t base) {
  if (p == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  uint32_t idx;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->in_flight >= p->depth) return YR_AMD_INVALID_ARGUMENT;   // call pipeline_next first
    idx = (p->head + p->in_flight) % (p->depth + 1);
    if ((int)idx == p->held) release_held(p);
    if (p->slots[idx].state != kIdle) return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  Slot& s = p->slots[idx];
  if (hipSetDevice(s.device) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR;
  const size_t need = size > 0 ? size : 16;
  if (need > s.d_cap) {
    if (s.d_buf) (void)hipFree(s.d_buf);
    s.d_buf = nullptr;
    s.d_cap = 0;
    if (hipMalloc((void**)&s.d_buf, need) != hipSuccess) {
      s.d_buf = nullptr;
      return YR_AMD_INSUFFICIENT_MEMORY;
    }
    s.d_cap = need;
  }
  if (need > s.h_cap) {
    if (s.h_pinned) (void)hipHostFree(s.h_pinned);
    s.h_pinned = nullptr;
    s.h_cap = 0;
    if (hipHostMalloc((void**)&s.h_pinned, need, hipHostMallocDefault) != hipSuccess) {
      s.h_pinned = nullptr;
      return YR_AMD_INSUFFICIENT_MEMORY;
    }
    s.h_cap = need;
  }
  // the caller's bytes into the pinned copy, several threads at once; when
  // it returns the caller may reuse its buffer (the worker DMAs the copy)
  if (size > 0) {
    if (p->copier == nullptr) {
      const unsigned hw = std::thread::hardware_concurrency();
      p->copier = new (std::nothrow) CopyPool(std::min(7u, hw > 1 ? hw / 2 : 0u));
      if (p->copier == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
    }
    p->copier->copy(s.h_pinned, data, size);
  }
  {
    std::lock_guard<std::mutex> lk(p->mu);
    s.dma = true;
    s.size = size;
    s.base = base;
    s.state = kSubmitted;
    ++p->in_flight;
  }
  p->cv.notify_all();
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_next(yr_amd_pipeline* p, const yr_amd_verify_rec** records, uint64_t* count,
                         const uint8_t** data, size_t* size, uint64_t* base) {
  if (p == nullptr) return YR_AMD_INVALID_ARGUMENT;
  std::unique_lock<std::mutex> lk(p->mu);
  release_held(p);
  if (p->in_flight == 0) return YR_AMD_INVALID_ARGUMENT;
  Slot& s = p->slots[p->head];
  p->cv.wait(lk, [&] { return s.state == kDone; });
  s.state = kHeld;
  p->held = (int)p->head;
  p->head = (p->head + 1) % (p->depth + 1);
  --p->in_flight;
  if (records) *records = s.recs;
  if (count) *count = s.rc == YR_AMD_SUCCESS ? s.count : 0;
  if (data) *data = s.dma ? s.h_pinned : s.buf;
  if (size) *size = s.size;
  if (base) *base = s.base;
  return s.rc;
}

int yr_amd_pipeline_drain(yr_amd_pipeline* p) {
  if (p == nullptr) return YR_AMD_INVALID_ARGUMENT;
  while (true) {
    {
      std::lock_guard<std::mutex> lk(p->mu);
      if (p->in_flight == 0) {
        release_held(p);
        return YR_AMD_SUCCESS;
      }
    }
    (void)yr_amd_pipeline_next(p, nullptr, nullptr, nullptr, nullptr, nullptr);
  }
}

}  // extern "C"
