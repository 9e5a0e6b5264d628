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
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

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
};

namespace {

void worker_main(yr_amd_pipeline* p, uint32_t idx) {
  Slot& s = p->slots[idx];
  std::unique_lock<std::mutex> lk(p->mu);
  for (;;) {
    p->cv.wait(lk, [&] { return p->stop || s.state == kSubmitted; });
    if (p->stop) return;
    lk.unlock();
    const yr_amd_verify_rec* recs = nullptr;
    uint64_t n = 0;
    const int rc = yr_amd_scan_block_verified(s.scanner, s.buf, s.size, s.base, &recs, &n);
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
  }
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
  for (Slot& s : p->slots) {
    const int r = yr_amd_scanner_create(tables, nullptr, &s.scanner);
    if (r != YR_AMD_SUCCESS) {
      yr_amd_pipeline_destroy(p);
      return r;
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
  if (data) *data = s.buf;
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
