// Block pipeline (include/yara_amd.h, yr_amd_pipeline_*): SURVEY.md §8f row 2,
// on one device or split across several (§8e).
//
// libyara's block driver (yr_scanner_scan_mem_blocks, scanner.c:417-583)
// handles one YR_MEMORY_BLOCK at a time: fetch, walk, verify, next.  On the
// GPU the per-block cost is H2D + scan + pre-verify on the device and the
// replay of the surviving calls on the host; the pipeline overlaps them: while
// the host replays block k, blocks k+1 .. k+depth are copied and scanned.
//
// Each slot owns one lane per device (hostio.h Lane: a scanner with its own
// HIP stream and device window buffer, and a persistent worker thread), a
// pinned host copy of its block and, for the single-device memcpy path, a
// pageable one.  Results are handed back strictly in submission order, so the
// replay order is the reference's block order; a block split across devices
// comes back as the concatenation of its lanes' records, which is exactly the
// single-device record stream of the whole block (multi.cpp).
//
// Two ways in.  yr_amd_pipeline_submit copies the block in the caller's thread
// (a fault on an mmap'ed block unwinds through the caller's YR_TRYCATCH);
// single-device, the worker then runs yr_amd_scan_block_verified on that copy
// (the runtime stages the H2D: two host passes over every byte, ~23 GB/s).
// yr_amd_pipeline_submit_dma instead copies the caller's bytes into the slot's
// PINNED buffer with several threads at once (hostio.h CopyPool: one host pass
// at the machine's memory bandwidth, not one core's) and returns -- the
// caller's buffer is free again -- and every lane DMAs its window of the
// pinned copy to its device and scans it; the pinned copy is what the replay
// reads.  The copy goes through the caller's copy function when one is set
// (yr_amd_pipeline_set_copy): the libyara shim passes one that copies inside
// YR_TRYCATCH on whichever thread runs it, so a fault on a helper thread is a
// failed copy (YR_AMD_COULD_NOT_MAP_FILE), never an unhandled SIGBUS.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/yara_amd.h"
#include "hostio.h"

using yamd::CopyFn;
using yamd::CopyPool;
using yamd::Lane;

namespace {

enum SlotState { kIdle, kSubmitted, kDone, kHeld };

struct Slot {
  std::vector<Lane> lanes;
  std::vector<std::thread> workers;   // one per lane
  uint8_t* buf = nullptr;             // pageable copy (single-device submit)
  size_t cap = 0;
  uint8_t* h_pinned = nullptr;        // pinned copy (submit_dma, and submit across devices)
  size_t h_cap = 0;
  size_t size = 0;
  uint64_t base = 0;
  SlotState state = kIdle;
  bool dma = false;
  uint64_t gen = 0;                   // submissions of this slot (wakes its lanes)
  std::condition_variable cv;         // the slot's lanes wait here (under the pipeline's mutex)
  uint32_t left = 0;                  // lanes still working on the submission
  int rc = 0;
  const yr_amd_verify_rec* recs = nullptr;
  uint64_t count = 0;
  std::vector<yr_amd_verify_rec> out;  // concatenated lane records
  // single device, pageable copy: the scanner's own records (valid until the
  // slot's next submission), no copy
  const yr_amd_verify_rec* direct = nullptr;
  uint64_t direct_count = 0;
};

}  // namespace

struct yr_amd_pipeline {
  std::vector<Slot> slots;       // depth + 1: one may be held by the caller
  uint32_t depth = 0;
  uint32_t n_lanes = 1;
  uint64_t halo_before = 0, halo_after = 0;
  uint64_t split_min = 0;        // blocks below this go whole to one lane
  uint64_t submitted = 0;        // (round-robin lane of whole blocks)
  uint32_t head = 0;             // oldest submitted (not yet returned) slot
  uint32_t in_flight = 0;        // submitted, not yet returned
  int held = -1;                 // slot returned by the last pipeline_next
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv;    // pipeline_next waits here for the oldest slot
  CopyFn copy;
  CopyPool* copier = nullptr;    // submit_dma's parallel host copy (created on first use)
};

namespace {

// One lane's share of a DMA submission: its window of the pinned copy to its
// device, then scan + pre-verification (records in L.recs).
int run_lane_dma(Slot& s, Lane& L) {
  L.recs.clear();
  L.candidates = 0;
  if (!L.active) return YR_AMD_SUCCESS;
  int r = yamd::lane_reserve(L);
  if (r) return r;
  if (hipSetDevice(L.device) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR;
  if (L.hi > L.lo && hipMemcpyAsync(L.d_win, s.h_pinned + L.lo, L.hi - L.lo, hipMemcpyHostToDevice,
                                    L.stream) != hipSuccess)
    return YR_AMD_INTERNAL_FATAL_ERROR;
  r = yamd::lane_scan(L, s.size, s.base);
  // (a failed scan may have left the DMA queued: the slot's pinned copy is
  // refilled by a later submission, so nothing may still read it)
  if (r != YR_AMD_SUCCESS) (void)hipStreamSynchronize(L.stream);
  return r;
}

void lane_main(yr_amd_pipeline* p, uint32_t idx, uint32_t k) {
  Slot& s = p->slots[idx];
  Lane& L = s.lanes[k];
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(p->mu);
  for (;;) {
    s.cv.wait(lk, [&] { return p->stop || (s.state == kSubmitted && s.gen != seen); });
    if (p->stop) return;
    seen = s.gen;
    lk.unlock();
    int rc;
    if (s.dma) {
      rc = run_lane_dma(s, L);
    } else {
      // single device, pageable copy: H2D + scan + pre-verification in one call
      const yr_amd_verify_rec* recs = nullptr;
      uint64_t n = 0;
      rc = yr_amd_scan_block_verified(L.scanner, s.buf, s.size, s.base, &recs, &n);
      s.direct = rc == YR_AMD_SUCCESS ? recs : nullptr;
      s.direct_count = rc == YR_AMD_SUCCESS ? n : 0;
      L.candidates = 0;
    }
    lk.lock();
    L.status = rc;
    if (--s.left == 0) {
      s.state = kDone;
      p->cv.notify_all();
    }
  }
}

void release_held(yr_amd_pipeline* p) {
  if (p->held >= 0) {
    p->slots[p->held].state = kIdle;
    p->held = -1;
  }
}

// The next free slot for a submission (under p->mu), or -1.
int claim_slot(yr_amd_pipeline* p, int* err) {
  if (p->in_flight >= p->depth) {   // call pipeline_next first
    *err = YR_AMD_INVALID_ARGUMENT;
    return -1;
  }
  const uint32_t idx = (p->head + p->in_flight) % (p->depth + 1);
  if ((int)idx == p->held) release_held(p);
  if (p->slots[idx].state != kIdle) {
    *err = YR_AMD_INTERNAL_FATAL_ERROR;
    return -1;
  }
  return (int)idx;
}

int reserve_pinned(Slot& s, size_t need, int device) {
  if (need <= s.h_cap) return YR_AMD_SUCCESS;
  if (hipSetDevice(device) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR;
  if (s.h_pinned) (void)hipHostFree(s.h_pinned);
  s.h_pinned = nullptr;
  s.h_cap = 0;
  if (hipHostMalloc((void**)&s.h_pinned, need, hipHostMallocPortable) != hipSuccess) {
    s.h_pinned = nullptr;
    return YR_AMD_INSUFFICIENT_MEMORY;
  }
  s.h_cap = need;
  return YR_AMD_SUCCESS;
}

// Hand a filled slot to its lanes.
void start_slot(yr_amd_pipeline* p, Slot& s, size_t size, uint64_t base, bool dma) {
  int whole = -1;
  if (p->n_lanes > 1 && size < p->split_min) whole = (int)(p->submitted % p->n_lanes);
  yamd::lanes_split(s.lanes, size, p->halo_before, p->halo_after, whole);
  {
    std::lock_guard<std::mutex> lk(p->mu);
    ++p->submitted;
    s.dma = dma;
    s.size = size;
    s.base = base;
    s.left = (uint32_t)s.lanes.size();
    for (Lane& L : s.lanes) L.status = YR_AMD_SUCCESS;
    ++s.gen;
    s.state = kSubmitted;
    ++p->in_flight;
  }
  s.cv.notify_all();
}

int create(yr_amd_tables* const* tables, uint32_t n, uint32_t depth, yr_amd_pipeline** out) {
  if (out == nullptr) return YR_AMD_INVALID_ARGUMENT;
  *out = nullptr;
  if (tables == nullptr || n == 0 || n > YR_AMD_MAX_DEVICES || depth == 0 || depth > 8)
    return YR_AMD_INVALID_ARGUMENT;
  yr_amd_tables_info ref{};
  for (uint32_t k = 0; k < n; ++k) {
    if (tables[k] == nullptr) return YR_AMD_INVALID_ARGUMENT;
    if (n == 1) break;
    // across devices: the same rule set on every device, with its strings
    yr_amd_tables_info info{};
    if (yr_amd_tables_get_info(tables[k], &info) != YR_AMD_SUCCESS) return YR_AMD_INVALID_ARGUMENT;
    if (k == 0) ref = info;
    if (info.n_slots != ref.n_slots || info.n_states != ref.n_states ||
        info.accepting_states != ref.accepting_states || info.verify_halo_before == 0 ||
        info.verify_halo_before != ref.verify_halo_before ||
        info.verify_halo_after != ref.verify_halo_after)
      return YR_AMD_INVALID_ARGUMENT;
  }
  yr_amd_pipeline* p = new (std::nothrow) yr_amd_pipeline();
  if (p == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
  p->depth = depth;
  p->n_lanes = n;
  p->halo_before = ref.verify_halo_before;
  p->halo_after = ref.verify_halo_after;
  p->slots = std::vector<Slot>(depth + 1);
  int r = YR_AMD_SUCCESS;
  for (Slot& s : p->slots) {
    s.lanes.resize(n);
    for (uint32_t k = 0; k < n && r == YR_AMD_SUCCESS; ++k) r = yamd::lane_open(s.lanes[k], tables[k]);
    if (r != YR_AMD_SUCCESS) break;
  }
  if (r != YR_AMD_SUCCESS) {
    yr_amd_pipeline_destroy(p);
    return r;
  }
  for (uint32_t i = 0; i <= depth; ++i)
    for (uint32_t k = 0; k < n; ++k) p->slots[i].workers.emplace_back(lane_main, p, i, k);
  *out = p;
  return YR_AMD_SUCCESS;
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
  for (Slot& s : p->slots) s.cv.notify_all();
  for (Slot& s : p->slots) {
    for (std::thread& t : s.workers) t.join();
    for (Lane& L : s.lanes) yamd::lane_close(L);
    free(s.buf);
    if (s.h_pinned) (void)hipHostFree(s.h_pinned);
  }
  delete p->copier;
  delete p;
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_create(yr_amd_tables* tables, uint32_t depth, yr_amd_pipeline** out) {
  return create(&tables, 1, depth, out);
}

int yr_amd_pipeline_create_multi(yr_amd_tables* const* tables, uint32_t n, uint32_t depth,
                                 yr_amd_pipeline** out) {
  return create(tables, n, depth, out);
}

int yr_amd_pipeline_set_copy(yr_amd_pipeline* p, yr_amd_copy_fn fn, void* user) {
  if (p == nullptr) return YR_AMD_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(p->mu);
  p->copy.fn = fn;
  p->copy.user = user;
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_set_split_min(yr_amd_pipeline* p, uint64_t bytes) {
  if (p == nullptr) return YR_AMD_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(p->mu);
  p->split_min = bytes;
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_submit(yr_amd_pipeline* p, const uint8_t* data, size_t size, uint64_t base) {
  if (p == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  int idx, err = YR_AMD_SUCCESS;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    idx = claim_slot(p, &err);
  }
  if (idx < 0) return err;
  Slot& s = p->slots[idx];
  // The copy runs in the caller's thread with no lock held: a fault on an
  // mmap'ed block unwinds through the caller's YR_TRYCATCH (exception.h)
  // exactly as the reference's in-walk read would (scanner.c:493-496).
  if (p->n_lanes == 1) {
    if (size > s.cap) {
      free(s.buf);
      s.cap = 0;
      s.buf = (uint8_t*)malloc(size);
      if (s.buf == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
      s.cap = size;
    }
    if (!p->copy(s.buf, data, size)) return YR_AMD_COULD_NOT_MAP_FILE;
    start_slot(p, s, size, base, false);
    return YR_AMD_SUCCESS;
  }
  // across devices: the lanes DMA their windows from a pinned copy
  const int r = reserve_pinned(s, size > 0 ? size : 16, s.lanes[0].device);
  if (r) return r;
  if (!p->copy(s.h_pinned, data, size)) return YR_AMD_COULD_NOT_MAP_FILE;
  start_slot(p, s, size, base, true);
  return YR_AMD_SUCCESS;
}

int yr_amd_pipeline_submit_dma(yr_amd_pipeline* p, const uint8_t* data, size_t size,
                               uint64_t base) {
  if (p == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  int idx, err = YR_AMD_SUCCESS;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    idx = claim_slot(p, &err);
  }
  if (idx < 0) return err;
  Slot& s = p->slots[idx];
  const int r = reserve_pinned(s, size > 0 ? size : 16, s.lanes[0].device);
  if (r) return r;
  // the caller's bytes into the pinned copy, several threads at once; when
  // it returns the caller may reuse its buffer (the lanes DMA the copy)
  if (size > 0) {
    if (p->copier == nullptr) {
      p->copier = new (std::nothrow) CopyPool(yamd::copy_helpers());
      if (p->copier == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
    }
    if (!p->copier->copy(s.h_pinned, data, size, p->copy)) return YR_AMD_COULD_NOT_MAP_FILE;
  }
  start_slot(p, s, size, base, true);
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
  s.rc = YR_AMD_SUCCESS;
  for (const Lane& L : s.lanes)
    if (L.status != YR_AMD_SUCCESS) {
      s.rc = L.status;
      break;
    }
  s.count = 0;
  s.recs = nullptr;
  if (s.rc == YR_AMD_SUCCESS) {
    if (!s.dma) {   // (single device)
      s.recs = s.direct;
      s.count = s.direct_count;
    } else if (s.lanes.size() == 1) {
      s.recs = s.lanes[0].recs.data();
      s.count = s.lanes[0].recs.size();
    } else {
      yamd::lanes_concat(s.lanes, s.out);
      s.recs = s.out.data();
      s.count = s.out.size();
    }
  }
  if (records) *records = s.recs;
  if (count) *count = s.count;
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
