// Multi-device block scans behind the C ABI (include/yara_amd.h
// yr_amd_multi_*), and the per-device lanes they share with the
// multi-device block pipeline (pipeline.cpp).
//
// One process drives n devices: a host block is split into n byte ranges
// (equal 1 MiB-aligned slices, the last takes the rest -- the same bounds as
// yara_amd/dist.py shard_bounds), device k receives only its WINDOW of the
// block (its range plus the tables' verify halos, yr_amd_tables_get_info),
// scans it with yr_amd_scan_window and pre-verifies its own candidates with
// yr_amd_verify_device.  Records are block-global, so their concatenation in
// device order is exactly the single-device record stream of the whole block
// (yr_amd_scan_block_verified): the libyara side replays it into the
// unmodified yr_scan_verify_match (scanner.c:105-121) as before.  No data-path
// exchange between devices; the "gather" is the host concatenation.
//
// Moving the block: the caller's bytes go through two pinned staging buffers
// of kStage bytes -- a parallel copy (CopyPool, through the caller's copy
// function: fault-reporting for mmapped data) fills one while the devices
// whose windows overlap the other DMA their part of it -- so the host makes
// one pass over the block at memory bandwidth and the devices take it at link
// rate, with bounded pinned memory (a 32 GiB block needs 2 x 256 MiB).  Then
// every device scans and pre-verifies its window on its own persistent worker
// thread.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/yara_amd.h"
#include "hostio.h"
#include "internal.h"

namespace yamd {

int lane_open(Lane& L, yr_amd_tables* tables) {
  L.tables = tables;
  L.device = yr_amd_tables_device(tables);
  if (L.device < 0 || hipSetDevice(L.device) != hipSuccess ||
      hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking) != hipSuccess) {
    L.stream = nullptr;
    return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  int r = yr_amd_scanner_create(tables, L.stream, &L.scanner);
  // a lane's scans serve its records only
  if (!r) r = yr_amd_scanner_set_verified_only(L.scanner, 1);
  return r;
}

void lane_close(Lane& L) {
  if (L.stream == nullptr) return;
  (void)hipSetDevice(L.device);
  (void)hipStreamSynchronize(L.stream);
  yr_amd_scanner_destroy(L.scanner);
  L.scanner = nullptr;
  if (L.d_win) (void)hipFree(L.d_win);
  L.d_win = nullptr;
  L.d_win_cap = 0;
  (void)hipStreamDestroy(L.stream);
  L.stream = nullptr;
}

int lane_reserve(Lane& L) {
  const uint64_t n = std::max<uint64_t>(L.hi - L.lo, 16);
  if (L.d_win != nullptr && n <= L.d_win_cap) return YR_AMD_SUCCESS;
  if (hipSetDevice(L.device) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR;
  if (L.d_win) (void)hipFree(L.d_win);
  L.d_win = nullptr;
  L.d_win_cap = 0;
  if (hipMalloc((void**)&L.d_win, n) != hipSuccess) {
    L.d_win = nullptr;
    return YR_AMD_INSUFFICIENT_MEMORY;
  }
  L.d_win_cap = n;
  return YR_AMD_SUCCESS;
}

int lane_scan(Lane& L, uint64_t size, uint64_t data_base) {
  L.recs.clear();
  L.candidates = 0;
  if (!L.active) return YR_AMD_SUCCESS;
  if (hipSetDevice(L.device) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR;
  int r = yr_amd_scan_window(L.scanner, L.d_win, L.lo, L.hi, size, L.begin, L.end);
  int all = 0;
  if (!r) r = yr_amd_scan_device_result(L.scanner, nullptr, nullptr, &all);
  // (the full stream's length: a verified-only scan's result may leave
  // candidates out, the records' candidate indices do not)
  if (!r) r = yr_amd_scan_device_stream_length(L.scanner, &L.candidates);
  // a root-accepting rule set: every position of (begin, end] is a candidate
  // (and position 0 on the lane that starts the block)
  if (all) L.candidates = (L.end - L.begin) + (L.begin == 0 ? 1u : 0u);
  const yr_amd_verify_rec* d_rec = nullptr;
  uint64_t cnt = 0;
  if (!r) r = yr_amd_verify_device(L.scanner, data_base, &d_rec, &cnt);
  if (r) return r;
  L.recs.resize(cnt);
  if (cnt > 0 &&
      (hipMemcpyAsync(L.recs.data(), d_rec, cnt * sizeof(yr_amd_verify_rec), hipMemcpyDeviceToHost,
                      L.stream) != hipSuccess ||
       hipStreamSynchronize(L.stream) != hipSuccess))
    return YR_AMD_INTERNAL_FATAL_ERROR;
  return YR_AMD_SUCCESS;
}

void lanes_concat(const std::vector<Lane>& lanes, std::vector<yr_amd_verify_rec>& out) {
  size_t total = 0;
  for (const Lane& L : lanes) total += L.recs.size();
  out.resize(total);
  size_t o = 0;
  uint64_t cand_base = 0;
  for (const Lane& L : lanes) {
    for (size_t i = 0; i < L.recs.size(); ++i) {
      out[o + i] = L.recs[i];
      out[o + i].candidate = (uint32_t)(L.recs[i].candidate + cand_base);
    }
    o += L.recs.size();
    cand_base += L.candidates;
  }
}

void lanes_split(std::vector<Lane>& lanes, uint64_t size, uint64_t halo_before, uint64_t halo_after,
                 int whole) {
  const uint32_t n = (uint32_t)lanes.size();
  for (uint32_t k = 0; k < n; ++k) {
    Lane& L = lanes[k];
    if (whole >= 0) {
      L.begin = L.lo = 0;
      L.end = L.hi = (int)k == whole ? size : 0;
      L.active = (int)k == whole;
      continue;
    }
    shard_of(size, n, k, L.begin, L.end);
    if (n == 1) {
      L.lo = 0;
      L.hi = size;
    } else {
      window_of(size, L.begin, L.end, halo_before, halo_after, L.lo, L.hi);
    }
    // an empty range owns no position (a block smaller than one slice per
    // device: the last device takes all of it, position 0 included); only an
    // empty block is scanned, by the last device, for its position 0
    L.active = L.begin != L.end || (size == 0 && k == n - 1);
  }
}

}  // namespace yamd

using yamd::CopyFn;
using yamd::CopyPool;
using yamd::Lane;

struct yr_amd_multi {
  std::vector<Lane> lanes;
  uint64_t halo_before = 0, halo_after = 0;
  std::vector<yr_amd_verify_rec> out;
  CopyFn copy;
  CopyPool* pool = nullptr;
  // staging: two pinned buffers, and per buffer one event per lane (its DMA
  // out of that buffer)
  static constexpr size_t kStage = 256u << 20;
  uint8_t* stage[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> staged[2];
  // persistent lane workers (scan + pre-verification)
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0, size = 0, base = 0;
  uint32_t left = 0;
  bool stop = false;
};

namespace {

void lane_worker(yr_amd_multi* m, uint32_t k) {
  Lane& L = m->lanes[k];
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(m->mu);
  for (;;) {
    m->cv.wait(lk, [&] { return m->stop || m->gen != seen; });
    if (m->stop) return;
    seen = m->gen;
    const uint64_t size = m->size, base = m->base;
    lk.unlock();
    if (L.status == YR_AMD_SUCCESS) {
      L.status = yamd::lane_scan(L, size, base);
      // a failed scan may leave this block's DMA queued on the lane's stream:
      // stage_block refills the pinned buffers on the next call without
      // waiting for it (the invariant stage_block's comment states)
      if (L.status != YR_AMD_SUCCESS) (void)hipStreamSynchronize(L.stream);
    }
    lk.lock();
    if (--m->left == 0) m->cv.notify_all();
  }
}

// The block's bytes into every active lane's window: staged through the two
// pinned buffers, each kStage piece copied once (in parallel, through the
// caller's copy function) and DMA'd to every lane whose window overlaps it.
int stage_block(yr_amd_multi* m, const uint8_t* data, uint64_t size) {
  uint64_t lo = UINT64_MAX, hi = 0;   // the union of the windows
  for (const Lane& L : m->lanes)
    if (L.active && L.hi > L.lo) {
      lo = std::min(lo, L.lo);
      hi = std::max(hi, L.hi);
    }
  if (lo >= hi) return YR_AMD_SUCCESS;
  for (int b = 0; b < 2; ++b) {
    if (m->stage[b] == nullptr) {
      (void)hipSetDevice(m->lanes[0].device);
      if (hipHostMalloc((void**)&m->stage[b], yr_amd_multi::kStage, hipHostMallocPortable) !=
          hipSuccess) {
        m->stage[b] = nullptr;
        return YR_AMD_INSUFFICIENT_MEMORY;
      }
    }
  }
  int rc = YR_AMD_SUCCESS;
  uint32_t piece = 0;
  for (uint64_t p0 = lo; p0 < hi && rc == YR_AMD_SUCCESS; p0 += yr_amd_multi::kStage, ++piece) {
    const uint32_t b = piece & 1u;
    const uint64_t p1 = std::min(hi, p0 + yr_amd_multi::kStage);
    // the DMAs that last read this buffer must be done before it is refilled
    for (size_t k = 0; k < m->lanes.size() && rc == YR_AMD_SUCCESS; ++k)
      if (piece >= 2 && hipEventSynchronize(m->staged[b][k]) != hipSuccess) rc = YR_AMD_INTERNAL_FATAL_ERROR;
    if (rc != YR_AMD_SUCCESS) break;
    if (!m->pool->copy(m->stage[b], data + p0, p1 - p0, m->copy)) {
      rc = YR_AMD_COULD_NOT_MAP_FILE;
      break;
    }
    for (size_t k = 0; k < m->lanes.size() && rc == YR_AMD_SUCCESS; ++k) {
      Lane& L = m->lanes[k];
      const uint64_t a = std::max(p0, L.lo), e = std::min(p1, L.hi);
      if (hipSetDevice(L.device) != hipSuccess ||
          (L.active && a < e &&
           hipMemcpyAsync(L.d_win + (a - L.lo), m->stage[b] + (a - p0), e - a, hipMemcpyHostToDevice,
                          L.stream) != hipSuccess) ||
          hipEventRecord(m->staged[b][k], L.stream) != hipSuccess)
        rc = YR_AMD_INTERNAL_FATAL_ERROR;
    }
  }
  // (the scans are queued behind the DMAs on the same streams.)  On failure no
  // DMA may still read a staging buffer when the call returns: the next call
  // refills both without waiting
  if (rc != YR_AMD_SUCCESS)
    for (size_t k = 0; k < m->lanes.size(); ++k) {
      (void)hipSetDevice(m->lanes[k].device);
      (void)hipStreamSynchronize(m->lanes[k].stream);
    }
  return rc;
}

}  // namespace

extern "C" {

int yr_amd_multi_create(yr_amd_tables* const* tables, uint32_t n, yr_amd_multi** multi) {
  if (multi == nullptr) return YR_AMD_INVALID_ARGUMENT;
  *multi = nullptr;
  if (tables == nullptr || n == 0 || n > YR_AMD_MAX_DEVICES) return YR_AMD_INVALID_ARGUMENT;
  yr_amd_tables_info ref{};
  for (uint32_t k = 0; k < n; ++k) {
    yr_amd_tables_info info{};
    if (tables[k] == nullptr || yr_amd_tables_get_info(tables[k], &info) != YR_AMD_SUCCESS)
      return YR_AMD_INVALID_ARGUMENT;
    // the same rule set on every device, with its strings (pre-verification)
    if (k == 0) ref = info;
    if (info.n_slots != ref.n_slots || info.n_states != ref.n_states ||
        info.accepting_states != ref.accepting_states || info.verify_halo_before == 0 ||
        info.verify_halo_before != ref.verify_halo_before ||
        info.verify_halo_after != ref.verify_halo_after)
      return YR_AMD_INVALID_ARGUMENT;
  }
  yr_amd_multi* m = new (std::nothrow) yr_amd_multi();
  if (m == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
  m->halo_before = ref.verify_halo_before;
  m->halo_after = ref.verify_halo_after;
  m->lanes.resize(n);
  int r = YR_AMD_SUCCESS;
  for (uint32_t k = 0; k < n && r == YR_AMD_SUCCESS; ++k) {
    r = yamd::lane_open(m->lanes[k], tables[k]);
    for (int b = 0; b < 2 && r == YR_AMD_SUCCESS; ++b) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) r = YR_AMD_INTERNAL_FATAL_ERROR;
      else m->staged[b].push_back(e);
    }
  }
  if (r == YR_AMD_SUCCESS) {
    m->pool = new (std::nothrow) CopyPool(yamd::copy_helpers());
    if (m->pool == nullptr) r = YR_AMD_INSUFFICIENT_MEMORY;
  }
  if (r == YR_AMD_SUCCESS)
    for (uint32_t k = 0; k < n; ++k) m->workers.emplace_back(lane_worker, m, k);
  if (r != YR_AMD_SUCCESS) {
    yr_amd_multi_destroy(m);
    return r;
  }
  *multi = m;
  return YR_AMD_SUCCESS;
}

int yr_amd_multi_destroy(yr_amd_multi* m) {
  if (m == nullptr) return YR_AMD_SUCCESS;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->stop = true;
  }
  m->cv.notify_all();
  for (std::thread& t : m->workers) t.join();
  for (Lane& L : m->lanes) yamd::lane_close(L);
  for (int b = 0; b < 2; ++b) {
    for (hipEvent_t e : m->staged[b]) (void)hipEventDestroy(e);
    if (m->stage[b]) (void)hipHostFree(m->stage[b]);
  }
  delete m->pool;
  delete m;
  return YR_AMD_SUCCESS;
}

int yr_amd_multi_set_copy(yr_amd_multi* m, yr_amd_copy_fn fn, void* user) {
  if (m == nullptr) return YR_AMD_INVALID_ARGUMENT;
  m->copy.fn = fn;
  m->copy.user = user;
  return YR_AMD_SUCCESS;
}

int yr_amd_multi_shard(const yr_amd_multi* m, uint64_t size, uint32_t k, uint64_t* begin,
                       uint64_t* end, uint64_t* window_begin, uint64_t* window_end) {
  if (m == nullptr || k >= m->lanes.size()) return YR_AMD_INVALID_ARGUMENT;
  uint64_t b, e, lo, hi;
  yamd::shard_of(size, (uint32_t)m->lanes.size(), k, b, e);
  yamd::window_of(size, b, e, m->halo_before, m->halo_after, lo, hi);
  if (begin) *begin = b;
  if (end) *end = e;
  if (window_begin) *window_begin = lo;
  if (window_end) *window_end = hi;
  return YR_AMD_SUCCESS;
}

int yr_amd_multi_scan_block_verified(yr_amd_multi* m, const uint8_t* data, size_t size,
                                     uint64_t data_base, const yr_amd_verify_rec** records,
                                     uint64_t* count) {
  if (m == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n = (uint32_t)m->lanes.size();
  // every device's window, as yr_amd_multi_shard reports it (n = 1 too)
  for (uint32_t k = 0; k < n; ++k) {
    Lane& L = m->lanes[k];
    yamd::shard_of(size, n, k, L.begin, L.end);
    yamd::window_of(size, L.begin, L.end, m->halo_before, m->halo_after, L.lo, L.hi);
    L.active = L.begin != L.end || (size == 0 && k == n - 1);
    // a device's candidates: positions (b, e], plus 0 on the first
    if ((L.end - L.begin) + (L.begin == 0 ? 1u : 0u) > YR_AMD_VERIFY_MAX_CANDIDATES)
      return YR_AMD_INVALID_ARGUMENT;
  }
  for (Lane& L : m->lanes) {
    L.status = YR_AMD_SUCCESS;
    if (L.active) {
      const int r = yamd::lane_reserve(L);
      if (r) return r;
    }
  }
  int rc = stage_block(m, data, size);
  if (rc) return rc;
  {
    std::unique_lock<std::mutex> lk(m->mu);
    m->size = size;
    m->base = data_base;
    m->left = n;
    ++m->gen;
    m->cv.notify_all();
    m->cv.wait(lk, [&] { return m->left == 0; });
  }
  for (const Lane& L : m->lanes)
    if (L.status != YR_AMD_SUCCESS) return L.status;
  yamd::lanes_concat(m->lanes, m->out);
  if (records) *records = m->out.data();
  if (count) *count = m->out.size();
  return YR_AMD_SUCCESS;
}

}  // extern "C"
