// Multi-device block scans behind the C ABI (include/yara_amd.h
// yr_amd_multi_*).
//
// One process drives n devices: a host block is split into n byte ranges
// (equal 1 MiB-aligned slices, the last takes the rest -- the same bounds as
// yara_amd/dist.py shard_bounds), device k receives only its WINDOW of the
// block (its range plus the tables' verify halos, yr_amd_tables_get_info),
// scans it with yr_amd_scan_window and pre-verifies its own candidates with
// yr_amd_verify_device, each device on its own stream driven by its own host
// thread.  Records are block-global, so their concatenation in device order
// is exactly the single-device record stream of the whole block
// (yr_amd_scan_block_verified): the libyara side replays it into the
// unmodified yr_scan_verify_match (scanner.c:105-121) as before.  No data-path
// exchange between devices; the "gather" is the host concatenation.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <thread>
#include <vector>

#include "../../include/yara_amd.h"
#include "internal.h"

namespace {

constexpr uint64_t kShardAlign = 1u << 20;   // dist.py shard_bounds

struct Lane {
  yr_amd_tables* tables = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;
  yr_amd_scanner* scanner = nullptr;
  uint8_t* d_win = nullptr;
  size_t d_win_cap = 0;
  std::vector<yr_amd_verify_rec> recs;
  uint64_t candidates = 0;
  int status = YR_AMD_SUCCESS;
  bool last = false;   // the last device (takes the rest of the block)
};

}  // namespace

struct yr_amd_multi {
  std::vector<Lane> lanes;
  uint64_t halo_before = 0, halo_after = 0;
  std::vector<yr_amd_verify_rec> out;
};

namespace {

// [begin, end) of device k in a block of `size` bytes (dist.py shard_bounds).
void shard_of(uint64_t size, uint32_t n, uint32_t k, uint64_t& begin, uint64_t& end) {
  const uint64_t per = (size / n) / kShardAlign * kShardAlign;
  begin = (uint64_t)k * per;
  end = k == n - 1 ? size : begin + per;
}

// [lo, hi): the bytes device k holds (dist.py shard_window).
void window_of(uint64_t size, uint64_t begin, uint64_t end, uint64_t before, uint64_t after,
               uint64_t& lo, uint64_t& hi) {
  before = std::max<uint64_t>(before, YR_AMD_MAX_ATOM_LENGTH);
  lo = (begin - std::min(begin, before)) / 16 * 16;
  hi = std::min(size, end + after);
}

// One device's share of a block: H2D of its window, scan, pre-verification,
// D2H of its records.
void run_lane(Lane& L, const uint8_t* data, uint64_t size, uint64_t data_base, uint64_t begin,
              uint64_t end, uint64_t lo, uint64_t hi) {
  L.recs.clear();
  L.candidates = 0;
  L.status = YR_AMD_SUCCESS;
  // an empty range owns no position (a block smaller than one slice per
  // device: the last device takes all of it, position 0 included); only an
  // empty block is scanned, by the last device, for its position 0
  if (begin == end && !(size == 0 && L.last)) return;
  if (hipSetDevice(L.device) != hipSuccess) {
    L.status = YR_AMD_INTERNAL_FATAL_ERROR;
    return;
  }
  const uint64_t n = hi - lo;
  if (n > L.d_win_cap || L.d_win == nullptr) {
    if (L.d_win) (void)hipFree(L.d_win);
    L.d_win = nullptr;
    L.d_win_cap = 0;
    if (hipMalloc((void**)&L.d_win, std::max<uint64_t>(n, 16)) != hipSuccess) {
      L.d_win = nullptr;
      L.status = YR_AMD_INSUFFICIENT_MEMORY;
      return;
    }
    L.d_win_cap = std::max<uint64_t>(n, 16);
  }
  if (n > 0 && hipMemcpyAsync(L.d_win, data + lo, n, hipMemcpyHostToDevice, L.stream) != hipSuccess) {
    L.status = YR_AMD_COULD_NOT_MAP_FILE;   // as yr_amd_scan_block
    return;
  }
  int r = yr_amd_scan_window(L.scanner, L.d_win, lo, hi, size, begin, end);
  int all = 0;
  if (!r) r = yr_amd_scan_device_result(L.scanner, nullptr, &L.candidates, &all);
  // a root-accepting rule set: every position of (begin, end] is a candidate
  // (and position 0 on the first device)
  if (all) L.candidates = (end - begin) + (begin == 0 ? 1u : 0u);
  const yr_amd_verify_rec* d_rec = nullptr;
  uint64_t cnt = 0;
  if (!r) r = yr_amd_verify_device(L.scanner, data_base, &d_rec, &cnt);
  if (r) {
    L.status = r;
    return;
  }
  L.recs.resize(cnt);
  if (cnt > 0 &&
      (hipMemcpyAsync(L.recs.data(), d_rec, cnt * sizeof(yr_amd_verify_rec), hipMemcpyDeviceToHost,
                      L.stream) != hipSuccess ||
       hipStreamSynchronize(L.stream) != hipSuccess))
    L.status = YR_AMD_INTERNAL_FATAL_ERROR;
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
    Lane& L = m->lanes[k];
    L.tables = tables[k];
    L.device = yr_amd_tables_device(tables[k]);
    L.last = k == n - 1;
    if (L.device < 0 || hipSetDevice(L.device) != hipSuccess ||
        hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking) != hipSuccess) {
      L.stream = nullptr;
      r = YR_AMD_INTERNAL_FATAL_ERROR;
      break;
    }
    r = yr_amd_scanner_create(L.tables, L.stream, &L.scanner);
  }
  if (r != YR_AMD_SUCCESS) {
    yr_amd_multi_destroy(m);
    return r;
  }
  *multi = m;
  return YR_AMD_SUCCESS;
}

int yr_amd_multi_destroy(yr_amd_multi* m) {
  if (m == nullptr) return YR_AMD_SUCCESS;
  for (Lane& L : m->lanes) {
    if (L.stream == nullptr) continue;
    (void)hipSetDevice(L.device);
    (void)hipStreamSynchronize(L.stream);
    yr_amd_scanner_destroy(L.scanner);
    if (L.d_win) (void)hipFree(L.d_win);
    (void)hipStreamDestroy(L.stream);
  }
  delete m;
  return YR_AMD_SUCCESS;
}

int yr_amd_multi_shard(const yr_amd_multi* m, uint64_t size, uint32_t k, uint64_t* begin,
                       uint64_t* end, uint64_t* window_begin, uint64_t* window_end) {
  if (m == nullptr || k >= m->lanes.size()) return YR_AMD_INVALID_ARGUMENT;
  uint64_t b, e, lo, hi;
  shard_of(size, (uint32_t)m->lanes.size(), k, b, e);
  window_of(size, b, e, m->halo_before, m->halo_after, lo, hi);
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
  std::vector<uint64_t> b(n), e(n), lo(n), hi(n);
  for (uint32_t k = 0; k < n; ++k) {
    shard_of(size, n, k, b[k], e[k]);
    window_of(size, b[k], e[k], m->halo_before, m->halo_after, lo[k], hi[k]);
    // a device's candidates: positions (b, e], plus 0 on the first
    if ((e[k] - b[k]) + (b[k] == 0 ? 1u : 0u) > YR_AMD_VERIFY_MAX_CANDIDATES)
      return YR_AMD_INVALID_ARGUMENT;
  }
  if (n == 1) {
    run_lane(m->lanes[0], data, size, data_base, b[0], e[0], lo[0], hi[0]);
  } else {
    // one host thread per device: the H2D copies of the windows (pageable
    // memory, staged by the runtime) and the scans proceed in parallel
    std::vector<std::thread> th;
    th.reserve(n);
    for (uint32_t k = 0; k < n; ++k)
      th.emplace_back(run_lane, std::ref(m->lanes[k]), data, (uint64_t)size, data_base, b[k], e[k],
                      lo[k], hi[k]);
    for (std::thread& t : th) t.join();
  }
  size_t total = 0;
  for (const Lane& L : m->lanes) {
    if (L.status != YR_AMD_SUCCESS) return L.status;
    total += L.recs.size();
  }
  // in device order = the whole block's order; each device's candidate index
  // rebased onto the whole block's stream (mod 2^32, as a single scan's)
  m->out.resize(total);
  size_t o = 0;
  uint64_t cand_base = 0;
  for (const Lane& L : m->lanes) {
    for (size_t i = 0; i < L.recs.size(); ++i) {
      m->out[o + i] = L.recs[i];
      m->out[o + i].candidate = (uint32_t)(L.recs[i].candidate + cand_base);
    }
    o += L.recs.size();
    cand_base += L.candidates;
  }
  if (records) *records = m->out.data();
  if (count) *count = total;
  return YR_AMD_SUCCESS;
}

}  // extern "C"
