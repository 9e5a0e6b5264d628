// C ABI of the MI355X Aho-Corasick atom scanner (include/yara_amd.h).
//
// Host orchestration of one block scan (the role of libyara's
// _yr_scanner_scan_mem_block, scanner.c:45-176):
//   H2D (host blocks only) -> scan_segments_kernel -> seg_offsets_kernel
//   -> seg_scatter_kernel (all queued; one host synchronisation)
//   -> [overflow retry] -> D2H of the candidate stream.
// and the host replay of candidates into the caller's verifier in the exact
// order of scanner.c:98-122 / :144-163.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <new>
#include <vector>

#include "../../include/yara_amd.h"
#include "internal.h"
#include "tables.h"
#include "re_program.h"
#include "verify.h"

namespace yamd {
hipError_t launch_scan(const ScanParams& p, int grid, hipStream_t s, int mode, hipEvent_t t0 = nullptr,
                       hipEvent_t t1 = nullptr);
hipError_t launch_compact(const ScanParams& p, uint64_t* seg_offset, uint64_t* summary,
                          uint64_t* positions, bool scatter, hipStream_t s);
hipError_t launch_xorshift(uint8_t* buf, uint64_t n, const uint64_t* states, uint32_t n_chunks,
                           uint32_t chunk, hipStream_t s);
hipError_t configure_scan_kernel();
hipError_t launch_trace_count(const uint32_t* T, const uint8_t* data, uint64_t n_pos,
                              uint32_t* block_count, uint32_t n_blocks, hipStream_t s);
hipError_t launch_trace_write(const uint32_t* T, const uint32_t* M, const uint8_t* data,
                              uint64_t n_pos, const uint64_t* block_offset,
                              yr_amd_trace_rec* out, uint64_t cap, uint32_t n_blocks,
                              hipStream_t s);
}  // namespace yamd

namespace yamd {
// Length of a general regexp program (yr_re_exec, re.c:1693): every
// instruction reachable from offset 0 through jumps, splits and repeat
// offsets is a known opcode lying inside [0, avail); returns the end of the
// furthest one, 0 if the program is malformed.
uint32_t re_general_extent(const uint8_t* c, uint64_t avail) {
  const uint64_t lim = std::min<uint64_t>(avail, 1u << 20);
  if (lim == 0) return 0;
  std::vector<uint8_t> seen(lim, 0);
  std::vector<int64_t> work{0};
  uint64_t end = 0;
  while (!work.empty()) {
    int64_t ip = work.back();
    work.pop_back();
    while (true) {
      if (ip < 0 || (uint64_t)ip >= lim) return 0;
      if (seen[ip]) break;
      seen[ip] = 1;
      const uint8_t op = c[ip];
      const uint32_t sz = re_op_size(op);
      if (sz == 0 || (uint64_t)ip + sz > lim) return 0;
      end = std::max<uint64_t>(end, (uint64_t)ip + sz);
      if (op == kOpMatch) break;
      if (op == kOpJump) {
        ip += re_i16(c + ip + 1);
        continue;
      }
      if (op == kOpSplitA || op == kOpSplitB) work.push_back(ip + re_i16(c + ip + 2));
      if (op == kOpRepeatStartGreedy || op == kOpRepeatStartUngreedy ||
          op == kOpRepeatEndGreedy || op == kOpRepeatEndUngreedy) {
        if (re_u16(c + ip + 1) > re_u16(c + ip + 3)) return 0;   // min > max
        work.push_back(ip + re_i32(c + ip + 5));
      }
      if ((op == kOpRepeatAnyGreedy || op == kOpRepeatAnyUngreedy) &&
          re_u16(c + ip + 1) > re_u16(c + ip + 3))
        return 0;
      ip += sz;
    }
  }
  return (uint32_t)end;
}
}  // namespace yamd

using namespace yamd;

struct yr_amd_tables {
  FlatTables flat;
  int device = 0;
  uint32_t* d_filter = nullptr;
  uint32_t* d_exact = nullptr;
  int num_cus = 256;

  // on-device literal pre-verification (yr_amd_tables_set_strings)
  bool has_strings = false;
  bool profile = false;               // yr_amd_tables_set_profiling
  // per 1-byte key: the guard that decides its list in the scan (ScanParams kd_*)
  uint32_t kd_m[4] = {0, 0, 0, 0}, kd_v[4] = {0, 0, 0, 0}, kd_info[4] = {0, 0, 0, 0};
  uint32_t kd_x0[4] = {0, 0, 0, 0}, kd_x1[4] = {0, 0, 0, 0};
  uint32_t kd_n[4] = {0, 0, 0, 0}, kd_head[4] = {0, 0, 0, 0}, kd_min_pos[4] = {0, 0, 0, 0};
  uint32_t kd_bm[4] = {0, 0, 0, 0}, kd_bv[4] = {0, 0, 0, 0};   // backward guards (ScanParams)
  uint32_t kd_idx[4][4] = {}, kd_bt[4][4] = {};   // a kept key's first list entries (VerifyParams)
  bool kd_any = false;
  bool kd_guard = false;              // some key's class is guard-decided (can be dead)
  bool kd_kept = false;               // some key's class is "kept" (every call a record)
  // one class plan for every key (key_plan; ScanParams::kp_on, kc[kKcPlan..])
  uint32_t kp_on = 0, kp_info = 0, kp_m = 0, kp_v = 0, kp_t = 0;
  uint32_t max_list = 0;              // the longest match list (pool chain)
  uint32_t kx_end = 2, kx_deep = 0, kx_next = 0;   // ScanParams::kx_end / kx_deep / kx_next
  uint32_t* d_nodes = nullptr;        // accepting nodes by string (FlatTables::nodes)
  uint32_t* d_kc = nullptr;           // [kKcWords] the key class records + the plan (ScanParams::kc)
  DevPoolRec* d_pool = nullptr;       // per pool entry: link, backtrack, string, programs
  uint8_t* d_str_bytes = nullptr;
  uint8_t* d_lowercase = nullptr;
  uint8_t* d_re_code = nullptr;       // yr_amd_tables_set_re_code
  std::vector<DevPoolRec> h_pool;     // host copy of the records (set_re_code fills .re)
  std::vector<uint32_t> h_str_flags, h_pool_string;   // host copies (validation)
  uint64_t max_str_bytes = 0;     // max over strings of the bytes a comparison reads
};

struct yr_amd_scanner {
  yr_amd_tables* tables = nullptr;
  hipStream_t stream = nullptr;
  bool own_stream = false;

  uint8_t* d_block = nullptr;           // staging for host blocks
  size_t d_block_cap = 0;
  uint32_t* d_seg_count = nullptr;
  uint64_t* d_seg_offset = nullptr;
  uint32_t seg_alloc = 0;               // segments the count/offset arrays hold
  uint32_t* d_seg_out = nullptr;
  size_t seg_out_cap = 0;               // entries
  uint64_t* d_positions = nullptr;
  uint8_t* d_dead = nullptr;            // per candidate: the scan proved its calls dead
  size_t dead_cap = 0;
  uint32_t* d_live = nullptr;           // per segment, its undecided candidates (ScanParams::live)
  size_t live_cap = 0;
  uint32_t* d_live_count = nullptr;     // [seg_alloc] (ScanParams::live_count)
  uint64_t* d_live_off = nullptr;       // [seg_alloc + 1] (VerifyParams::live_off)
  uint32_t* d_seg_x = nullptr;          // beside the segment outputs (ScanParams::seg_x)
  size_t seg_x_cap = 0;
  // verified-only scans (yr_amd_scanner_set_verified_only; ScanParams::drop_dead)
  bool verified_only = false;
  uint32_t* d_seg_full = nullptr;       // [seg_alloc] each segment's full-stream length
  uint64_t* d_seg_full_offset = nullptr;   // [seg_alloc + 1]
  uint32_t* d_cand_index = nullptr;     // per output candidate: its full-stream index
  size_t cand_index_cap = 0;
  uint64_t last_full_count = 0;         // the last scan's full-stream length
  size_t positions_cap = 0;             // entries
  uint64_t* h_summary = nullptr;        // pinned, coherent: {total, max per segment}
  uint64_t* d_hsum = nullptr;           // h_summary mapped for the device: the offsets
                                        // kernel writes it directly (no copy launch)
  uint64_t* d_summary = nullptr;

  std::vector<uint64_t> h_positions;

  // yr_amd_trace_walk (debugging): the verbatim transition and match tables
  uint32_t* d_trace_T = nullptr;
  uint32_t* d_trace_M = nullptr;

  // state of the last yr_amd_scan_window / yr_amd_scan_device
  ScanParams last{};
  uint64_t win_lo = 0, win_hi = 0;      // bytes of the block present in HBM
  int last_grid = 0;
  bool last_all = false;
  bool last_empty = false;
  bool pending = false;
  uint64_t last_count = 0;

  // optional kernel timing (HIP events on the scan stream)
  bool timing = false;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr, ev_compact = nullptr;
  // recorded behind a scan's result copy: yr_amd_scan_device_result waits for
  // this scan only, so scanners sharing a stream can have the next scan queued
  hipEvent_t ev_done = nullptr;
  hipEvent_t last_done = nullptr;   // ev_done, or ev_compact when the scan was timed
  // verified-only scans: recorded behind the offsets kernels, so that
  // yr_amd_scan_device_result has the counts (host-mapped summary) while the
  // scatter still runs and pre-verification queues behind it with no gap
  hipEvent_t ev_counted = nullptr;
  hipEvent_t last_counted = nullptr;   // ev_counted for the pending scan, else null
  bool ev_valid = false;

  int diag_mode = 0;   // profiling ablation of the scan kernel (0 = product)
  // candidates per KiB a segment has needed (x 1.25), learned from the last
  // overflowing scan: later scans size the segments' output for it, so a
  // rule set with dense candidates (1-byte keys) pays the exact-offset rerun
  // once per scanner instead of on every scan
  uint32_t dense_per_kib = 0;
  uint64_t* d_seg_base = nullptr; // exact per-segment output offsets (overflow rerun)
  uint32_t* d_seg_next = nullptr; // dynamic segment counter (YAMD_SEG_KIB experiments)
  size_t seg_base_cap = 0;
  uint64_t rerun_total = 0;

  // pre-verification workspace
  uint32_t* d_vcount = nullptr;
  size_t vcount_cap = 0;
  uint32_t* d_vkeep = nullptr;    // pre-verification keep masks + states (2 x count)
  size_t vkeep_cap = 0;
  uint64_t* d_vblock = nullptr;   // per-group (64 candidates) record counts -> offsets
  uint64_t* d_vchunk = nullptr;   // per-chunk (1024 groups) offsets
  size_t vchunk_cap = 0;
  size_t vblock_cap = 0;
  VerifyRec* d_vrec = nullptr;
  size_t vrec_cap = 0;
  std::vector<yr_amd_verify_rec> h_vrec;
};

static_assert(sizeof(VerifyRec) == sizeof(yr_amd_verify_rec), "record layout");

// Debug output, the analogue of libyara's YR_DEBUG_VERBOSITY (globals.h:51-90):
// the same environment variable; at level >= 2 the host replay prints every
// candidate's state and match-table entry as the reference walk does at
// scanner.c:83-96, and pre-verification prints its records.
static int debug_level() {
  static int level = -1;
  if (level < 0) {
    const char* e = getenv("YR_DEBUG_VERBOSITY");
    level = e ? atoi(e) : 0;
  }
  return level;
}


#define HIP_TRY(expr)                                   \
  do {                                                  \
    if ((expr) != hipSuccess) return YR_AMD_INTERNAL_FATAL_ERROR; \
  } while (0)

namespace {

template <typename T>
int grow(T*& p, size_t& cap, size_t need) {
  if (need <= cap && p != nullptr) return YR_AMD_SUCCESS;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  size_t n = std::max<size_t>(need, 1);
  if (hipMalloc((void**)&p, n * sizeof(T)) != hipSuccess) {
    p = nullptr;
    return YR_AMD_INSUFFICIENT_MEMORY;
  }
  cap = n;
  return YR_AMD_SUCCESS;
}

int ensure_segments(yr_amd_scanner* s, uint32_t n_segments, uint32_t seg_cap) {
  if (n_segments > s->seg_alloc) {
    size_t c = 0;
    for (void* q : {(void*)s->d_seg_count, (void*)s->d_seg_offset, (void*)s->d_seg_full,
                    (void*)s->d_seg_full_offset, (void*)s->d_live_count, (void*)s->d_live_off})
      if (q) (void)hipFree(q);
    s->d_live_count = nullptr;
    s->d_live_off = nullptr;
    s->d_seg_count = nullptr;
    s->d_seg_offset = nullptr;
    s->d_seg_full = nullptr;
    s->d_seg_full_offset = nullptr;
    s->seg_alloc = 0;
    if (grow(s->d_seg_count, c, n_segments)) return YR_AMD_INSUFFICIENT_MEMORY;
    // (+1: the offsets kernel stores the total behind the offsets)
    c = 0;
    if (grow(s->d_seg_offset, c, (size_t)n_segments + 1)) return YR_AMD_INSUFFICIENT_MEMORY;
    c = 0;
    if (grow(s->d_seg_full, c, n_segments)) return YR_AMD_INSUFFICIENT_MEMORY;
    c = 0;
    if (grow(s->d_seg_full_offset, c, (size_t)n_segments + 1)) return YR_AMD_INSUFFICIENT_MEMORY;
    c = 0;
    if (grow(s->d_live_count, c, n_segments)) return YR_AMD_INSUFFICIENT_MEMORY;
    c = 0;
    if (grow(s->d_live_off, c, (size_t)n_segments + 1)) return YR_AMD_INSUFFICIENT_MEMORY;
    s->seg_alloc = n_segments;
  }
  return grow(s->d_seg_out, s->seg_out_cap, (size_t)n_segments * seg_cap);
}

uint32_t choose_seg_bytes(uint64_t nbytes, int num_cus, uint32_t target) {
  // k segments of at most `target` bytes per wave of a full-chip launch (the
  // same k for every wave: waves take segments round-robin), 4+ tiles each.
  // (One 1 MiB segment per wave for a 4 GiB block.  128 KiB segments, 8 per
  // wave, measured 3-4 % faster in back-to-back kernel timings but 1-2 %
  // slower in the bench's pipelined steps, profiles/r02_segment_size.json.)
  const uint64_t waves = (uint64_t)num_cus * kWavesPerWG;
  const uint64_t k = std::max<uint64_t>(1, (nbytes + waves * target - 1) / (waves * target));
  uint64_t per = (nbytes + waves * k - 1) / (waves * k);
  per = (per + kTile - 1) / kTile * kTile;
  return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(per, 4 * kTile), kSegment);
}

int run_scan(yr_amd_scanner* s) {
  // scan, per-segment offsets and the scatter are queued back to back: the
  // output is sized for the clipped worst case (every segment at capacity),
  // so the host synchronises once, in yr_amd_scan_device_result
  const ScanParams& p = s->last;
  const size_t out_cap = p.seg_base ? s->rerun_total : (size_t)p.n_segments * p.seg_cap;
  int r = grow(s->d_positions, s->positions_cap, out_cap);
  if (!r && s->tables->kd_any) r = grow(s->d_dead, s->dead_cap, out_cap);
  if (!r && s->tables->kd_any) r = grow(s->d_live, s->live_cap, out_cap);
  if (!r && s->tables->kd_any) r = grow(s->d_seg_x, s->seg_x_cap, out_cap);
  if (!r && p.drop_dead) r = grow(s->d_cand_index, s->cand_index_cap, out_cap);
  if (r) return r;
  s->last.dead = s->tables->kd_any ? s->d_dead : nullptr;
  s->last.live = s->tables->kd_any ? s->d_live : nullptr;
  s->last.live_count = s->tables->kd_any ? s->d_live_count : nullptr;
  s->last.seg_x = s->tables->kd_any ? s->d_seg_x : nullptr;
  s->last.seg_full = p.drop_dead ? s->d_seg_full : nullptr;
  s->last.seg_full_offset = p.drop_dead ? s->d_seg_full_offset : nullptr;
  s->last.cand_index = p.drop_dead ? s->d_cand_index : nullptr;
  // (timing: the kernel's own start / end stamps -- not two markers around
  // the launch, which would also count its dispatch)
  if (s->timing) {
    HIP_TRY(launch_scan(p, s->last_grid, s->stream, s->diag_mode, s->ev_begin, s->ev_end));
    s->ev_valid = true;
  } else {
    HIP_TRY(launch_scan(p, s->last_grid, s->stream, s->diag_mode));
  }
  HIP_TRY(launch_compact(p, s->d_seg_offset, s->d_hsum, nullptr, false, s->stream));
  s->last_counted = nullptr;
  if (s->verified_only) {
    HIP_TRY(hipEventRecord(s->ev_counted, s->stream));
    s->last_counted = s->ev_counted;
  }
  HIP_TRY(launch_compact(p, s->d_seg_offset, s->d_hsum, s->d_positions, true, s->stream));
  // one event marks the end of the scan's work: the timed one when timing (a
  // second event record at the same point would add a ~5 us gap per scan on
  // the stream, profiles/r03_step_gaps.json)
  s->last_done = s->timing ? s->ev_compact : s->ev_done;
  HIP_TRY(hipEventRecord(s->last_done, s->stream));
  return YR_AMD_SUCCESS;
}

}  // namespace

extern "C" {

const char* yr_amd_version(void) { return "yara_amd 0.1.0 (gfx950)"; }

int yr_amd_tables_create(const uint32_t* transition_table, const uint32_t* match_table,
                         uint32_t n_slots, const uint32_t* pool_next,
                         const uint16_t* pool_backtrack, uint32_t n_pool, int device,
                         yr_amd_tables** tables) {
  if (tables == nullptr) return YR_AMD_INVALID_ARGUMENT;
  *tables = nullptr;
  yr_amd_tables* t = new (std::nothrow) yr_amd_tables();
  if (t == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
  int r = flatten_tables(transition_table, match_table, n_slots, pool_next, pool_backtrack, n_pool,
                         t->flat);
  if (r != YR_AMD_SUCCESS) {
    delete t;
    return r;
  }
  t->device = device;
  if (device < 0) {  // host-only: flattening + replay
    *tables = t;
    return YR_AMD_SUCCESS;
  }
  if (hipSetDevice(device) != hipSuccess ||
      hipDeviceGetAttribute(&t->num_cus, hipDeviceAttributeMultiprocessorCount, device) !=
          hipSuccess ||
      configure_scan_kernel() != hipSuccess ||
      hipMalloc((void**)&t->d_filter, t->flat.filter.size() * 4) != hipSuccess ||
      hipMalloc((void**)&t->d_exact, t->flat.exact.size() * 4) != hipSuccess ||
      hipMemcpy(t->d_filter, t->flat.filter.data(), t->flat.filter.size() * 4,
                hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(t->d_exact, t->flat.exact.data(), t->flat.exact.size() * 4,
                hipMemcpyHostToDevice) != hipSuccess) {
    yr_amd_tables_destroy(t);
    return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  *tables = t;
  return YR_AMD_SUCCESS;
}

int yr_amd_tables_destroy(yr_amd_tables* t) {
  if (t == nullptr) return YR_AMD_SUCCESS;
  for (void* p : {(void*)t->d_filter, (void*)t->d_exact, (void*)t->d_nodes, (void*)t->d_kc, (void*)t->d_pool,
                  (void*)t->d_str_bytes, (void*)t->d_lowercase, (void*)t->d_re_code})
    if (p) (void)hipFree(p);
  delete t;
  return YR_AMD_SUCCESS;
}

int yr_amd_tables_device(const yr_amd_tables* t) { return t == nullptr ? -1 : t->device; }

int yr_amd_tables_set_profiling(yr_amd_tables* t, int enable) {
  if (t == nullptr) return YR_AMD_INVALID_ARGUMENT;
  t->profile = enable != 0;
  return YR_AMD_SUCCESS;
}

int yr_amd_tables_get_info(const yr_amd_tables* t, yr_amd_tables_info* info) {
  if (t == nullptr || info == nullptr) return YR_AMD_INVALID_ARGUMENT;
  memset(info, 0, sizeof(*info));
  const FlatTables& f = t->flat;
  info->n_slots = f.n_slots;
  info->n_states = f.n_states;
  info->max_depth = f.max_depth;
  for (int d = 0; d <= YR_AMD_MAX_ATOM_LENGTH; ++d) {
    info->states_by_depth[d] = f.by_depth[d];
    info->keys_by_length[d] = f.keys_by_len[d];
  }
  info->accepting_states = f.accepting;
  info->root_accepting = f.root_accepting ? 1 : 0;
  info->filter_bits = kFilterLog2Bits;
  info->filter_set_bits = f.filter_set_bits;
  info->filter_mode = f.filter_mode;
  info->exact_slots = 4 * (f.t3_mask + 1 + f.t4_mask + 1);
  uint32_t mb = 0;
  for (uint16_t b : f.pool_backtrack) mb = std::max<uint32_t>(mb, b);
  info->max_backtrack = mb;
  // a shard's verify window (yr_amd_scan_window + yr_amd_verify_device):
  // candidates i in (begin, end] make calls at offsets >= begin + 1 - max
  // backtrack whose reads reach YR_RE_SCAN_LIMIT further back, and at offsets
  // <= end whose reads reach max(YR_RE_SCAN_LIMIT, 2 * string length) forward
  // (verify.hip call_matters); without strings only the 4-byte warm-up
  info->verify_halo_before = t->has_strings ? mb + (uint64_t)kReScanLimit : YR_AMD_MAX_ATOM_LENGTH;
  info->verify_halo_after =
      t->has_strings ? std::max<uint64_t>((uint64_t)kReScanLimit, t->max_str_bytes) : 0;
  return YR_AMD_SUCCESS;
}

int yr_amd_scanner_create(yr_amd_tables* tables, void* stream, yr_amd_scanner** scanner) {
  if (tables == nullptr || scanner == nullptr || tables->device < 0) return YR_AMD_INVALID_ARGUMENT;
  *scanner = nullptr;
  yr_amd_scanner* s = new (std::nothrow) yr_amd_scanner();
  if (s == nullptr) return YR_AMD_INSUFFICIENT_MEMORY;
  s->tables = tables;
  if (hipSetDevice(tables->device) != hipSuccess) {
    delete s;
    return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  if (stream != nullptr) {
    s->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
      delete s;
      return YR_AMD_INTERNAL_FATAL_ERROR;
    }
    s->own_stream = true;
  }
  // {total, max per segment, full-stream total, max} (ScanParams::drop_dead)
  if (hipHostMalloc((void**)&s->h_summary, 4 * sizeof(uint64_t), hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&s->d_hsum, s->h_summary, 0) != hipSuccess ||
      hipMalloc((void**)&s->d_summary, 2 * sizeof(uint64_t)) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_counted, hipEventDisableTiming) != hipSuccess) {
    yr_amd_scanner_destroy(s);
    return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  *scanner = s;
  return YR_AMD_SUCCESS;
}

int yr_amd_scanner_destroy(yr_amd_scanner* s) {
  if (s == nullptr) return YR_AMD_SUCCESS;
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (void* p : {(void*)s->d_block, (void*)s->d_seg_count,
                  (void*)s->d_seg_offset,
                  (void*)s->d_seg_out, (void*)s->d_positions, (void*)s->d_dead, (void*)s->d_live,
                  (void*)s->d_seg_x, (void*)s->d_seg_full, (void*)s->d_seg_full_offset,
                  (void*)s->d_cand_index, (void*)s->d_live_count, (void*)s->d_live_off,
                  (void*)s->d_summary,
                  (void*)s->d_vcount, (void*)s->d_vkeep, (void*)s->d_vblock, (void*)s->d_vrec,
                  (void*)s->d_vchunk, (void*)s->d_seg_base,
                  (void*)s->d_seg_next, (void*)s->d_trace_T, (void*)s->d_trace_M})
    if (p) (void)hipFree(p);
  if (s->h_summary) (void)hipHostFree(s->h_summary);
  if (s->ev_begin) (void)hipEventDestroy(s->ev_begin);
  if (s->ev_end) (void)hipEventDestroy(s->ev_end);
  if (s->ev_compact) (void)hipEventDestroy(s->ev_compact);
  if (s->ev_done) (void)hipEventDestroy(s->ev_done);
  if (s->ev_counted) (void)hipEventDestroy(s->ev_counted);
  if (s->own_stream && s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
  return YR_AMD_SUCCESS;
}

int yr_amd_scanner_set_verified_only(yr_amd_scanner* s, int enable) {
  if (s == nullptr) return YR_AMD_INVALID_ARGUMENT;
  s->verified_only = enable != 0;
  return YR_AMD_SUCCESS;
}

int yr_amd_scan_device_stream_length(yr_amd_scanner* s, uint64_t* length) {
  if (s == nullptr || length == nullptr || s->pending) return YR_AMD_INVALID_ARGUMENT;
  *length = s->last_full_count;
  return YR_AMD_SUCCESS;
}

int yr_amd_scanner_set_timing(yr_amd_scanner* s, int enable) {
  if (s == nullptr) return YR_AMD_INVALID_ARGUMENT;
  if (enable && s->ev_begin == nullptr) {
    HIP_TRY(hipSetDevice(s->tables->device));
    // the kernel's begin/end markers only time it: no system-scope fence (a
    // cache writeback + invalidate at each record, ~5 us of stream gap per
    // marker, profiles/r03_step_gaps.json); ev_compact also completes the scan
    // for the host (last_done) and keeps it
    // (timing markers without a system-scope fence)
    const unsigned marker = hipEventDisableSystemFence;
    HIP_TRY(hipEventCreateWithFlags(&s->ev_begin, marker));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_end, marker));
    HIP_TRY(hipEventCreate(&s->ev_compact));
  }
  s->timing = enable != 0;
  s->ev_valid = false;
  return YR_AMD_SUCCESS;
}

#if YAMD_DIAG
// Diagnostic builds only (not declared in include/yara_amd.h): profiling
// ablations of the scan kernel (tools/ablate.py).  Any mode other than 0
// produces wrong results.
// Candidates of the last scan that the drain proved dead (ScanParams::dead).
int64_t yr_amd__diag_dead_count(yr_amd_scanner* s) {
  if (s == nullptr || s->last.dead == nullptr || s->last_count == 0) return -1;
  std::vector<uint8_t> h(s->last_count);
  if (hipMemcpy(h.data(), s->last.dead, h.size(), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  int64_t n = 0;
  for (uint8_t x : h) n += x != 0;
  return n;
}

// The key classes of a table (key_classes), out[40]: out[0] = kx_end, [1] = the
// 1-byte keys, [2] = their count, [3..6] = kd_info, [7..10] = kd_m, [11..14] = kd_v.
int yr_amd__diag_key_classes(const yr_amd_tables* t, uint32_t* out) {
  if (t == nullptr || out == nullptr) return YR_AMD_INVALID_ARGUMENT;
  out[0] = t->kx_end;
  out[1] = t->flat.byte_keys;
  out[2] = t->flat.n_byte_keys;
  for (int k = 0; k < 4; ++k) out[3 + k] = t->kd_info[k], out[7 + k] = t->kd_m[k], out[11 + k] = t->kd_v[k];
  // [15..18] kd_x0, [19..22] kd_x1, [23..26] kd_min_pos, [27] kx_deep, [28] kx_next
  for (int k = 0; k < 4; ++k) out[15 + k] = t->kd_x0[k], out[19 + k] = t->kd_x1[k], out[23 + k] = t->kd_min_pos[k];
  out[27] = t->kx_deep;
  out[28] = t->kx_next;
  // [29] the one-plan drop instance (key_plan), [30] / [31] its forward tests
  out[29] = t->kp_on;
  out[30] = t->kp_m;
  out[31] = t->kp_v;
  // [32..35] kd_bm, [36..39] kd_bv
  for (int k = 0; k < 4; ++k) out[32 + k] = t->kd_bm[k], out[36 + k] = t->kd_bv[k];
  return YR_AMD_SUCCESS;
}

int yr_amd__diag_kernel_mode(yr_amd_scanner* s, int mode) {
  if (s == nullptr || mode < 0 || (mode > 13 && mode != 24 && mode != 25 && (mode < 101 || mode > 104)))
    return YR_AMD_INVALID_ARGUMENT;
  s->diag_mode = mode;
  return YR_AMD_SUCCESS;
}
#endif

int yr_amd_scanner_kernel_ms(yr_amd_scanner* s, float* ms) {
  if (s == nullptr || ms == nullptr || !s->ev_valid) return YR_AMD_INVALID_ARGUMENT;
  HIP_TRY(hipEventSynchronize(s->ev_end));
  HIP_TRY(hipEventElapsedTime(ms, s->ev_begin, s->ev_end));
  return YR_AMD_SUCCESS;
}

int yr_amd_scanner_scan_ms(yr_amd_scanner* s, float* ms) {
  if (s == nullptr || ms == nullptr || !s->ev_valid) return YR_AMD_INVALID_ARGUMENT;
  HIP_TRY(hipEventSynchronize(s->ev_compact));
  HIP_TRY(hipEventElapsedTime(ms, s->ev_begin, s->ev_compact));
  return YR_AMD_SUCCESS;
}

int yr_amd_scan_device(yr_amd_scanner* s, const uint8_t* d_data, uint64_t block_size,
                       uint64_t byte_begin, uint64_t byte_end) {
  return yr_amd_scan_window(s, d_data, 0, block_size, block_size, byte_begin, byte_end);
}

int yr_amd_scan_window(yr_amd_scanner* s, const uint8_t* d_window, uint64_t window_begin,
                       uint64_t window_end, uint64_t block_size, uint64_t byte_begin,
                       uint64_t byte_end) {
  if (s == nullptr || byte_begin > byte_end || byte_end > window_end ||
      window_begin > window_end || window_end > block_size)
    return YR_AMD_INVALID_ARGUMENT;
  // the 4-byte warm-up before byte_begin must be in the window
  if (byte_begin - std::min<uint64_t>(byte_begin, YR_AMD_MAX_ATOM_LENGTH) < window_begin)
    return YR_AMD_INVALID_ARGUMENT;
  if ((byte_begin & 15) != 0 || (window_begin & 15) != 0 || (((uintptr_t)d_window) & 15) != 0)
    return YR_AMD_INVALID_ARGUMENT;
  const yr_amd_tables* t = s->tables;
  s->pending = true;
  s->last_count = 0;
  s->last_full_count = 0;
  s->ev_valid = false;
  s->win_lo = window_begin;
  s->win_hi = window_end;
  // the kernels address the block by its own positions: position p of the
  // block is d_window[p - window_begin] (only [window_begin, window_end) is
  // ever read, kernels.hip scan_segment / verify.hip call_matters)
  const uint8_t* d_data =
      d_window == nullptr ? nullptr : (const uint8_t*)((uintptr_t)d_window - (uintptr_t)window_begin);
  s->last.data = d_data;
  s->last.block_size = block_size;
  s->last.byte_begin = byte_begin;
  s->last.byte_end = byte_end;
  s->last_all = t->flat.root_accepting;
  s->last_empty = s->last_all || byte_end == byte_begin;
  s->last.dead = nullptr;
  s->last.live = nullptr;
  s->last.live_count = nullptr;
  s->last.seg_x = nullptr;
  s->last.drop_dead = 0;
  s->last.seg_full = nullptr;
  s->last.seg_full_offset = nullptr;
  s->last.cand_index = nullptr;
  if (s->last_empty) return YR_AMD_SUCCESS;
  if (d_window == nullptr) return YR_AMD_INVALID_ARGUMENT;
  HIP_TRY(hipSetDevice(t->device));

  const uint64_t nbytes = byte_end - byte_begin;
  // YAMD_SEG_KIB=<k>: segment target k KiB instead of kSegmentTarget, and with
  // YAMD_SEG_DYNAMIC set, segments after a wave's first are claimed from a
  // counter (scan_segments_kernel's seg_next) -- diagnostic builds only
  static const uint32_t seg_target = [] {
    const char* e = diag_env("YAMD_SEG_KIB");
    const uint32_t k = e ? (uint32_t)atoi(e) : 0u;
    return k >= 4 && k * 1024u <= kSegment ? k * 1024u : kSegmentTarget;
  }();
  static const bool dynamic = diag_env("YAMD_SEG_DYNAMIC") != nullptr;
  const uint32_t seg_bytes = choose_seg_bytes(nbytes, t->num_cus, seg_target);
  const uint64_t n_segments64 = (nbytes + seg_bytes - 1) / seg_bytes;
  if (n_segments64 > 0xFFFFFFFFull) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n_segments = (uint32_t)n_segments64;
  const uint32_t learned = (uint32_t)std::min<uint64_t>(
      (uint64_t)s->dense_per_kib * seg_bytes / 1024, seg_bytes / 64);   // (bounded workspace)
  const uint32_t seg_cap = std::max<uint32_t>(std::max<uint32_t>(64, seg_bytes / 256), learned);
  int r = ensure_segments(s, n_segments, seg_cap);
  if (r) return r;

  ScanParams& p = s->last;
  p.data = d_data;
  p.block_size = block_size;
  p.byte_begin = byte_begin;
  p.byte_end = byte_end;
  p.filter = t->d_filter;
  p.exact = t->d_exact;
  p.t3_off = t->flat.t3_off;
  p.t3_mask = t->flat.t3_mask;
  p.t4_off = t->flat.t4_off;
  p.t4_mask = t->flat.t4_mask;
  p.exact_flags = t->flat.exact_flags;
  p.len_mask = t->flat.len_mask;
  p.byte_keys = t->flat.byte_keys;
  p.n_byte_keys = t->flat.n_byte_keys;
  p.pair_keys[0] = t->flat.pair_keys[0];
  p.pair_keys[1] = t->flat.pair_keys[1];
  p.n_pair_keys = t->flat.n_pair_keys;
  p.kx_end = t->kx_end;
  p.kx_deep = t->kx_deep;
  p.kx_next = t->kx_next;
  for (int k = 0; k < 4; ++k) {
    p.kd_m[k] = t->kd_m[k];
    p.kd_v[k] = t->kd_v[k];
    p.kd_info[k] = t->kd_info[k];
    p.kd_x0[k] = t->kd_x0[k];
    p.kd_x1[k] = t->kd_x1[k];
    p.kd_n[k] = t->kd_n[k];
    p.kd_head[k] = t->kd_head[k];
    p.kd_min_pos[k] = t->kd_min_pos[k];
  }
  p.kd_bguard = ((t->kd_info[0] | t->kd_info[1] | t->kd_info[2] | t->kd_info[3]) & 8u) ? 1u : 0u;
  p.kp_on = t->kp_on;
  p.filter_mode = t->flat.filter_mode;
  // verified-only: the byte-key kernel decides the certain candidates' classes
  // and leaves the dead ones out (kd_any: 1-byte keys with classes; never with
  // profiling, whose count-only records need every call)
  p.drop_dead = s->verified_only && t->kd_guard && !t->profile && t->flat.n_byte_keys != 0 ? 1u : 0u;
  p.kc = t->d_kc;
  p.n_segments = n_segments;
  p.seg_bytes = seg_bytes;
  p.seg_cap = seg_cap;
  p.seg_count = s->d_seg_count;
  p.seg_out = s->d_seg_out;
  p.seg_base = nullptr;
  s->last_grid = (int)std::min<uint64_t>((n_segments + kWavesPerWG - 1) / kWavesPerWG,
                                         (uint64_t)t->num_cus);
  p.seg_next = nullptr;
  if (dynamic) {
    if (s->d_seg_next == nullptr) HIP_TRY(hipMalloc(&s->d_seg_next, sizeof(uint32_t)));
    p.seg_next = s->d_seg_next;
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)s->d_seg_next,
                              (int)((uint32_t)s->last_grid * kWavesPerWG), 1, s->stream));
  }
  return run_scan(s);
}

int yr_amd_scan_device_result(yr_amd_scanner* s, const uint64_t** d_positions, uint64_t* count,
                              int* all_positions) {
  if (s == nullptr || !s->pending) return YR_AMD_INVALID_ARGUMENT;
  if (all_positions) *all_positions = s->last_all ? 1 : 0;
  if (s->last_empty) {
    s->pending = false;
    if (d_positions) *d_positions = s->d_positions;
    if (count) *count = 0;
    return YR_AMD_SUCCESS;
  }
  // (verified-only: the counts are final once the offsets kernels ran; the
  // scatter's positions, classes and live lists follow in stream order)
  HIP_TRY(hipEventSynchronize(s->last_counted ? s->last_counted
                                              : (s->last_done ? s->last_done : s->ev_done)));
  uint64_t total = s->h_summary[0];
  const uint64_t maxc = s->h_summary[1];
  static const bool no_learn = diag_env("YAMD_NO_CAP_LEARN") != nullptr;   // A/B only
  if (maxc > s->last.seg_cap && !no_learn) {
    s->dense_per_kib = std::max<uint32_t>(
        s->dense_per_kib, (uint32_t)std::min<uint64_t>((maxc * 1280 + s->last.seg_bytes - 1) /
                                                           s->last.seg_bytes, 1u << 20));
  }
  if (maxc > s->last.seg_cap) {
    // some segment overflowed its capacity: rerun once with every segment
    // writing at its exact offset (counts are kept past the capacity), so the
    // workspace is exactly the candidate count however skewed the segments
    ScanParams exact = s->last;
    exact.seg_cap = 0xFFFFFFFFu;
    HIP_TRY(launch_compact(exact, s->d_seg_offset, s->d_hsum, nullptr, false, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    total = s->h_summary[0];
    int r = grow(s->d_seg_out, s->seg_out_cap, std::max<uint64_t>(total, 1));
    if (!r) r = grow(s->d_seg_base, s->seg_base_cap, s->last.n_segments);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(s->d_seg_base, s->d_seg_offset, s->last.n_segments * sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, s->stream));
    s->last.seg_out = s->d_seg_out;
    s->last.seg_base = s->d_seg_base;
    s->last.seg_cap = 0xFFFFFFFFu;
    s->rerun_total = std::max<uint64_t>(total, 1);
    r = run_scan(s);
    if (r) return r;
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (s->h_summary[0] != total) return YR_AMD_INTERNAL_FATAL_ERROR;
  }
  s->last_count = total;
  s->last_full_count = s->last.drop_dead ? s->h_summary[2] : total;
  s->pending = false;
  if (d_positions) *d_positions = s->d_positions;
  if (count) *count = total;
  return YR_AMD_SUCCESS;
}

int yr_amd_scan_block(yr_amd_scanner* s, const uint8_t* data, size_t size,
                      const uint64_t** positions, uint64_t* count, int* all_positions) {
  if (s == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  HIP_TRY(hipSetDevice(s->tables->device));
  if (size > 0) {
    int r = grow(s->d_block, s->d_block_cap, size);
    if (r) return r;
    if (hipMemcpyAsync(s->d_block, data, size, hipMemcpyHostToDevice, s->stream) != hipSuccess)
      return YR_AMD_COULD_NOT_MAP_FILE;
  }
  int r = yr_amd_scan_device(s, s->d_block, size, 0, size);
  if (r) return r;
  const uint64_t* d_pos = nullptr;
  uint64_t n = 0;
  int all = 0;
  r = yr_amd_scan_device_result(s, &d_pos, &n, &all);
  if (r) return r;
  s->h_positions.resize(n);
  if (n > 0) {
    HIP_TRY(hipMemcpyAsync(s->h_positions.data(), d_pos, n * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
  }
  if (positions) *positions = s->h_positions.data();
  if (count) *count = n;
  if (all_positions) *all_positions = all;
  return YR_AMD_SUCCESS;
}

extern "C++" {
namespace {
template <typename T>
int upload(T*& d, const T* h, size_t n) {
  if (hipMalloc((void**)&d, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
    d = nullptr;
    return YR_AMD_INSUFFICIENT_MEMORY;
  }
  if (n > 0 && hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
    return YR_AMD_INTERNAL_FATAL_ERROR;
  return YR_AMD_SUCCESS;
}
}  // namespace
}  // extern "C++"

extern "C++" {   // (internal helpers: C++ linkage, not exported)
namespace {
void key_classes(yr_amd_tables* t);
}  // namespace
}  // extern "C++"

int yr_amd_tables_set_strings(yr_amd_tables* t, const uint32_t* pool_string, uint32_t n_pool,
                              const yr_amd_string* strings, uint32_t n_strings,
                              const uint8_t* bytes, uint64_t n_bytes, const uint8_t* lowercase) {
  if (t == nullptr || lowercase == nullptr || t->has_strings) return YR_AMD_INVALID_ARGUMENT;
  if (n_pool != t->flat.pool_next.size()) return YR_AMD_INVALID_ARGUMENT;
  if ((n_pool > 0 && pool_string == nullptr) || (n_strings > 0 && strings == nullptr) ||
      (n_bytes > 0 && bytes == nullptr))
    return YR_AMD_INVALID_ARGUMENT;
  for (uint32_t k = 0; k < n_pool; ++k)
    if (pool_string[k] >= n_strings) return YR_AMD_INVALID_ARGUMENT;
  for (uint32_t k = 0; k < n_strings; ++k) {
    const yr_amd_string& x = strings[k];
    if (x.bytes_offset > n_bytes || x.length > n_bytes - x.bytes_offset)
      return YR_AMD_INVALID_ARGUMENT;
  }
  if (t->device < 0) return YR_AMD_INVALID_ARGUMENT;   // device feature
  const FlatTables& f = t->flat;
  // one record per pool entry with its string's fields (verify.h DevPoolRec)
  t->h_pool.assign(n_pool, DevPoolRec{});
  for (uint32_t k = 0; k < n_pool; ++k) {
    const yr_amd_string& x = strings[pool_string[k]];
    DevPoolRec& e = t->h_pool[k];
    e.next = f.pool_next[k];
    e.backtrack = f.pool_backtrack[k];
    e.flags = x.flags & ~kPoolFwdFiberSafe;   // (that bit is the device's own)
    e.length = x.length;
    e.fixed_offset = x.fixed_offset;
    e.bytes_off = x.bytes_offset;
    e.re = DevRe{0, 0, 0, 0};
  }
  HIP_TRY(hipSetDevice(t->device));
  int r = YR_AMD_SUCCESS;
  if (!r) r = upload(t->d_nodes, f.nodes.data(), f.nodes.size());
  if (!r) r = upload(t->d_pool, t->h_pool.data(), t->h_pool.size());
  {
    // 64 bytes of padding: verify.hip stage_str reads three aligned 16-byte
    // chunks from a string's start (one 16-byte chunk below it at most)
    std::vector<uint8_t> padded((size_t)n_bytes + 64, 0);
    if (n_bytes > 0) memcpy(padded.data(), bytes, (size_t)n_bytes);
    if (!r) r = upload(t->d_str_bytes, padded.data(), padded.size());
  }
  if (!r) r = upload(t->d_lowercase, lowercase, 256);
  if (r) return r;   // partial uploads are freed with the tables
  t->h_pool_string.assign(pool_string, pool_string + n_pool);
  t->h_str_flags.resize(n_strings);
  for (uint32_t k = 0; k < n_strings; ++k) {
    t->h_str_flags[k] = strings[k].flags;
    // a wide literal compares 2 * length bytes; its FULL_WORD test reads the
    // two after them (scan.c:680-682, verify.hip call_matters)
    t->max_str_bytes = std::max<uint64_t>(t->max_str_bytes, 2ull * strings[k].length + 2);
  }
  t->has_strings = true;
  key_classes(t);   // (again with the guards once regexp programs are attached)
  return YR_AMD_SUCCESS;
}

extern "C++" {   // (internal helpers: C++ linkage, not exported)
namespace {
// Length of a linear fast-exec program (opcodes of yr_re_fast_exec,
// re.c:2150-2391) that ends with MATCH exactly at `len`, else 0.
uint32_t fast_program_ok(const uint8_t* c, uint32_t len) {
  uint32_t n = 0;
  while (n < len) {
    switch (c[n]) {
      case kReAny: n += 1; break;
      case kReLiteral: case kReNotLiteral: n += 2; break;
      case kReMaskedLiteral: case kReMaskedNotLiteral: n += 3; break;
      case kReRepeatAnyUngreedy: {
        if (n + 5 > len) return 0;
        const uint32_t mn = c[n + 1] | (c[n + 2] << 8), mx = c[n + 3] | (c[n + 4] << 8);
        if (mn > mx) return 0;
        n += 5;
        break;
      }
      case kReMatch: return n + 1 == len ? len : 0;
      default: return 0;
    }
  }
  return 0;
}

struct GuardPos { uint8_t m, v; };   // one consumed position: (mask, value), m = 0 untested

// The guard (verify.h DevGuard) from a program's consumed positions: `head` =
// the positions from its start at fixed distances, `tail` = those right after a
// REPEAT_ANY {mn, mx} that follows `head` (repeat), the 4 positions with the
// most tested bits, ignoring the first `skip` (the atom's bytes, which every
// candidate has).  false when nothing would be tested.
bool pick_guard(const std::vector<GuardPos>& head, const std::vector<GuardPos>& tail, bool repeat,
                uint32_t mn, uint32_t mx, uint32_t skip, bool backwards, DevGuard& g, uint8_t& bs) {
  auto bits = [](const std::vector<GuardPos>& r, uint32_t s, uint32_t from) {
    uint32_t b = 0;
    for (uint32_t t = 0; t < 4 && s + t < r.size(); ++t)
      if (s + t >= from) b += (uint32_t)__builtin_popcount(r[s + t].m);
    return b;
  };
  uint32_t best = 0, base = 0, span = 0;
  const std::vector<GuardPos>* src = nullptr;
  uint32_t src_at = 0;
  for (uint32_t s0 = 0; s0 < std::max<size_t>(head.size(), 1) && s0 <= 15; ++s0) {
    const uint32_t b = bits(head, s0, skip);
    if (b > best) { best = b; base = s0; span = 0; src = &head; src_at = s0; }
  }
  if (repeat && head.size() + mn <= 15 && mx - mn <= 8) {
    const uint32_t b = bits(tail, 0, 0);
    if (b > best) { best = b; base = (uint32_t)head.size() + mn; span = mx - mn; src = &tail; src_at = 0; }
  }
  if (best == 0) return false;
  g = DevGuard{0u, 0u};
  for (uint32_t t = 0; t < 4 && src_at + t < src->size(); ++t) {
    const GuardPos q = (*src)[src_at + t];
    const uint32_t sh = 8 * (backwards ? 3 - t : t);
    g.m |= (uint32_t)q.m << sh;
    g.v |= (uint32_t)(q.m ? q.v : 0) << sh;
  }
  bs = (uint8_t)(base | span << 4);
  return true;
}

// The guard of a linear fast-exec program (yr_re_fast_exec, re.c:2150-2391):
// its run of literal / masked / any opcodes from the start, and the run right
// after its first REPEAT_ANY.
bool fast_guard(const uint8_t* c, uint32_t len, uint32_t skip, bool backwards, DevGuard& g,
                uint8_t& bs) {
  std::vector<GuardPos> head, tail;
  uint32_t mn = 0, mx = 0;
  bool repeat = false;
  for (uint32_t n = 0; n < len;) {
    const uint8_t op = c[n];
    std::vector<GuardPos>& run = repeat ? tail : head;
    if (op == kReMatch) break;
    if (op == kReRepeatAnyUngreedy) {
      if (repeat) break;
      mn = c[n + 1] | (c[n + 2] << 8);
      mx = c[n + 3] | (c[n + 4] << 8);
      repeat = true;
      n += 5;
      continue;
    }
    switch (op) {
      case kReLiteral: run.push_back({0xFF, c[n + 1]}); n += 2; break;
      case kReMaskedLiteral: run.push_back({c[n + 2], c[n + 1]}); n += 3; break;
      case kReNotLiteral: run.push_back({0, 0}); n += 2; break;          // consumes, not tested
      case kReMaskedNotLiteral: run.push_back({0, 0}); n += 3; break;
      case kReAny: run.push_back({0, 0}); n += 1; break;
      default: return false;
    }
    if (repeat && tail.size() >= 4) break;
  }
  return pick_guard(head, tail, repeat, mn, mx, skip, backwards, g, bs);
}

// The guard of a yr_re_exec program (re.c:1693-2072), for its ascii attempt:
// the consuming opcodes from its start, following JUMPs and stepping over the
// zero-width assertions, up to its first SPLIT, REPEAT or MATCH.  Until there
// the program is a single fiber, so every byte test on the way must pass (and
// a call that fails one cannot run out of fibers).  Nocase strings compare
// through the host's case folding: their literals are left untested.
bool general_guard(const uint8_t* c, uint32_t len, uint32_t skip, bool backwards, bool nocase,
                   DevGuard& g, uint8_t& bs) {
  // head: the single fiber's consumed positions from the start; tail: those
  // right after its first REPEAT_ANY {mn, mx} (re.c:1810-1821: the fiber
  // forks over every repetition count, each fork consuming mn..mx bytes
  // and then the same opcodes -- the tail lies at distance head + mn + j,
  // j <= mx - mn, as for a fast program's REPEAT_ANY_UNGREEDY)
  std::vector<GuardPos> head, tail;
  uint32_t mn = 0, mx = 0;
  bool repeat = false;
  uint32_t n = 0;
  for (int steps = 0; steps < 256 && n < len && head.size() < 20; ++steps) {
    std::vector<GuardPos>& run = repeat ? tail : head;
    const uint8_t op = c[n];
    const uint32_t sz = re_op_size(op);
    if (sz == 0 || n + sz > len) break;
    if (op == kOpJump) {
      const int64_t t = (int64_t)n + re_i16(c + n + 1);
      if (t < 0 || t >= (int64_t)len) break;
      n = (uint32_t)t;
      continue;
    }
    if (op == kOpWordBoundary || op == kOpNonWordBoundary || op == kOpMatchAtStart ||
        op == kOpMatchAtEnd) {
      n += sz;   // zero width
      continue;
    }
    if (op == kOpRepeatAnyGreedy || op == kOpRepeatAnyUngreedy) {
      if (repeat) break;        // a second repeat: the tail's distance is no longer fixed
      mn = re_u16(c + n + 1);
      mx = re_u16(c + n + 3);
      if (mn > mx) break;
      repeat = true;
      n += sz;
      continue;
    }
    if (op == kOpLiteral) {
      run.push_back(nocase ? GuardPos{0, 0} : GuardPos{0xFF, c[n + 1]});
    } else if (op == kOpMaskedLiteral) {
      run.push_back(nocase ? GuardPos{0, 0} : GuardPos{c[n + 2], c[n + 1]});
    } else if (op == kOpAny || op == kOpClass || op == kOpNotLiteral || op == kOpMaskedNotLiteral ||
               op == kOpWordChar || op == kOpNonWordChar || op == kOpSpace || op == kOpNonSpace ||
               op == kOpDigit || op == kOpNonDigit) {
      run.push_back({0, 0});    // consumes one byte, not tested here
    } else {
      break;                    // MATCH, SPLIT, REPEAT_START/END: the single fiber ends
    }
    n += sz;
    if (repeat && tail.size() >= 4) break;
  }
  return pick_guard(head, tail, repeat, mn, mx, skip, backwards, g, bs);
}
}  // namespace
}  // extern "C++"

extern "C++" {   // (internal helpers: C++ linkage, not exported)
namespace {
// Whether yr_re_exec running `code` (re.c:1693-2072) provably stays below
// RE_MAX_FIBERS (limits.h: 1024), so that it cannot fail with
// ERROR_TOO_MANY_RE_FIBERS (re.c:1228-1229).  Without REPEAT_START/END the
// fibers' stacks stay empty, and live fibers are distinct in (ip, rc) after
// each step (_yr_re_fiber_exists, re.c:1278-1310; rc in -1..max of a
// REPEAT_ANY, re.c:1586-1625): at most ops x (max + 2).  A step's syncs grow
// each of them by at most one fiber per SPLIT / REPEAT_ANY before the next
// dedup (_yr_re_fiber_sync, re.c:1441-1560).  Bound both, conservatively.
bool re_fiber_safe(const uint8_t* c, uint32_t len) {
  uint64_t ops = 0, forks = 0, mx = 0;
  for (uint32_t n = 0; n < len;) {
    const uint8_t op = c[n];
    const uint32_t sz = re_op_size(op);
    if (sz == 0 || n + sz > len) return false;
    if (op == kOpRepeatStartGreedy || op == kOpRepeatEndGreedy || op == kOpRepeatStartUngreedy ||
        op == kOpRepeatEndUngreedy)
      return false;
    if (op == kOpSplitA || op == kOpSplitB) ++forks;
    if (op == kOpRepeatAnyGreedy || op == kOpRepeatAnyUngreedy) {
      ++forks;
      mx = std::max<uint64_t>(mx, re_u16(c + n + 3));
    }
    ++ops;
    n += sz;
  }
  return ops * (mx + 2) * (forks + 2) < 1024;
}

// The 1-byte keys whose calls the scan kernel can classify (kernels.hip
// key_class).  The key's state is its own node unless the byte before it is
// one of at most 8 bytes x with a trie node of depth >= 2 ending in x, key (a
// deeper state has such a suffix; those candidates stay undecided).  Then
// either
//  * "kept": every call of the node's list is kept whatever the bytes --
//    plain literals that fit in the atom (call_matters: backtrack != 0, no
//    FULL_WORD / base64 / fixed offset), made at every position from the
//    largest backtrack on (scanner.c:107) -- or
//  * the list is one regexp call that call_matters drops whenever its forward
//    guard fails (a FAST ascii program, or a yr_re_exec one with only the
//    ascii attempt) and whose tested bytes fit the four bytes the scan keeps
//    beside a certain candidate (the one before the key, the key, two after);
//    the compaction tests it.  (YR_AC_MATCH offsets: the call's offset is
//    position - backtrack, the guard's region starts `base` bytes after it.)
// Pre-verification then never reads the input for such candidates.
// One class plan for every 1-byte key (the drop kernels' kDropPlanModes
// instance): every key's class is a forward guard -- no key without a class,
// none "kept", no exclusions, no backward guard -- with the same region and
// the same tests once each key's test of its own byte (a full-mask compare
// with the key at the key byte, which every candidate of that key passes:
// drain_classes skips it too) is left out, and that is one full-byte compare.
// Then the drain decides all certain candidates of an entry at once, whatever
// their key, in straight-line code (rx: both keys test the byte after them
// against 0xC3).  Measured, one process, both orders
// (profiles/r06_key_plan_ab/): rx's drop kernel 0.94 -> 0.825 ms; the same plan with exclusions and a backward guard (fuzz0) was 2 %
// slower than the per-key loop, and as a drop kernel for a "kept" key (short,
// fuzz3) 7-8 % slower than their non-drop kernel: neither shape takes it.
void key_plan(yr_amd_tables* t) {
  t->kp_on = 0;
  const uint32_t nk = std::min<uint32_t>(t->flat.n_byte_keys, 4);
  if (!t->kd_any || nk == 0) return;
  uint32_t m0 = 0, v0 = 0;
  for (uint32_t k = 0; k < nk; ++k) {
    const uint32_t info = t->kd_info[k];
    if (!(info & 1u) || (info & (2u | 4u | 8u))) return;
    const uint32_t key = (t->flat.byte_keys >> (8 * k)) & 0xFFu;
    const int rs = (int)(int8_t)(info >> 8);
    const uint32_t tmax = (info >> 20) & 3u;
    uint32_t m = t->kd_m[k], v = t->kd_v[k];
    for (uint32_t q = 0; q <= tmax; ++q) {
      const uint32_t mt = (m >> (8 * q)) & 0xFFu, vt = (v >> (8 * q)) & 0xFFu;
      if (rs + (int)q == 0 && mt == 0xFFu && vt == key) {
        m &= ~(0xFFu << (8 * q));
        v &= ~(0xFFu << (8 * q));
      }
    }
    v &= m;
    if (k == 0) {
      m0 = m, v0 = v;
    } else if (info != t->kd_info[0] || m != m0 || v != v0) {
      return;
    }
  }
  // ... and one full-byte compare left (rx: the byte after the key is 0xC3):
  // the drain's one byte_test24 then needs no mask and no loop over the bytes
  int tested = -1;
  for (int q = 0; q < 4; ++q) {
    const uint32_t mt = (m0 >> (8 * q)) & 0xFFu;
    if (mt == 0u) continue;
    if (mt != 0xFFu || tested >= 0) return;
    tested = q;
  }
  if (tested < 0) return;
  t->kp_info = t->kd_info[0];
  t->kp_m = m0;
  t->kp_v = v0;
  t->kp_t = (uint32_t)tested;
  t->kp_on = diag_env("YAMD_NO_KEY_PLAN") != nullptr ? 0u : 1u;
}

void key_classes(yr_amd_tables* t) {
  const FlatTables& f = t->flat;
  t->kp_on = 0;
  t->kd_any = false;
  t->kd_guard = false;
  t->kd_kept = false;
  t->kx_end = 2;
  {
    // the longest match list: the longest chain of pool links (each list is
    // a chain from its head)
    // chain, memoised (lists share tails: a state's list ends with its
    // failure state's, ahocorasick.c:254-300); a bad link counts as overlong
    const size_t np = t->h_pool.size();
    std::vector<uint32_t> len(np + 1, 0), path;
    t->max_list = 0;
    for (size_t q0 = 1; q0 <= np; ++q0) {
      path.clear();
      uint32_t q = (uint32_t)q0, tail = 0;
      while (q != 0 && len[q] == 0) {
        if (q > np || path.size() > np) { tail = 1000; break; }
        path.push_back(q);
        q = t->h_pool[q - 1].next;
      }
      if (tail == 0 && q != 0) tail = len[q];
      for (size_t e = path.size(); e-- > 0;) len[path[e]] = ++tail;
      t->max_list = std::max(t->max_list, len[q0]);
    }
  }
  t->kx_deep = 0;
  t->kx_next = 0;
  for (int k = 0; k < 4; ++k)
    for (int e = 0; e < 4; ++e) t->kd_idx[k][e] = t->kd_bt[k][e] = 0;
  for (int k = 0; k < 4; ++k)
    t->kd_m[k] = t->kd_v[k] = t->kd_info[k] = t->kd_x0[k] = t->kd_x1[k] = t->kd_n[k] =
        t->kd_head[k] = t->kd_min_pos[k] = t->kd_bm[k] = t->kd_bv[k] = 0;
  if (f.root_accepting || t->h_pool.empty() || diag_env("YAMD_NO_KEY_CLASSES") != nullptr) return;
  // Per key the class it can have, then the five bytes the scan keeps beside
  // its certain candidates (kernels.hip key_class): lane bytes key - kp ..
  // key - kp + 4 for one kp in {1, 0, -1} per table (kx_end = 3 - kp), the one
  // under which the most keys are decided.  With one 1-byte key the scan can
  // also test the byte before it against the key's exclusions (kx_deep), so
  // the five bytes may all lie after the key.
  struct Desc {
    bool ok = false, kept = false, bok = false;
    uint32_t nx = 0, xs0 = 0, xs1 = 0, m = 0, v = 0, n = 0, head = 0, min_pos = 0, bm = 0, bv = 0;
    int rs = 0, span = 0, tmax = 0, end = 0, bs = 0, bspan = 0, btmax = 0;
  } d[4];
  const uint32_t nk = std::min<uint32_t>(f.n_byte_keys, 4);
  for (uint32_t k = 0; k < nk; ++k) {
    const uint32_t b = (f.byte_keys >> (8 * k)) & 0xFFu;
    Desc& o = d[k];
    bool too_many = false;
    if ((f.deep_last[b >> 5] >> (b & 31)) & 1u) {
      for (uint32_t x = 0; x < 256; ++x) {
        if (!((f.deep_pair[b * 8 + (x >> 5)] >> (x & 31)) & 1u)) continue;
        if (o.nx == 8) { too_many = true; break; }
        (o.nx < 4 ? o.xs0 : o.xs1) |= x << (8 * (o.nx & 3));
        ++o.nx;
      }
    }
    if (too_many) continue;
    for (uint32_t q = o.nx; q < 8 && o.nx; ++q)   // the first exclusion repeated to fill
      (q < 4 ? o.xs0 : o.xs1) |= (o.xs0 & 0xFFu) << (8 * (q & 3));
    const uint32_t head = f.nodes[kNodeL1 + b];
    if (head == 0 || head > t->h_pool.size()) continue;
    // "kept": every entry a plain fits-in-atom literal (call_matters' early
    // decision), at most 30 of them (pass 1's keep mask)
    uint32_t n = 0, max_bt = 0;
    bool kept = true;
    for (uint32_t q = head; q != 0 && kept; q = t->h_pool[q - 1].next) {
      const DevPoolRec& e = t->h_pool[q - 1];
      kept = (e.flags & (kStrLiteral | kStrFitsInAtom)) == (kStrLiteral | kStrFitsInAtom) &&
             !(e.flags & (kStrUnmodelled | kStrFullWord | kStrFixedOffset)) && e.backtrack != 0 &&
             ++n <= 30;
      max_bt = std::max<uint32_t>(max_bt, e.backtrack);
    }
    if (kept && n > 0) {
      o.ok = o.kept = true;
      o.n = n;
      o.head = head;
      o.min_pos = max_bt;
      continue;
    }
    const DevPoolRec& e = t->h_pool[head - 1];
    const uint32_t fl = e.flags;
    if (e.next != 0 || (fl & kStrLiteral) || e.re.fwd_len == 0 || e.fguard.m == 0) continue;
    if (fl & kStrFastRegexp) {
      if (!(fl & kStrAscii) || (fl & (kStrWide | kStrBase64Any))) continue;
    } else if (((fl & kStrWide) && !(fl & kStrBase64Any)) || !(fl & (kStrAscii | kStrBase64Any))) {
      continue;
    }
    const int base = e.fguard_bs & 15, span = e.fguard_bs >> 4;
    o.rs = base + 1 - (int)e.backtrack;           // region start - key byte
    o.end = base + span + 4 - (int)e.backtrack;   // region end - position
    o.span = span;
    o.tmax = (31 - __builtin_clz(e.fguard.m)) >> 3;   // last tested byte of the 4
    if (o.end < -128 || o.end > 127) continue;
    o.m = e.fguard.m;
    o.v = e.fguard.v;
    o.ok = true;
    // The backward guard as well: with a backward program, a call whose
    // backward run fails never reaches _yr_scan_match_callback
    // (_yr_scan_verify_re_match, scan.c:843-880; verify.hip re_call_matters),
    // and the guard's bytes are that run's single-fiber prefix.  The backward
    // run comes after the forward one, so a yr_re_exec program only when its
    // forward run cannot end in ERROR_TOO_MANY_RE_FIBERS (a scan error the host
    // must still see); yr_re_fast_exec has no such error.
    if (e.re.bwd_len > 0 && e.bguard.m != 0 && ((fl & kStrFastRegexp) || (fl & kPoolFwdFiberSafe))) {
      // region [offset - L, offset), offset = key byte + 1 - backtrack; byte
      // tmin of the guard's four is its lowest tested one
      const int L = (e.bguard_bs & 15) + (e.bguard_bs >> 4) + 4;
      const int tmin = __builtin_ctz(e.bguard.m) >> 3, tmx = (31 - __builtin_clz(e.bguard.m)) >> 3;
      o.bs = 1 - (int)e.backtrack - L + tmin;
      o.bspan = e.bguard_bs >> 4;
      o.btmax = tmx - tmin;
      o.bm = e.bguard.m >> (8 * tmin);
      o.bv = e.bguard.v >> (8 * tmin);
      // (one position only: the scan kernel tests it with one compare; and
      // within the two bytes before the key that its eight-byte windows hold
      // -- a guard further back would only cost the drop kernel its test)
      o.bok = o.bs >= -2 && o.bs < 0 && o.bspan == 0;
      // ... and only where the forward guard alone leaves many candidates
      // undecided: the backward-guard drop instance costs the scan kernel
      // 4-7 % (profiles/r05_ab_inproc.json r5h30: rx, whose forward guard
      // passes 1 in 256, lost more there than its live list gained when a
      // wider window let its guard five bytes back in).  Undecided = passing
      // the forward guard on random bytes (its tested bits, less the key's own
      // byte) or lying past the eight bytes of the window.
      if (o.bok) {
        int bits = __builtin_popcount(o.m);
        if (o.rs <= 0 && o.rs + 3 >= 0 && ((o.m >> (8 * -o.rs)) & 0xFFu) != 0u) bits -= 8;
        const double pass = std::min(1.0, (o.span + 1) * std::ldexp(1.0, -std::max(bits, 0)));
        const int hi = o.rs + o.span + o.tmax;   // last tested byte after the key
        const double outside = o.rs < -2 ? 1.0 : std::min(1.0, std::max(0, hi - 2) / 16.0);
        o.bok = pass + outside >= 0.02;
      }
    }
  }
  // a key is decided at place kp if its identity, the byte before it (with
  // exclusions; or the scan's test of it) and every byte its guard tests lie
  // in the five
  auto fits = [&](const Desc& o, int kp) {
    if (!o.ok || (kp < 0 && nk != 1) || (o.nx && kp < 1 && nk != 1)) return false;
    return o.kept || (kp + o.rs >= 0 && kp + o.rs + o.span + o.tmax <= 4);
  };
  int best_kp = 1, best = 0;
  for (int kp = 1; kp >= -1; --kp) {
    int c = 0;
    for (uint32_t k = 0; k < nk; ++k) c += fits(d[k], kp);
    if (c > best) best = c, best_kp = kp;
  }
  if (best == 0) return;
  t->kx_end = (uint32_t)(3 - best_kp);
  t->kx_deep = best_kp < 1 && nk == 1 && d[0].nx > 0 ? 1u : 0u;
  for (uint32_t k = 0; k < nk; ++k) {
    const Desc& o = d[k];
    if (!fits(o, best_kp)) continue;
    uint32_t info = 1u | (o.nx ? 2u : 0u);
    if (o.kept) {
      info |= 4u;
      t->kd_kept = true;
      t->kd_n[k] = o.n;
      t->kd_head[k] = o.head;
      t->kd_min_pos[k] = o.min_pos;
      uint32_t q = o.head;
      for (uint32_t e = 0; e < 4 && q != 0; ++e, q = t->h_pool[q - 1].next) {
        t->kd_idx[k][e] = q - 1;
        t->kd_bt[k][e] = t->h_pool[q - 1].backtrack;
      }
    } else {
      t->kd_m[k] = o.m;
      t->kd_v[k] = o.v;
      if (o.bok) {
        info |= 8u;
        t->kd_min_pos[k] = (uint32_t)(uint8_t)(int8_t)o.bs | (uint32_t)o.btmax << 12;
        t->kd_bm[k] = o.bm;
        t->kd_bv[k] = o.bv;
      }
      t->kd_guard = true;
      t->kx_next = 1;   // (a guard's bytes may run past the lane: keep the next lane's two)
      info |= ((uint32_t)(uint8_t)(int8_t)o.rs << 8) | ((uint32_t)o.span << 16) |
              ((uint32_t)o.tmax << 20) | ((uint32_t)(uint8_t)(int8_t)o.end << 24);
    }
    t->kd_info[k] = info;
    t->kd_x0[k] = o.xs0;
    t->kd_x1[k] = o.xs1;
    t->kd_any = true;
  }
  key_plan(t);
  // the records the scan kernel reads (ScanParams::kc); without them, no
  // classes at all (the scan then keeps every candidate: still exact)
  uint32_t kc[kKcWords] = {};
  for (int k = 0; k < 4; ++k) {
    const uint32_t r[8] = {t->kd_info[k], t->kd_m[k], t->kd_v[k], t->kd_x0[k],
                           t->kd_x1[k], t->kd_min_pos[k], t->kd_bm[k], t->kd_bv[k]};
    for (int f = 0; f < 8; ++f) kc[8 * k + f] = r[f];
  }
  // the plan (kernels.hip drain_classes): info, the compared byte's value
  // replicated, its shift (rs + t + 4)
  if (t->kp_on) {
    const int32_t rs = (int32_t)(int8_t)(t->kp_info >> 8);
    kc[kKcPlan] = t->kp_info;
    kc[kKcPlan + 1] = ((t->kp_v >> (8 * t->kp_t)) & 0xFFu) * 0x01010101u;
    kc[kKcPlan + 2] = (uint32_t)(rs + (int32_t)t->kp_t + 4);
  }
  if ((t->d_kc == nullptr && hipMalloc((void**)&t->d_kc, sizeof(kc)) != hipSuccess) ||
      hipMemcpy(t->d_kc, kc, sizeof(kc), hipMemcpyHostToDevice) != hipSuccess) {
    if (t->d_kc) (void)hipFree(t->d_kc);
    t->d_kc = nullptr;
    t->kd_any = false;
    t->kp_on = 0;
    t->kd_guard = false;
    t->kd_kept = false;
  }
}
}  // namespace
}  // extern "C++"

// Not declared in include/yara_amd.h: re_fiber_safe on one yr_re_exec
// program, for the CPU tests (tests/test_guards.py): 1 if its run provably
// stays below RE_MAX_FIBERS, else 0.
int yr_amd__re_fiber_safe(const uint8_t* code, uint32_t len) {
  if (code == nullptr) return -1;
  return re_fiber_safe(code, len) ? 1 : 0;
}

// Not declared in include/yara_amd.h: the guard compiler on one program, for
// the CPU tests (tests/test_guards.py).  Returns 1 and the guard (verify.h
// DevGuard: m, v, base | span << 4) if the program has one, else 0.
int yr_amd__program_guard(const uint8_t* code, uint32_t len, uint32_t skip, int backwards,
                          int general, int nocase, uint32_t* m, uint32_t* v, uint32_t* bs) {
  if (code == nullptr || m == nullptr || v == nullptr || bs == nullptr) return -1;
  DevGuard g{0u, 0u};
  uint8_t b = 0;
  const bool ok = general ? general_guard(code, len, skip, backwards != 0, nocase != 0, g, b)
                          : fast_guard(code, len, skip, backwards != 0, g, b);
  *m = ok ? g.m : 0u;
  *v = ok ? g.v : 0u;
  *bs = ok ? b : 0u;
  return ok ? 1 : 0;
}

int yr_amd_re_code_extent(const uint8_t* code, uint64_t avail, uint32_t* extent) {
  using yamd::re_general_extent;
  if (code == nullptr || extent == nullptr) return YR_AMD_INVALID_ARGUMENT;
  *extent = re_general_extent(code, avail);
  return *extent ? YR_AMD_SUCCESS : YR_AMD_INVALID_ARGUMENT;
}

int yr_amd_tables_set_re_code(yr_amd_tables* t, uint32_t n_pool, const uint32_t* fwd_off,
                              const uint32_t* fwd_len, const uint32_t* bwd_off,
                              const uint32_t* bwd_len, const uint8_t* code, uint64_t code_len) {
  if (t == nullptr || !t->has_strings || t->d_re_code != nullptr) return YR_AMD_INVALID_ARGUMENT;
  if (n_pool != t->flat.pool_next.size()) return YR_AMD_INVALID_ARGUMENT;
  if (n_pool > 0 && (fwd_off == nullptr || fwd_len == nullptr || bwd_off == nullptr ||
                     bwd_len == nullptr))
    return YR_AMD_INVALID_ARGUMENT;
  if (code_len > 0 && code == nullptr) return YR_AMD_INVALID_ARGUMENT;
  std::vector<DevRe> re(n_pool);
  for (uint32_t k = 0; k < n_pool; ++k) {
    re[k] = DevRe{fwd_off[k], fwd_len[k], bwd_off[k], bwd_len[k]};
    if (fwd_len[k] == 0) {
      re[k] = DevRe{0, 0, 0, 0};
      continue;
    }
    if ((uint64_t)fwd_off[k] + fwd_len[k] > code_len || (uint64_t)bwd_off[k] + bwd_len[k] > code_len)
      return YR_AMD_INVALID_ARGUMENT;
    // FAST_REGEXP strings run yr_re_fast_exec (a linear program), the others
    // yr_re_exec (any well-formed program of exactly the given length)
    const bool fast = t->h_str_flags[t->h_pool_string[k]] & kStrFastRegexp;
    auto ok = [&](uint32_t off, uint32_t len) {
      return fast ? fast_program_ok(code + off, len) == len
                  : re_general_extent(code + off, len) == len;
    };
    if (!ok(fwd_off[k], fwd_len[k])) return YR_AMD_INVALID_ARGUMENT;
    if (bwd_len[k] > 0 && !ok(bwd_off[k], bwd_len[k])) return YR_AMD_INVALID_ARGUMENT;
  }
  HIP_TRY(hipSetDevice(t->device));
  // the blob with 64 bytes of zero padding: the verify kernel stages programs
  // with aligned 16-byte loads that may reach past the last one
  std::vector<uint8_t> padded((size_t)code_len + 64, 0);
  if (code_len > 0) memcpy(padded.data(), code, (size_t)code_len);
  int r = upload(t->d_re_code, padded.data(), padded.size());
  if (r) return r;
  // the programs go into the pool records (uploaded again) with their guards
  // (the forward program starts at the atom: its first `backtrack` bytes are
  // the atom's)
  const bool no_guards = diag_env("YAMD_NO_GUARDS") != nullptr;   // A/B measurements only
  for (uint32_t k = 0; k < n_pool; ++k) {
    DevPoolRec& e = t->h_pool[k];
    e.re = re[k];
    e.fguard = e.bguard = DevGuard{0u, 0u};
    e.fguard_bs = e.bguard_bs = 0;
    if (re[k].fwd_len == 0) continue;
    if (no_guards) continue;
    const uint32_t sflags = t->h_str_flags[t->h_pool_string[k]];
    const bool nocase = sflags & kStrNoCase;
    auto guard = [&](uint32_t off, uint32_t len, uint32_t skip, bool bw, DevGuard& g, uint8_t& bs) {
      const bool ok = (sflags & kStrFastRegexp)
                          ? fast_guard(code + off, len, skip, bw, g, bs)
                          : general_guard(code + off, len, skip, bw, nocase, g, bs);
      if (!ok) g = DevGuard{0u, 0u};
    };
    guard(re[k].fwd_off, re[k].fwd_len, e.backtrack, false, e.fguard, e.fguard_bs);
    if (re[k].bwd_len > 0) guard(re[k].bwd_off, re[k].bwd_len, 0, true, e.bguard, e.bguard_bs);
    e.flags &= ~kPoolFwdFiberSafe;
    if (!(sflags & kStrFastRegexp) && re_fiber_safe(code + re[k].fwd_off, re[k].fwd_len))
      e.flags |= kPoolFwdFiberSafe;
  }
  if (n_pool > 0 && hipMemcpy(t->d_pool, t->h_pool.data(), n_pool * sizeof(DevPoolRec),
                              hipMemcpyHostToDevice) != hipSuccess)
    return YR_AMD_INTERNAL_FATAL_ERROR;
  key_classes(t);
  return YR_AMD_SUCCESS;
}

int yr_amd_verify_device(yr_amd_scanner* s, uint64_t data_base, const yr_amd_verify_rec** d_records,
                         uint64_t* count) {
  if (s == nullptr || s->pending || !s->tables->has_strings) return YR_AMD_INVALID_ARGUMENT;
  const yr_amd_tables* t = s->tables;
  const ScanParams& L = s->last;
  HIP_TRY(hipSetDevice(t->device));
  VerifyParams v{};
  v.data = L.data;
  v.size = L.block_size;
  v.win_lo = s->win_lo;
  v.win_hi = s->win_hi;
  v.data_base = data_base;
  v.all = s->last_all ? 1 : 0;
  if (v.all) {
    // every position of the scanned range: (byte_begin, byte_end], plus 0
    v.all_first = L.byte_begin == 0 ? 0 : L.byte_begin + 1;
    v.count = L.byte_end + 1 - v.all_first;
    if (L.byte_begin == L.byte_end && L.byte_begin != 0) v.count = 0;
  } else {
    v.positions = s->d_positions;
    v.count = s->last_count;
    // (profiling needs every call past the early returns: no skipping; the
    // live list counts in 32 bits, so a stream of 2^32 candidates -- all of
    // them possibly undecided -- is decided without the classes too)
    const bool classes = !t->profile && s->last_count <= 0xFFFFFFFFull;
    v.dead = classes ? L.dead : nullptr;
    v.live = classes ? L.live : nullptr;
    v.live_count = L.live_count;
    v.live_first = s->d_seg_offset;
    v.live_segs = L.n_segments;
    v.live_off = s->d_live_off;
    // records in most groups (every candidate of a "kept" key is one): the
    // write pass as one wave per group
    v.direct = classes && t->kd_kept && t->max_list <= 31 ? 1 : 0;
    // a verified-only scan that left candidates out: the records still index
    // the full stream
    v.cand_index = L.drop_dead && s->last_full_count != s->last_count ? L.cand_index : nullptr;
    for (int k = 0; k < 4; ++k) {
      v.kd_n[k] = L.kd_n[k];
      v.kd_head[k] = L.kd_head[k];
      for (int e = 0; e < 4; ++e) {
        v.kd_idx[k][e] = t->kd_idx[k][e];
        v.kd_bt[k][e] = t->kd_bt[k][e];
      }
    }
  }
  const FlatTables& f = t->flat;
  v.nodes = t->d_nodes;
  v.n3_off = f.n3_off;
  v.n3_mask = f.n3_mask;
  v.n4_off = f.n4_off;
  v.n4_mask = f.n4_mask;
  v.root_head = f.M[0];
  v.pool = t->d_pool;
  v.str_bytes = t->d_str_bytes;
  v.lowercase = t->d_lowercase;
  v.re_on = t->d_re_code != nullptr ? 1 : 0;
  v.profile = t->profile ? 1 : 0;
  v.re_code = t->d_re_code;
  uint64_t total = 0;
  // records carry a 32-bit candidate index: a candidate stream longer than
  // YR_AMD_VERIFY_MAX_CANDIDATES (2^32; possible only on blocks of 4 GiB or
  // more) is refused -- replay it on the host (yr_amd_scan_block +
  // yr_amd_replay) instead, as the libyara shim does for such blocks
  if (v.count > YR_AMD_VERIFY_MAX_CANDIDATES ||
      (!v.all && s->last_full_count > YR_AMD_VERIFY_MAX_CANDIDATES))
    return YR_AMD_INVALID_ARGUMENT;
  if (v.count > 0) {
    if (v.data == nullptr) return YR_AMD_INVALID_ARGUMENT;
    // (d_vcount: the live list's dense copy behind the counts, only when the
    // scan made one -- a 2^32-candidate stream has none and needs 16 GiB less)
    int r = grow(s->d_vcount, s->vcount_cap, (v.live != nullptr ? 2 : 1) * v.count);
    if (!r) r = grow(s->d_vkeep, s->vkeep_cap, 2 * v.count);
    if (!r) r = grow(s->d_vblock, s->vblock_cap, verify_groups(v.count) + 1);
    if (!r) r = grow(s->d_vchunk, s->vchunk_cap, verify_chunks(v.count) + 1);
    // record space before the count is known (one per 16 candidates, capped;
    // the buffer is kept, so mostly a scanner's first calls outgrow it): the
    // write pass is queued behind the count pass with no host round trip in
    // between, and re-run into a larger buffer only when the records did not fit
    if (!r) r = grow(s->d_vrec, s->vrec_cap, std::min<uint64_t>(v.count / 16 + 1, 1u << 20));
    if (r) return r;
    v.counts = s->d_vcount;
    v.live_dense = v.live != nullptr ? s->d_vcount + v.count : nullptr;
    v.keep = s->d_vkeep;
    v.heads = s->d_vkeep + v.count;
    v.block_off = s->d_vblock;
    v.chunk_off = s->d_vchunk;
    v.out = s->d_vrec;
    v.out_cap = s->vrec_cap;
    // count pass -> block offsets (total straight into the host-mapped
    // summary) -> write pass, then one wait
    if (v.live != nullptr) {
      // the scan's live list: only its candidates are decided, their record
      // counts added to the groups' (zeroed by the live list's gather)
      HIP_TRY(launch_verify_live(v, s->d_summary, s->stream));
    } else {
      HIP_TRY(launch_verify(v, 0, s->stream));
    }
    KeptLists kept{{v.kd_n[0], v.kd_n[1], v.kd_n[2], v.kd_n[3]}};
    HIP_TRY(launch_block_offsets(s->d_vblock, s->d_vchunk, v.count, s->d_hsum, v.dead, kept,
                                 s->stream));
    HIP_TRY(launch_verify(v, 1, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    total = s->h_summary[0];
    if (total > v.out_cap) {
      // geometric growth: a scanner whose record counts creep upward re-runs
      // the write pass O(log) times, not once per call
      r = grow(s->d_vrec, s->vrec_cap, std::max<uint64_t>(total, 2 * s->vrec_cap));
      if (r) return r;
      v.out = s->d_vrec;
      v.out_cap = s->vrec_cap;
      HIP_TRY(launch_verify(v, 1, s->stream));
      HIP_TRY(hipStreamSynchronize(s->stream));
    }
  }
  if (debug_level() >= 2 && total > 0) {
    std::vector<yr_amd_verify_rec> h(total);
    if (hipMemcpy(h.data(), s->d_vrec, total * sizeof(yr_amd_verify_rec), hipMemcpyDeviceToHost) ==
        hipSuccess)
      for (const yr_amd_verify_rec& r : h)
        fprintf(stderr, "- verify pool=%u offset=%llu candidate=%u base=0x%llx // yr_amd_verify_device()\n",
                r.pool_index, (unsigned long long)r.offset, r.candidate,
                (unsigned long long)data_base);
  }
  if (debug_level() >= 1)
    fprintf(stderr, "- %llu candidates -> %llu verify calls // yr_amd_verify_device()\n",
            (unsigned long long)v.count, (unsigned long long)total);
  if (d_records) *d_records = reinterpret_cast<const yr_amd_verify_rec*>(s->d_vrec);
  if (count) *count = total;
  return YR_AMD_SUCCESS;
}

int yr_amd_scan_block_verified(yr_amd_scanner* s, const uint8_t* data, size_t size,
                               uint64_t data_base, const yr_amd_verify_rec** records,
                               uint64_t* count) {
  if (s == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  if (!s->tables->has_strings) return YR_AMD_INVALID_ARGUMENT;
  HIP_TRY(hipSetDevice(s->tables->device));
  // (a device buffer even for an empty block: a root-accepting rule set
  // pre-verifies its position 0, which needs a data pointer)
  int rg = grow(s->d_block, s->d_block_cap, std::max<size_t>(size, 16));
  if (rg) return rg;
  if (size > 0 &&
      hipMemcpyAsync(s->d_block, data, size, hipMemcpyHostToDevice, s->stream) != hipSuccess)
    return YR_AMD_COULD_NOT_MAP_FILE;
  // (a verified-only scan: nothing but the records leaves this call)
  const bool was = s->verified_only;
  s->verified_only = true;
  int r = yr_amd_scan_device(s, s->d_block, size, 0, size);
  if (!r) r = yr_amd_scan_device_result(s, nullptr, nullptr, nullptr);
  s->verified_only = was;
  const yr_amd_verify_rec* d_rec = nullptr;
  uint64_t n = 0;
  if (!r) r = yr_amd_verify_device(s, data_base, &d_rec, &n);
  if (r) return r;
  s->h_vrec.resize(n);
  if (n > 0) {
    HIP_TRY(hipMemcpyAsync(s->h_vrec.data(), d_rec, n * sizeof(yr_amd_verify_rec),
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
  }
  if (records) *records = s->h_vrec.data();
  if (count) *count = n;
  return YR_AMD_SUCCESS;
}

int yr_amd_trace_walk(yr_amd_scanner* s, const uint8_t* d_data, size_t size, uint64_t data_base,
                      yr_amd_trace_rec* out, uint64_t cap, uint64_t* count) {
  if (s == nullptr || count == nullptr || (d_data == nullptr && size > 0) ||
      (out == nullptr && cap > 0))
    return YR_AMD_INVALID_ARGUMENT;
  const FlatTables& f = s->tables->flat;
  const uint64_t n_pos = (uint64_t)size + 1;   // positions 0 .. size
  const uint64_t n_blocks64 = (n_pos + 255) / 256;
  if (n_blocks64 > 0x7FFFFFFFu) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n_blocks = (uint32_t)n_blocks64;
  HIP_TRY(hipSetDevice(s->tables->device));
  if (s->d_trace_T == nullptr) {
    // both tables into locals first: the cache is set only once complete, so
    // a failed allocation or upload leaves it empty for the next call
    uint32_t *dT = nullptr, *dM = nullptr;
    const size_t nT = f.T.size() * sizeof(uint32_t), nM = f.M.size() * sizeof(uint32_t);
    if (hipMalloc(&dT, nT) != hipSuccess || hipMalloc(&dM, nM) != hipSuccess ||
        hipMemcpy(dT, f.T.data(), nT, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dM, f.M.data(), nM, hipMemcpyHostToDevice) != hipSuccess) {
      if (dT) (void)hipFree(dT);
      if (dM) (void)hipFree(dM);
      return YR_AMD_INTERNAL_FATAL_ERROR;
    }
    s->d_trace_T = dT;
    s->d_trace_M = dM;
  }
  // per-block counts -> offsets on the host (a debugging path: blocks are small)
  uint32_t* d_cnt = nullptr;
  uint64_t* d_off = nullptr;
  yr_amd_trace_rec* d_out = nullptr;
  int r = YR_AMD_SUCCESS;
  std::vector<uint32_t> cnt(n_blocks);
  std::vector<uint64_t> off(n_blocks);
  uint64_t total = 0;
  if (hipMalloc(&d_cnt, n_blocks * sizeof(uint32_t)) != hipSuccess ||
      launch_trace_count(s->d_trace_T, d_data, n_pos, d_cnt, n_blocks, s->stream) != hipSuccess ||
      hipMemcpyAsync(cnt.data(), d_cnt, n_blocks * sizeof(uint32_t), hipMemcpyDeviceToHost,
                     s->stream) != hipSuccess ||
      hipStreamSynchronize(s->stream) != hipSuccess) {
    r = YR_AMD_INTERNAL_FATAL_ERROR;
  } else {
    for (uint32_t b = 0; b < n_blocks; ++b) {
      off[b] = total;
      total += cnt[b];
    }
    const uint64_t rows = std::min<uint64_t>(total, cap);
    if (rows > 0 &&
        (hipMalloc(&d_off, n_blocks * sizeof(uint64_t)) != hipSuccess ||
         hipMalloc(&d_out, rows * sizeof(yr_amd_trace_rec)) != hipSuccess ||
         hipMemcpyAsync(d_off, off.data(), n_blocks * sizeof(uint64_t), hipMemcpyHostToDevice,
                        s->stream) != hipSuccess ||
         launch_trace_write(s->d_trace_T, s->d_trace_M, d_data, n_pos, d_off, d_out, rows, n_blocks,
                            s->stream) != hipSuccess ||
         hipMemcpyAsync(out, d_out, rows * sizeof(yr_amd_trace_rec), hipMemcpyDeviceToHost,
                        s->stream) != hipSuccess ||
         hipStreamSynchronize(s->stream) != hipSuccess))
      r = YR_AMD_INTERNAL_FATAL_ERROR;
    if (!r && debug_level() >= 2)
      for (uint64_t k = 0; k < rows; ++k)
        fprintf(stderr,
                "- match_table[state=%u]=%u i=%llu block_data=%p block->base=0x%llx // "
                "yr_amd_trace_walk()\n",
                out[k].state, out[k].match, (unsigned long long)out[k].position,
                (const void*)d_data, (unsigned long long)data_base);
  }
  for (void* p : {(void*)d_cnt, (void*)d_off, (void*)d_out})
    if (p) (void)hipFree(p);
  if (!r) *count = total;
  return r;
}

int yr_amd_replay(const yr_amd_tables* t, const uint8_t* data, size_t size,
                  const uint64_t* positions, uint64_t count, int all_positions,
                  yr_amd_verify_fn verify, void* user) {
  if (t == nullptr || verify == nullptr || (data == nullptr && size > 0)) return YR_AMD_INVALID_ARGUMENT;
  if (!all_positions && count > 0 && positions == nullptr) return YR_AMD_INVALID_ARGUMENT;
  const FlatTables& f = t->flat;
  const uint32_t* T = f.T.data();
  const uint32_t* M = f.M.data();
  const uint32_t* nx = f.pool_next.data();
  const uint16_t* bt = f.pool_backtrack.data();
  const uint64_t n = all_positions ? (uint64_t)size + 1 : count;
  uint64_t prev = 0;
  for (uint64_t c = 0; c < n; ++c) {
    const uint64_t i = all_positions ? c : positions[c];
    if (i > size || (c > 0 && i <= prev)) return YR_AMD_INVALID_ARGUMENT;  // must ascend
    prev = i;
    // state at i from root over the last <= YR_MAX_ATOM_LENGTH bytes
    uint32_t state = 0;
    for (uint64_t j = i > YR_AMD_MAX_ATOM_LENGTH ? i - YR_AMD_MAX_ATOM_LENGTH : 0; j < i; ++j)
      state = ac_step(T, state, data[j]);
    if (M[state] == 0) return YR_AMD_INTERNAL_FATAL_ERROR;
    if (debug_level() >= 2)
      fprintf(stderr, "- match_table[state=%u]=%u i=%llu block_data=%p // yr_amd_replay()\n", state,
              M[state], (unsigned long long)i, (const void*)data);
    // scanner.c:105-121
    for (uint32_t k = M[state]; k != 0; k = nx[k - 1]) {
      if (bt[k - 1] <= i) {
        const int r = verify(user, k - 1, i - bt[k - 1]);
        if (r != 0) return r;
      }
    }
  }
  return YR_AMD_SUCCESS;
}

// ---------------------------------------------------------------------------
// xorshift64 jump-ahead: the generator is linear over GF(2)^64, so the state
// after m steps is A^m x0; chunk start states are computed on the host.
// ---------------------------------------------------------------------------
extern "C++" {   // (internal helpers: C++ linkage, not exported)
namespace {
struct Mat64 {
  uint64_t col[64];
};
inline uint64_t xs_step(uint64_t x) {
  x ^= x << 13;
  x ^= x >> 7;
  x ^= x << 17;
  return x;
}
inline uint64_t apply(const Mat64& m, uint64_t v) {
  uint64_t r = 0;
  for (int j = 0; j < 64; ++j)
    if ((v >> j) & 1) r ^= m.col[j];
  return r;
}
Mat64 compose(const Mat64& a, const Mat64& b) {  // a(b(.))
  Mat64 r;
  for (int j = 0; j < 64; ++j) r.col[j] = apply(a, b.col[j]);
  return r;
}
Mat64 power(uint64_t m) {
  Mat64 base, acc;
  for (int j = 0; j < 64; ++j) {
    base.col[j] = xs_step(1ull << j);
    acc.col[j] = 1ull << j;
  }
  while (m) {
    if (m & 1) acc = compose(base, acc);
    base = compose(base, base);
    m >>= 1;
  }
  return acc;
}
}  // namespace
}  // extern "C++"

int yr_amd_fill_xorshift64(void* d_buf, uint64_t n, uint64_t seed, uint64_t offset, void* stream) {
  if (n == 0) return YR_AMD_SUCCESS;
  if (d_buf == nullptr || (((uintptr_t)d_buf) & 15) != 0) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t chunk = 1u << 16;
  const uint64_t n_chunks64 = (n + chunk - 1) / chunk;
  if (n_chunks64 > 0xFFFFFFFFull) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n_chunks = (uint32_t)n_chunks64;
  std::vector<uint64_t> states(n_chunks);
  const Mat64 jump = power(chunk);
  uint64_t x = apply(power(offset), 0x9E3779B97F4A7C15ull * seed);
  for (uint32_t c = 0; c < n_chunks; ++c) {
    states[c] = x;
    x = apply(jump, x);
  }
  uint64_t* d_states = nullptr;
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipMalloc((void**)&d_states, n_chunks * sizeof(uint64_t)));
  int r = YR_AMD_SUCCESS;
  if (hipMemcpyAsync(d_states, states.data(), n_chunks * sizeof(uint64_t), hipMemcpyHostToDevice,
                     st) != hipSuccess ||
      launch_xorshift((uint8_t*)d_buf, n, d_states, n_chunks, chunk, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    r = YR_AMD_INTERNAL_FATAL_ERROR;
  (void)hipFree(d_states);
  return r;
}

}  // extern "C"
