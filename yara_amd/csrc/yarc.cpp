// Device tables straight from a compiled rules file.
//
// A .yarc file (yarac output, yr_rules_save) is libyara's arena serialised by
// yr_arena_save_stream (libyara/arena.c:627-700) and read back by
// yr_arena_load_stream (arena.c:543-625); yr_rules_from_arena (rules.c:326-370)
// then points YR_RULES at its sections.  Layout (little endian, version 19):
//
//   header   {u8 magic[4] = "YARA", u8 version, u8 num_buffers}   (arena.c:43-48)
//   table    num_buffers x {u64 offset, u32 size}                  (arena.c:50-54)
//   buffers  the contents of every non-empty buffer, in order
//   relocs   {u32 buffer_id, u32 offset} until EOF: the 8 bytes at that place
//            hold a YR_ARENA_REF {u32 buffer_id, u32 offset} of the target
//            instead of a pointer ({~0, ~0} = NULL)              (arena.c:660-700)
//
// Sections (compiler.h:58-69) used here: 3 strings table (YR_STRING, 56 bytes),
// 5 SZ pool (string bytes), 7 RE code, 8 AC transition table (u32 slots),
// 9 AC match table (u32, 1-based pool index), 10 AC match pool (YR_AC_MATCH,
// 40 bytes), 11 summary {num_rules, num_strings, num_namespaces}.  Struct
// offsets are those of the x86-64 build the file format fixes (types.h:211-346,
// pack(8); DECLARE_REFERENCE fields are 8 bytes):
//   YR_STRING    flags @0 u32, idx @4, fixed_offset @8 i64, rule_idx @16,
//                length @20 i32, string @24 ref, chained_to @32, gaps @40/44,
//                identifier @48
//   YR_AC_MATCH  string @0 ref, forward_code @8, backward_code @16, next @24,
//                backtrack @32 u16
// Nothing of libyara is linked: the pool's references become the flat arrays
// yr_amd_tables_create / _set_strings / _set_re_code take.
#include <string.h>

#include <vector>

#include "../../include/yara_amd.h"
#include "re_program.h"

namespace {

constexpr uint32_t kArenaVersion = 19;
constexpr uint32_t kStringsTable = 3, kSzPool = 5, kReCode = 7, kAcTransition = 8,
                   kAcMatchTable = 9, kAcMatchPool = 10, kSummary = 11;
constexpr uint32_t kStringSize = 56, kMatchSize = 40;
constexpr uint32_t kFastRegexp = 0x40, kLiteral = 0x400;

struct Ref {
  uint32_t buffer, offset;
  bool null() const { return buffer == 0xFFFFFFFFu && offset == 0xFFFFFFFFu; }
};

template <typename T>
T rd(const uint8_t* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}

struct Arena {
  std::vector<const uint8_t*> data;
  std::vector<uint32_t> size;
  std::vector<std::vector<uint8_t>> reloc_mark;   // 1 at offsets holding a ref

  const uint8_t* at(uint32_t b, uint64_t off, uint64_t n) const {
    if (b >= data.size() || off + n > size[b]) return nullptr;
    return data[b] + off;
  }
  // A relocatable field: must be listed in the relocation table.
  bool ref(uint32_t b, uint64_t off, Ref& r) const {
    const uint8_t* p = at(b, off, 8);
    if (p == nullptr || reloc_mark[b].empty() || !reloc_mark[b][off]) return false;
    r = Ref{rd<uint32_t>(p), rd<uint32_t>(p + 4)};
    return true;
  }
};

int parse(const uint8_t* f, size_t n, Arena& a) {
  if (n < 6 || memcmp(f, "YARA", 4) != 0) return YR_AMD_INVALID_ARGUMENT;
  if (f[4] != kArenaVersion) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t nb = f[5];
  if (nb <= kSummary || n < 6 + 12ull * nb) return YR_AMD_INVALID_ARGUMENT;
  a.data.resize(nb);
  a.size.resize(nb);
  a.reloc_mark.resize(nb);
  uint64_t pos = 6 + 12ull * nb;
  for (uint32_t i = 0; i < nb; ++i) {
    const uint64_t off = rd<uint64_t>(f + 6 + 12 * i);
    const uint32_t sz = rd<uint32_t>(f + 6 + 12 * i + 8);
    // buffers follow each other in order (arena.c:644-658)
    if (sz > 0 && (off != pos || off + sz > n)) return YR_AMD_INVALID_ARGUMENT;
    a.data[i] = f + off;
    a.size[i] = sz;
    pos += sz;
  }
  if ((n - pos) % 8 != 0) return YR_AMD_INVALID_ARGUMENT;
  for (; pos < n; pos += 8) {
    const uint32_t b = rd<uint32_t>(f + pos), o = rd<uint32_t>(f + pos + 4);
    if (b >= nb || (uint64_t)o + 8 > a.size[b]) return YR_AMD_INVALID_ARGUMENT;
    if (a.reloc_mark[b].empty()) a.reloc_mark[b].assign(a.size[b], 0);
    a.reloc_mark[b][o] = 1;
  }
  return YR_AMD_SUCCESS;
}

// Length (incl. MATCH) of a linear fast-exec program starting at p (re.c
// opcodes, re.h:65-92), bounded by the section end; 0 if not one.
uint32_t fast_len(const uint8_t* p, uint64_t avail) {
  uint64_t n = 0;
  while (n < avail) {
    switch (p[n]) {
      case 0xA0: n += 1; break;
      case 0xA2: case 0xAE: n += 2; break;
      case 0xA4: case 0xAF: n += 3; break;
      case 0xB5: n += 5; break;
      case 0xAD: return (uint32_t)(n + 1);
      default: return 0;
    }
  }
  return 0;
}

}  // namespace

extern "C" int yr_amd_tables_load_yarc(const uint8_t* file, size_t file_size, int device,
                                       yr_amd_tables** tables) {
  if (tables == nullptr || (file == nullptr && file_size > 0)) return YR_AMD_INVALID_ARGUMENT;
  *tables = nullptr;
  Arena a;
  int r = parse(file, file_size, a);
  if (r) return r;

  const uint8_t* summary = a.at(kSummary, 0, 12);
  if (summary == nullptr) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n_strings = rd<uint32_t>(summary + 4);
  if ((uint64_t)n_strings * kStringSize > a.size[kStringsTable]) return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n_slots = a.size[kAcTransition] / 4;
  // the match table grows in steps of 257 pointers, the transition table in
  // steps of 257 u32 (ahocorasick.c:446-449): only its first n_slots entries
  // are meaningful (rules.c:442 sizes both by the transition table)
  if (n_slots == 0 || a.size[kAcMatchTable] < 4ull * n_slots || a.size[kAcTransition] % 4)
    return YR_AMD_INVALID_ARGUMENT;
  const uint32_t n_pool = a.size[kAcMatchPool] / kMatchSize;
  if (a.size[kAcMatchPool] % kMatchSize) return YR_AMD_INVALID_ARGUMENT;

  std::vector<uint32_t> T(n_slots), M(n_slots);
  memcpy(T.data(), a.data[kAcTransition], 4ull * n_slots);
  memcpy(M.data(), a.data[kAcMatchTable], 4ull * n_slots);

  // pool: next -> 1-based index, string -> index, backtrack, RE programs
  const size_t np1 = n_pool ? n_pool : 1;   // never hand out null arrays
  std::vector<uint32_t> nx(np1), ps(np1), fo(np1), fl(np1), bo(np1), bl(np1);
  std::vector<uint16_t> bt(np1);
  std::vector<uint8_t> code;
  std::vector<uint32_t> sflags(n_strings ? n_strings : 1);
  for (uint32_t k = 0; k < n_strings; ++k)
    sflags[k] = rd<uint32_t>(a.data[kStringsTable] + (uint64_t)k * kStringSize);
  for (uint32_t k = 0; k < n_pool; ++k) {
    const uint64_t base = (uint64_t)k * kMatchSize;
    Ref rs, rf, rb, rn;
    if (!a.ref(kAcMatchPool, base + 0, rs) || !a.ref(kAcMatchPool, base + 8, rf) ||
        !a.ref(kAcMatchPool, base + 16, rb) || !a.ref(kAcMatchPool, base + 24, rn))
      return YR_AMD_INVALID_ARGUMENT;
    if (rs.null() || rs.buffer != kStringsTable || rs.offset % kStringSize ||
        rs.offset / kStringSize >= n_strings)
      return YR_AMD_INVALID_ARGUMENT;
    ps[k] = rs.offset / kStringSize;
    if (rn.null()) {
      nx[k] = 0;
    } else {
      if (rn.buffer != kAcMatchPool || rn.offset % kMatchSize || rn.offset / kMatchSize >= n_pool)
        return YR_AMD_INVALID_ARGUMENT;
      nx[k] = rn.offset / kMatchSize + 1;
    }
    bt[k] = rd<uint16_t>(a.data[kAcMatchPool] + base + 32);
    fo[k] = fl[k] = bo[k] = bl[k] = 0;
    const uint32_t sf = sflags[ps[k]];
    if (!(sf & kLiteral) && !rf.null() && rf.buffer == kReCode && rf.offset < a.size[kReCode]) {
      // FAST_REGEXP (hex) strings: linear fast-exec programs; other regexps:
      // every instruction reachable from the start (yr_re_exec)
      auto len_of = [&](uint32_t off) {
        const uint8_t* p = a.data[kReCode] + off;
        const uint64_t avail = a.size[kReCode] - off;
        return (sf & kFastRegexp) ? fast_len(p, avail) : yamd::re_general_extent(p, avail);
      };
      const uint32_t f = len_of(rf.offset);
      uint32_t b = 0;
      bool ok = f > 0;
      if (ok && !rb.null()) {
        ok = rb.buffer == kReCode && rb.offset < a.size[kReCode];
        if (ok) b = len_of(rb.offset);
        ok = ok && b > 0;
      }
      if (ok) {
        fo[k] = (uint32_t)code.size();
        fl[k] = f;
        code.insert(code.end(), a.data[kReCode] + rf.offset, a.data[kReCode] + rf.offset + f);
        bo[k] = (uint32_t)code.size();
        bl[k] = b;
        if (b) code.insert(code.end(), a.data[kReCode] + rb.offset, a.data[kReCode] + rb.offset + b);
      }
    }
  }

  // YR_STRING records and their bytes (SZ pool)
  std::vector<yr_amd_string> st(n_strings ? n_strings : 1);
  std::vector<uint8_t> blob;
  for (uint32_t k = 0; k < n_strings; ++k) {
    const uint8_t* s = a.data[kStringsTable] + (uint64_t)k * kStringSize;
    const int32_t len = rd<int32_t>(s + 20);
    Ref rstr;
    if (len < 0 || !a.ref(kStringsTable, (uint64_t)k * kStringSize + 24, rstr))
      return YR_AMD_INVALID_ARGUMENT;
    st[k].flags = rd<uint32_t>(s);
    st[k].length = (uint32_t)len;
    st[k].fixed_offset = rd<int64_t>(s + 8);
    st[k].bytes_offset = blob.size();
    if (len > 0) {
      const uint8_t* b =
          rstr.null() || rstr.buffer != kSzPool ? nullptr : a.at(rstr.buffer, rstr.offset, (uint64_t)len);
      if (b == nullptr) return YR_AMD_INVALID_ARGUMENT;
      blob.insert(blob.end(), b, b + len);
    }
  }

  yr_amd_tables* t = nullptr;
  r = yr_amd_tables_create(T.data(), M.data(), n_slots, nx.data(), bt.data(), n_pool, device, &t);
  if (r) return r;
  if (device >= 0) {
    // C-locale yr_lowercase (libyara.c:258): the compiled file carries no locale
    uint8_t lower[256];
    for (int i = 0; i < 256; ++i) lower[i] = (uint8_t)(i >= 'A' && i <= 'Z' ? i + 32 : i);
    r = yr_amd_tables_set_strings(t, ps.data(), n_pool, st.data(), n_strings, blob.data(),
                                  blob.size(), lower);
    if (!r)
      r = yr_amd_tables_set_re_code(t, n_pool, fo.data(), fl.data(), bo.data(), bl.data(),
                                    code.data(), code.size());
    if (r) {
      yr_amd_tables_destroy(t);
      return r;
    }
  }
  *tables = t;
  return YR_AMD_SUCCESS;
}
