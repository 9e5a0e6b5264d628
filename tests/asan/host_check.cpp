// Host-code sanitizer driver (ASan + UBSan build of libyara_amd's host side:
// tables.cpp flattening, yarc.cpp parsing, scanner.cpp replay and regexp
// program validation).  Test infrastructure: tests/test_asan.py builds it
// with yara_amd/csrc/Makefile's `asan` target and runs it on CPU -- no GPU
// is touched (device = -1 tables only).
//
//   host_check tables <dir>   T.bin M.bin nx.bin bt.bin data.bin expect.txt:
//                             flatten, walk (restated scanner.c:72-163
//                             candidate rule) + yr_amd_replay, compare the
//                             verify-call count with expect.txt
//   host_check yarc <file> <mutations> <seed>
//                             load the .yarc, then <mutations> mutated copies
//                             (byte flips, truncations, splices); every load
//                             must return (any error code), never fault
//   host_check re <code.bin> every offset of a program blob through
//                             yr_amd_re_code_extent (malformed programs)
//   host_check copypool <jobs> <seed> [first generation]
//                             hostio.h CopyPool: <jobs> back-to-back copies
//                             of 8-40 MiB (the parallel path), some with a copy
//                             function that fails one chunk; every job must
//                             copy all its bytes and report exactly its failure
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/yara_amd.h"
#include "../../yara_amd/csrc/hostio.h"

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

template <typename T>
static std::vector<T> slurp_as(const std::string& path) {
  std::vector<uint8_t> b = slurp(path.c_str());
  std::vector<T> v(b.size() / sizeof(T));
  if (!v.empty()) memcpy(v.data(), b.data(), v.size() * sizeof(T));
  return v;
}

static uint32_t step(const std::vector<uint32_t>& T, uint32_t s, uint8_t c) {
  const uint32_t idx = (uint32_t)c + 1;
  uint32_t t = T[s + idx];
  while ((t & 0x1FFu) != idx) {
    if (s == 0) return 0;
    s = T[s] >> 9;
    t = T[s + idx];
  }
  return t >> 9;
}

static int count_cb(void* user, uint32_t, uint64_t) {
  ++*(uint64_t*)user;
  return 0;
}

static int run_tables(const std::string& d) {
  auto T = slurp_as<uint32_t>(d + "/T.bin");
  auto M = slurp_as<uint32_t>(d + "/M.bin");
  auto nx = slurp_as<uint32_t>(d + "/nx.bin");
  auto bt = slurp_as<uint16_t>(d + "/bt.bin");
  auto data = slurp(( d + "/data.bin").c_str());
  unsigned long long expect = 0;
  FILE* f = fopen((d + "/expect.txt").c_str(), "r");
  if (!f || fscanf(f, "%llu", &expect) != 1) return 2;
  fclose(f);
  yr_amd_tables* t = nullptr;
  int r = yr_amd_tables_create(T.data(), M.data(), (uint32_t)T.size(), nx.data(), bt.data(),
                               (uint32_t)nx.size(), -1, &t);
  if (r) {
    fprintf(stderr, "tables_create %d\n", r);
    return 1;
  }
  yr_amd_tables_info info;
  if (yr_amd_tables_get_info(t, &info)) return 1;
  std::vector<uint64_t> pos;
  uint32_t s = 0;
  for (size_t i = 0; i <= data.size(); ++i) {
    if (M[s]) pos.push_back(i);
    if (i < data.size()) s = step(T, s, data[i]);
  }
  uint64_t calls = 0;
  r = yr_amd_replay(t, data.data(), data.size(), pos.data(), pos.size(),
                    info.root_accepting ? 1 : 0, count_cb, &calls);
  yr_amd_tables_destroy(t);
  printf("tables: %zu candidates, %llu verify calls (expect %llu), rc %d\n", pos.size(),
         (unsigned long long)calls, expect, r);
  return (r == 0 && calls == expect) ? 0 : 1;
}

static uint64_t rng = 88172645463325252ull;
static uint64_t next() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

static int run_yarc(const char* path, int mutations, uint64_t seed) {
  std::vector<uint8_t> good = slurp(path);
  rng ^= seed * 0x9E3779B97F4A7C15ull;
  yr_amd_tables* t = nullptr;
  int r = yr_amd_tables_load_yarc(good.data(), good.size(), -1, &t);
  if (r) {
    fprintf(stderr, "good file rejected: %d\n", r);
    return 1;
  }
  yr_amd_tables_destroy(t);
  int accepted = 0;
  for (int m = 0; m < mutations; ++m) {
    std::vector<uint8_t> b = good;
    switch (next() % 4) {
      case 0:   // byte flips
        for (int k = 0, n = 1 + (int)(next() % 8); k < n; ++k) b[next() % b.size()] ^= (uint8_t)(1 + next() % 255);
        break;
      case 1:   // truncation
        b.resize(next() % b.size());
        break;
      case 2: {   // a 32-bit field overwritten with a large value
        size_t o = next() % (b.size() - 4) & ~(size_t)3;
        uint32_t v = (uint32_t)next() | 0x80000000u;
        memcpy(&b[o], &v, 4);
        break;
      }
      default: {   // splice: copy a range elsewhere
        size_t a = next() % b.size(), c = next() % b.size(), n = next() % 64;
        for (size_t k = 0; k < n && a + k < b.size() && c + k < b.size(); ++k) b[c + k] = b[a + k];
      }
    }
    // exact-size heap copy so any overread past the end is caught
    uint8_t* p = (uint8_t*)malloc(b.size() ? b.size() : 1);
    if (!b.empty()) memcpy(p, b.data(), b.size());
    t = nullptr;
    r = yr_amd_tables_load_yarc(p, b.size(), -1, &t);
    if (r == 0) {
      ++accepted;
      yr_amd_tables_info info;
      yr_amd_tables_get_info(t, &info);
      yr_amd_tables_destroy(t);
    }
    free(p);
  }
  printf("yarc %s: %d mutations, %d accepted\n", path, mutations, accepted);
  return 0;
}

static int run_re(const char* path) {
  std::vector<uint8_t> code = slurp(path);
  int ok = 0;
  for (size_t o = 0; o < code.size(); ++o) {
    uint8_t* p = (uint8_t*)malloc(code.size() - o);
    memcpy(p, code.data() + o, code.size() - o);
    uint32_t ext = 0;
    if (yr_amd_re_code_extent(p, code.size() - o, &ext) == 0) {
      ++ok;
      if (ext > code.size() - o) return 1;
    }
    free(p);
  }
  printf("re: %zu offsets, %d well-formed programs\n", code.size(), ok);
  return 0;
}

struct FailAt {
  const uint8_t* src;
  size_t bad;   // fail the chunk holding this source offset (SIZE_MAX: none)
};
static int fail_copy(void* user, void* dst, const void* src, size_t n) {
  const FailAt* f = (const FailAt*)user;
  const size_t off = (const uint8_t*)src - f->src;
  memcpy(dst, src, n);   // (a failing chunk still writes: the caller must not care)
  return f->bad >= off && f->bad < off + n ? 1 : 0;
}

static int run_copypool(int jobs, uint64_t seed, uint64_t first_gen) {
  yamd::CopyPool pool(7, first_gen);
  const size_t max = 40u << 20;
  std::vector<uint8_t> src(max), dst(max);
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (size_t i = 0; i < max; i += 8) {
    const uint64_t v = rnd();
    memcpy(&src[i], &v, 8);
  }
  int failures = 0;
  for (int j = 0; j < jobs; ++j) {
    const size_t size = (8u << 20) + rnd() % (max - (8u << 20));
    const size_t so = rnd() % 64, dofs = rnd() % 64;   // unaligned starts
    const size_t n = size - 64;
    memset(dst.data(), 0, max);
    FailAt f{src.data() + so, (rnd() % 3 == 0) ? rnd() % n : SIZE_MAX};
    yamd::CopyFn fn;
    fn.fn = fail_copy;
    fn.user = &f;
    const bool ok = pool.copy(dst.data() + dofs, src.data() + so, n, fn);
    if (ok != (f.bad == SIZE_MAX)) {
      fprintf(stderr, "job %d: copy returned %d, injected failure at %zu\n", j, ok, f.bad);
      return 1;
    }
    if (memcmp(dst.data() + dofs, src.data() + so, n) != 0) {
      fprintf(stderr, "job %d: bytes differ\n", j);
      return 1;
    }
    failures += !ok;
  }
  printf("%d copy jobs, %d with an injected failure: ok\n", jobs, failures);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 4 && !strcmp(argv[1], "copypool"))
    return run_copypool(atoi(argv[2]), strtoull(argv[3], 0, 10), argc >= 5 ? strtoull(argv[4], 0, 10) : 0);
  if (argc >= 3 && !strcmp(argv[1], "tables")) return run_tables(argv[2]);
  if (argc >= 5 && !strcmp(argv[1], "yarc")) return run_yarc(argv[2], atoi(argv[3]), strtoull(argv[4], 0, 10));
  if (argc >= 3 && !strcmp(argv[1], "re")) return run_re(argv[2]);
  fprintf(stderr, "usage: host_check tables <dir> | yarc <file> <n> <seed> | re <code.bin>\n");
  return 2;
}
