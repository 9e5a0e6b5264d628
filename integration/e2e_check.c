/*
 * e2e_check -- end-to-end match-set parity: stock libyara vs the GPU driver.
 *
 * Test infrastructure: compiles a rule file with the stock libyara compiler,
 * scans the same data twice --
 *   stock:  yr_scanner_scan_mem[_blocks]          (scanner.c:417/:633)
 *   gpu:    yr_gpu_scanner_scan_mem[_blocks]      (integration/yr_gpu_scanner.c)
 * -- and compares the complete match sets ({string idx, base+offset, length,
 * xor key} of every match of every string, private ones included) and the
 * per-rule RULE_MATCHING / RULE_NOT_MATCHING reports.  Prints one JSON line.
 *
 *   e2e_check <rules.yar> <data file | xs:SEED:SIZE> [block_size overlap]
 *   (E2E_PREVERIFY=0: GPU path without the on-device literal pre-verification)
 *   E2E_MODE = mem (default) | file | fd | proc: the entry point compared --
 *   yr_scanner_scan_mem[_blocks] / _scan_file / _scan_fd / _scan_proc against
 *   the shim's twins (scanner.c:417-722).  proc scans a stopped child process
 *   that holds the data (forked before any GPU initialisation).
 *   E2E_REPEAT = N: time N more runs of each side, report the minimum.
 *   E2E_FAST=1: SCAN_FLAGS_FAST_MODE; E2E_ABORT=n: the callback returns
 *   CALLBACK_ABORT on the n-th matching rule (scanner.c:540-548).
 *   E2E_TIMEOUT=s: yr_scanner_set_timeout(s); E2E_SLEEP_TOO_MANY=ms: the
 *   callback sleeps on CALLBACK_MSG_TOO_MANY_MATCHES (a deterministic way to
 *   exceed the timeout in the middle of a block, scanner.c:74-81).
 *   E2E_MODE=truncmap: both sides scan_mem an mmap of the data file whose
 *   file was truncated to half its size (the tail faults: scanner.c:493-496
 *   maps that to ERROR_COULD_NOT_MAP_FILE).
 *   E2E_DEVICES=d0,d1,...: the GPU side on several devices (a device may
 *   repeat: logical devices on one GPU), blocks of at least E2E_MULTI_MIN
 *   bytes split across them (yr_gpu_rules_create_multi).
 *   E2E_THREADS=n: afterwards n threads, each with its own YR_SCANNER and
 *   YR_GPU_SCANNER on the one shared YR_GPU_RULES, scan the data
 *   E2E_THREAD_REPS times concurrently; every result must equal stock's
 *   (docs/capi.rst:330-347, cli/yara.c:1564-1608).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>
#include <yara.h>

#include "yr_gpu_scanner.h"

typedef struct
{
  uint64_t off;
  uint32_t s, len, xk, pad; /* no implicit padding: records are memcmp'd */
} rec;

typedef struct
{
  YR_RULES* rules;
  rec* r;
  size_t n, cap;
  uint8_t* rule_msg; /* 1 matching, 2 not matching */
  int dumped;
  int finished;
  int abort_after; /* E2E_ABORT=n: CALLBACK_ABORT on the n-th RULE_MATCHING */
  int n_matching;
  int too_many;    /* CALLBACK_MSG_TOO_MANY_MATCHES messages seen */
  uint64_t* atom_matches; /* E2E profiling build: per rule, after the scan */
} collect;

static void push(collect* c, rec x)
{
  if (c->n == c->cap)
  {
    c->cap = c->cap ? 2 * c->cap : 1024;
    c->r = (rec*) realloc(c->r, c->cap * sizeof(rec));
  }
  c->r[c->n++] = x;
}

static int cb(YR_SCAN_CONTEXT* ctx, int msg, void* data, void* user)
{
  collect* c = (collect*) user;
  if (msg == CALLBACK_MSG_RULE_MATCHING || msg == CALLBACK_MSG_RULE_NOT_MATCHING)
  {
    YR_RULE* rule = (YR_RULE*) data;
    c->rule_msg[rule - c->rules->rules_table] =
        msg == CALLBACK_MSG_RULE_MATCHING ? 1 : 2;
    if (!c->dumped)
    {
      for (uint32_t k = 0; k < c->rules->num_strings; k++)
        for (YR_MATCH* m = ctx->matches[k].head; m != NULL; m = m->next)
        {
          rec x = {(uint64_t) (m->base + m->offset), k, (uint32_t) m->match_length,
                   m->xor_key, 0};
          push(c, x);
        }
      c->dumped = 1;
    }
  }
  else if (msg == CALLBACK_MSG_SCAN_FINISHED)
  {
    c->finished = 1;
  }
  else if (msg == CALLBACK_MSG_TOO_MANY_MATCHES)
  {
    c->too_many++;
    const char* sl = getenv("E2E_SLEEP_TOO_MANY");
    if (sl != NULL) usleep(1000 * atoi(sl));
  }
  if (msg == CALLBACK_MSG_RULE_MATCHING && c->abort_after > 0 &&
      ++c->n_matching >= c->abort_after)
    return CALLBACK_ABORT;
  return CALLBACK_CONTINUE;
}

static void xorshift_fill(uint8_t* buf, size_t n, uint64_t seed)
{
  uint64_t x = 0x9E3779B97F4A7C15ull * seed;
  for (size_t i = 0; i < n; i++)
  {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    buf[i] = (uint8_t) (x >> 24);
  }
}

static uint8_t* load(const char* spec, size_t* n)
{
  if (strncmp(spec, "xs:", 3) == 0)
  {
    unsigned long long seed, sz;
    sscanf(spec + 3, "%llu:%llu", &seed, &sz);
    uint8_t* b = (uint8_t*) malloc(sz ? sz : 1);
    xorshift_fill(b, sz, seed);
    *n = sz;
    return b;
  }
  FILE* f = fopen(spec, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* b = (uint8_t*) malloc(sz ? sz : 1);
  if (fread(b, 1, sz, f) != (size_t) sz) return NULL;
  fclose(f);
  *n = (size_t) sz;
  return b;
}

/* overlapping block iterator (tests/util.c:136-209 semantics) */
typedef struct
{
  const uint8_t* data;
  size_t size, bsize, overlap, next_base;
  YR_MEMORY_BLOCK blk;
} blk_iter;

static const uint8_t* blk_fetch(YR_MEMORY_BLOCK* b)
{
  return ((blk_iter*) b->context)->data + b->base;
}

static YR_MEMORY_BLOCK* blk_next(YR_MEMORY_BLOCK_ITERATOR* iter)
{
  blk_iter* it = (blk_iter*) iter->context;
  if (it->next_base >= it->size) return NULL;
  size_t base = it->next_base;
  size_t len = it->size - base < it->bsize ? it->size - base : it->bsize;
  it->blk.base = base;
  it->blk.size = len;
  it->blk.context = it;
  it->blk.fetch_data = blk_fetch;
  it->next_base = base + len >= it->size ? it->size : base + len - it->overlap;
  return &it->blk;
}

static YR_MEMORY_BLOCK* blk_first(YR_MEMORY_BLOCK_ITERATOR* iter)
{
  ((blk_iter*) iter->context)->next_base = 0;
  return blk_next(iter);
}

static uint64_t blk_file_size(YR_MEMORY_BLOCK_ITERATOR* iter)
{
  return ((blk_iter*) iter->context)->size;
}

static int cmp_rec(const void* a, const void* b)
{
  return memcmp(a, b, sizeof(rec));
}

static double now(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static const char* g_mode = "mem";
static const char* g_path = NULL; /* file / fd modes */
static int g_pid = 0;             /* proc mode */

static int run(YR_RULES* rules, YR_GPU_SCANNER* gs, const uint8_t* data, size_t n,
               size_t bsize, size_t overlap, collect* c, double* secs)
{
  YR_SCANNER* sc;
  int r = yr_scanner_create(rules, &sc);
  if (r) return r;
  int flags = SCAN_FLAGS_REPORT_RULES_MATCHING | SCAN_FLAGS_REPORT_RULES_NOT_MATCHING;
  if (getenv("E2E_FAST") && strcmp(getenv("E2E_FAST"), "1") == 0) flags |= SCAN_FLAGS_FAST_MODE;
  yr_scanner_set_flags(sc, flags);
  if (getenv("E2E_TIMEOUT")) yr_scanner_set_timeout(sc, atoi(getenv("E2E_TIMEOUT")));
  c->abort_after = getenv("E2E_ABORT") ? atoi(getenv("E2E_ABORT")) : 0;
  yr_scanner_set_callback(sc, cb, c);
#ifdef E2E_BLOCK_SCANNER
  /* libyara patched with integration/libyara-block-scanner.patch: the GPU
   * side runs through libyara's OWN entry points, the block scanner attached */
  if (gs != NULL)
  {
    r = yr_gpu_scanner_attach(sc, gs);
    if (r) return r;
    gs = NULL;
  }
#endif
  double t0 = now();
  if (strcmp(g_mode, "file") == 0 && c->rules != NULL && data == NULL)
  {
    r = gs ? yr_gpu_scanner_scan_file(sc, gs, g_path) : yr_scanner_scan_file(sc, g_path);
  }
  else if (strcmp(g_mode, "fd") == 0 && data == NULL)
  {
    FILE* f = fopen(g_path, "rb");
    r = gs ? yr_gpu_scanner_scan_fd(sc, gs, fileno(f)) : yr_scanner_scan_fd(sc, fileno(f));
    fclose(f);
  }
  else if (strcmp(g_mode, "proc") == 0 && data == NULL)
  {
    r = gs ? yr_gpu_scanner_scan_proc(sc, gs, g_pid) : yr_scanner_scan_proc(sc, g_pid);
  }
  else if (bsize == 0)
  {
    r = gs ? yr_gpu_scanner_scan_mem(sc, gs, data, n) : yr_scanner_scan_mem(sc, data, n);
  }
  else
  {
    blk_iter it = {data, n, bsize, overlap, 0};
    YR_MEMORY_BLOCK_ITERATOR iter = {&it, blk_first, blk_next, blk_file_size, ERROR_SUCCESS};
    r = gs ? yr_gpu_scanner_scan_mem_blocks(sc, gs, &iter) : yr_scanner_scan_mem_blocks(sc, &iter);
  }
  *secs = now() - t0;
#ifdef YR_PROFILING_ENABLED
  /* libyara's per-rule verify-call counts (scan.c:1083) of this scan */
  free(c->atom_matches);
  c->atom_matches = (uint64_t*) calloc(rules->num_rules + 1, sizeof(uint64_t));
  for (uint32_t i = 0; i < rules->num_rules; i++)
    c->atom_matches[i] = sc->profiling_info[i].atom_matches;
#endif
  yr_scanner_destroy(sc);
  return r;
}

typedef struct
{
  YR_RULES* rules;
  YR_GPU_RULES* gr;
  const uint8_t* data;
  size_t n, bsize, overlap;
  const collect* want;
  int reps;
  int ok;
} thread_job;

static void* thread_main(void* arg)
{
  thread_job* j = (thread_job*) arg;
  YR_GPU_SCANNER* gs;
  j->ok = 0;
  if (yr_gpu_scanner_create(j->gr, &gs) != 0) return NULL;
  int good = 1;
  for (int k = 0; k < j->reps && good; k++)
  {
    collect x = {j->rules};
    x.rule_msg = (uint8_t*) calloc(j->rules->num_rules + 1, 1);
    double t;
    int r = run(j->rules, gs, j->data, j->n, j->bsize, j->overlap, &x, &t);
    qsort(x.r, x.n, sizeof(rec), cmp_rec);
    good = r == 0 && x.n == j->want->n &&
           (x.n == 0 || memcmp(x.r, j->want->r, x.n * sizeof(rec)) == 0) &&
           memcmp(x.rule_msg, j->want->rule_msg, j->rules->num_rules) == 0;
    free(x.r);
    free(x.rule_msg);
  }
  yr_gpu_scanner_destroy(gs);
  j->ok = good;
  return NULL;
}

int main(int argc, char** argv)
{
  if (argc < 3)
  {
    fprintf(stderr, "usage: e2e_check rules data [block overlap]\n");
    return 2;
  }
  size_t bsize = argc > 4 ? strtoull(argv[3], NULL, 10) : 0;
  size_t overlap = argc > 4 ? strtoull(argv[4], NULL, 10) : 0;
  yr_initialize();
  YR_COMPILER* comp;
  YR_RULES* rules;
  FILE* f = fopen(argv[1], "r");
  if (!f || yr_compiler_create(&comp) || yr_compiler_add_file(comp, f, NULL, argv[1]) ||
      yr_compiler_get_rules(comp, &rules))
  {
    fprintf(stderr, "rule compilation failed\n");
    return 2;
  }
  size_t n;
  uint8_t* data = load(argv[2], &n);
  if (!data)
  {
    fprintf(stderr, "cannot load data\n");
    return 2;
  }
  if (getenv("E2E_MODE")) g_mode = getenv("E2E_MODE");
  char tmpl[] = "/tmp/e2e_check_XXXXXX";
  const uint8_t* scan_data = data;
  if (strcmp(g_mode, "truncmap") == 0)
  {
    int fd = mkstemp(tmpl);
    if (fd < 0 || write(fd, data, n) != (ssize_t) n) return 2;
    void* m = mmap(NULL, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED || ftruncate(fd, n / 2) != 0) return 2;
    close(fd);
    g_path = tmpl;
    scan_data = (const uint8_t*) m;
    g_mode = "mem";
  }
  else if (strcmp(g_mode, "file") == 0 || strcmp(g_mode, "fd") == 0)
  {
    int fd = mkstemp(tmpl);
    if (fd < 0 || write(fd, data, n) != (ssize_t) n) return 2;
    close(fd);
    g_path = tmpl;
  }
  else if (strcmp(g_mode, "proc") == 0)
  {
    /* before any GPU initialisation: the child's address space holds the
     * data and no device mappings */
    g_pid = fork();
    if (g_pid < 0) return 2;
    if (g_pid == 0)
    {
      volatile uint8_t sink = 0;
      for (size_t i = 0; i < n; i += 4096) sink ^= data[i]; /* keep it resident */
      (void) sink;
      raise(SIGSTOP);
      _exit(0);
    }
    int st;
    waitpid(g_pid, &st, WUNTRACED);
  }
  int scan_whole = strcmp(g_mode, "mem") != 0; /* entry points take no data pointer */
  YR_GPU_RULES* gr;
  YR_GPU_SCANNER* gs;
  /* E2E_DEVICES=d0,d1,...: the multi-device path (yr_gpu_rules_create_multi;
   * devices may repeat), blocks of at least E2E_MULTI_MIN bytes split */
  int devs[YR_AMD_MAX_DEVICES] = {0};
  int n_devs = 1;
  if (getenv("E2E_DEVICES"))
  {
    n_devs = 0;
    for (const char* p = getenv("E2E_DEVICES"); *p && n_devs < YR_AMD_MAX_DEVICES;)
    {
      devs[n_devs++] = (int) strtol(p, (char**) &p, 10);
      if (*p == ',') p++;
    }
  }
  int r = yr_gpu_rules_create_multi(rules, devs, n_devs, &gr);
  if (r == 0) r = yr_gpu_scanner_create(gr, &gs);
  if (r == 0 && getenv("E2E_MULTI_MIN"))
    yr_gpu_scanner_set_multi_min_block(gs, strtoull(getenv("E2E_MULTI_MIN"), NULL, 10));
  const char* pv = getenv("E2E_PREVERIFY"); /* "0": replay the full candidate stream */
  if (r == 0 && pv != NULL && strcmp(pv, "0") == 0) yr_gpu_scanner_set_preverify(gs, 0);
  if (r)
  {
    fprintf(stderr, "gpu setup failed: %d\n", r);
    return 3;
  }
  collect a = {rules}, b = {rules};
  a.rule_msg = (uint8_t*) calloc(rules->num_rules + 1, 1);
  b.rule_msg = (uint8_t*) calloc(rules->num_rules + 1, 1);
  double ts, tg, tw;
  collect warm = {rules};
  warm.rule_msg = (uint8_t*) calloc(rules->num_rules + 1, 1);
  const char* mode = g_mode;
  g_mode = "mem";
  run(rules, gs, data, n < 4096 ? n : 4096, 0, 0, &warm, &tw); /* GPU warm-up */
  g_mode = mode;
  const uint8_t* d_arg = scan_whole ? NULL : scan_data;
  int rs = run(rules, NULL, d_arg, n, bsize, overlap, &a, &ts);
  double tm0[3], tm1[3], tmin[3] = {0, 0, 0};
  yr_gpu_scanner_timing(gs, tm0);
  int rg = run(rules, gs, d_arg, n, bsize, overlap, &b, &tg);
  yr_gpu_scanner_timing(gs, tm1);
  for (int k = 0; k < 3; k++) tmin[k] = tm1[k] - tm0[k];
  /* E2E_REPEAT=N: N more timed runs of each side (steady state: warm caches,
   * allocated staging); the reported times are the minimum */
  int reps = getenv("E2E_REPEAT") ? atoi(getenv("E2E_REPEAT")) : 0;
  for (int k = 0; k < reps; k++)
  {
    double t;
    collect x = {rules};
    x.rule_msg = (uint8_t*) calloc(rules->num_rules + 1, 1);
    run(rules, NULL, d_arg, n, bsize, overlap, &x, &t);
    if (t < ts) ts = t;
    free(x.r);
    x.n = x.cap = 0;
    x.r = NULL;
    x.dumped = 0;
    yr_gpu_scanner_timing(gs, tm0);
    run(rules, gs, d_arg, n, bsize, overlap, &x, &t);
    yr_gpu_scanner_timing(gs, tm1);
    if (t < tg)
    {
      tg = t;
      for (int q = 0; q < 3; q++) tmin[q] = tm1[q] - tm0[q];
    }
    free(x.r);
    free(x.rule_msg);
  }
  int threads = getenv("E2E_THREADS") ? atoi(getenv("E2E_THREADS")) : 0;
  int threads_ok = 1;
  if (threads > 0)
  {
    thread_job jobs[32];
    pthread_t tid[32];
    if (threads > 32) threads = 32;
    collect want = a;
    qsort(want.r, want.n, sizeof(rec), cmp_rec);
    for (int k = 0; k < threads; k++)
    {
      thread_job j = {rules, gr, d_arg, n, bsize, overlap, &want,
                      getenv("E2E_THREAD_REPS") ? atoi(getenv("E2E_THREAD_REPS")) : 4, 0};
      jobs[k] = j;
      pthread_create(&tid[k], NULL, thread_main, &jobs[k]);
    }
    for (int k = 0; k < threads; k++)
    {
      pthread_join(tid[k], NULL);
      threads_ok &= jobs[k].ok;
    }
  }
  if (g_pid > 0)
  {
    kill(g_pid, SIGKILL);
    waitpid(g_pid, NULL, 0);
  }
  if (g_path) unlink(g_path);
  qsort(a.r, a.n, sizeof(rec), cmp_rec);
  qsort(b.r, b.n, sizeof(rec), cmp_rec);
  int same_matches = a.n == b.n && (a.n == 0 || memcmp(a.r, b.r, a.n * sizeof(rec)) == 0);
  int same_rules = memcmp(a.rule_msg, b.rule_msg, rules->num_rules) == 0;
  int n_match_rules = 0;
  for (uint32_t i = 0; i < rules->num_rules; i++) n_match_rules += a.rule_msg[i] == 1;
#ifdef YR_PROFILING_ENABLED
  /* profiling-counter parity: every rule's atom_matches, stock vs GPU */
  uint64_t am_stock = 0, am_gpu = 0;
  int am_equal = a.atom_matches != NULL && b.atom_matches != NULL;
  for (uint32_t i = 0; a.atom_matches != NULL && b.atom_matches != NULL && i < rules->num_rules; i++)
  {
    am_stock += a.atom_matches[i];
    am_gpu += b.atom_matches[i];
    if (a.atom_matches[i] != b.atom_matches[i]) am_equal = 0;
  }
  printf("{\"profiling\": true, \"atom_matches_equal\": %s, \"atom_matches_stock\": %llu, "
         "\"atom_matches_gpu\": %llu}\n",
         am_equal ? "true" : "false", (unsigned long long) am_stock, (unsigned long long) am_gpu);
#endif
  printf("{\"mode\": \"%s\", \"size\": %zu, \"block\": %zu, \"rc_stock\": %d, \"rc_gpu\": %d, "
         "\"matches_stock\": %zu, \"matches_gpu\": %zu, \"rules_matching\": %d, "
         "\"same_matches\": %s, \"same_rule_reports\": %s, \"finished\": [%d, %d], "
         "\"stock_s\": %.4f, \"gpu_s\": %.4f, \"too_many\": [%d, %d], \"threads\": %d, "
         "\"threads_ok\": %s, \"devices\": %d, \"multi_blocks\": %llu, "
         "\"gpu_copy_s\": %.4f, \"gpu_wait_s\": %.4f, \"gpu_replay_s\": %.4f}\n",
         g_mode, n, bsize, rs, rg, a.n, b.n, n_match_rules, same_matches ? "true" : "false",
         same_rules ? "true" : "false", a.finished, b.finished, ts, tg, a.too_many, b.too_many,
         threads, threads_ok ? "true" : "false", n_devs,
         (unsigned long long) yr_gpu_scanner_multi_blocks(gs), tmin[0], tmin[1], tmin[2]);
  yr_gpu_scanner_destroy(gs);
  yr_gpu_rules_destroy(gr);
  yr_rules_destroy(rules);
  yr_compiler_destroy(comp);
  yr_finalize();
  return (rs == rg && same_matches && same_rules && threads_ok) ? 0 : 1;
}
