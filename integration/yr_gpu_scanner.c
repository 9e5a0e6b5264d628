/*
 * yr_gpu_scanner.c -- libyara-side integration of the MI355X atom scanner.
 *
 * This is the code a libyara maintainer adds: it is compiled
 * against libyara's own headers and linked with an UNMODIFIED libyara (here
 * the stock reference build, oracle/_ref/libyara_ref.so) and libyara_amd.so.
 *
 * libyara's per-block walk _yr_scanner_scan_mem_block (scanner.c:45-176) is
 * static, so the driver that calls it, yr_scanner_scan_mem_blocks
 * (scanner.c:417-583), is re-hosted here step for step; the only change is
 * the per-block call (scanner.c:493-496), which becomes
 *     the block pipeline (yr_amd_pipeline_*: copy, H2D, GPU candidate stream
 *       and on-device literal pre-verification, which drops the calls that
 *       provably have no effect, scan.c:887-990 / :1013 / :1023), two blocks
 *       in flight while the host replays the previous one
 *  -> the remaining calls, in the reference's order, into the unmodified
 *     verifier yr_scan_verify_match (scan.c:992)
 * or, with pre-verification off, one block at a time: the full candidate
 * stream (yr_amd_scan_block) replayed by yr_amd_replay.  Either way followed,
 * as in the reference, by yr_execute_code (exec.c:418) and the rule-report
 * loop (scanner.c:524-556).  scan_file / scan_fd / scan_proc wrap it exactly
 * like scanner.c:674-722.
 *
 * Built with -DYR_HAVE_BLOCK_SCANNER against a libyara patched with
 * integration/libyara-block-scanner.patch, it also provides
 * yr_gpu_scanner_attach(): the patched libyara's own driver then calls the
 * per-block replacement here, and the re-hosted driver above is not needed.
 */
#include "yr_gpu_scanner.h"

#include <pthread.h>
#include <setjmp.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <yara.h>
#include <yara/arena.h>
#include <yara/compiler.h>
#include <yara/exec.h>
#include <yara/exefiles.h>
#include <yara/globals.h>
#include <yara/filemap.h>
#include <yara/notebook.h>
#include <yara/proc.h>
#include <yara/re.h>
#include <yara/scan.h>
#include <yara/stopwatch.h>

#include <time.h>

#include "exception.h" /* libyara/exception.h: YR_TRYCATCH (exception.h:150-185) */

struct YR_GPU_RULES
{
  YR_RULES* rules;
  yr_amd_tables* tables;   /* == dev_tables[0]: single-device scans */
  uint32_t n_devices;
  yr_amd_tables* dev_tables[YR_AMD_MAX_DEVICES]; /* yr_gpu_rules_create_multi */
};

struct YR_GPU_SCANNER
{
  YR_GPU_RULES* gpu_rules;
  yr_amd_scanner* scanner;
  uint8_t* staging; /* host copy of the block being scanned */
  size_t staging_size;
  int preverify;    /* on-device literal pre-verification (default on) */
  yr_amd_pipeline* pipe; /* blocks in flight on the GPU (preverify path) */
  uint32_t depth;
  uint32_t inflight;
  int direct;            /* single in-memory block (scan_mem): no staging copy */
  yr_amd_multi* multi;   /* n_devices > 1: a large direct block split across the devices */
  uint64_t multi_min;    /* smallest block that is split */
  uint64_t multi_blocks; /* blocks scanned across the devices (statistics) */
  int trycatch;          /* the scan's !SCAN_FLAGS_NO_TRYCATCH, for _guarded_copy */
  double t_copy, t_gpu, t_replay; /* yr_gpu_scanner_timing */
#ifdef YR_HAVE_BLOCK_SCANNER
  YR_BLOCK_SCANNER block_scanner; /* yr_gpu_scanner_attach */
#endif
};

/* Length (incl. MATCH) of a linear fast-exec program (the opcodes
 * yr_re_fast_exec runs, re.c:2150-2391), or 0. */
static uint32_t _fast_code_len(const uint8_t* code)
{
  uint32_t n = 0;
  while (n < 65536)
  {
    switch (code[n])
    {
    case RE_OPCODE_ANY: n += 1; break;
    case RE_OPCODE_LITERAL: case RE_OPCODE_NOT_LITERAL: n += 2; break;
    case RE_OPCODE_MASKED_LITERAL: case RE_OPCODE_MASKED_NOT_LITERAL: n += 3; break;
    case RE_OPCODE_REPEAT_ANY_UNGREEDY: n += 5; break;
    case RE_OPCODE_MATCH: return n + 1;
    default: return 0;
    }
  }
  return 0;
}

/* Forward/backward regexp programs of the pool entries for
 * yr_amd_tables_set_re_code (YR_AC_MATCH.forward_code / backward_code): the
 * linear fast-exec program of a hex string, or every reachable instruction of
 * another regexp's yr_re_exec program (yr_amd_re_code_extent). */
static int _attach_re_code(YR_RULES* rules, uint32_t n_pool, yr_amd_tables* t)
{
  uint32_t* a = (uint32_t*) calloc(4 * (size_t) (n_pool ? n_pool : 1), sizeof(uint32_t));
  if (a == NULL) return ERROR_INSUFFICIENT_MEMORY;
  uint32_t *fo = a, *fl = a + n_pool, *bo = a + 2 * n_pool, *bl = a + 3 * n_pool;
  uint64_t total = 0;
  const uint8_t* re_base = (const uint8_t*) yr_arena_get_ptr(rules->arena, YR_RE_CODE_SECTION, 0);
  const size_t re_size = yr_arena_get_current_offset(rules->arena, YR_RE_CODE_SECTION);
  for (uint32_t pass = 0; pass < 2; pass++)
  {
    uint8_t* code = pass ? (uint8_t*) malloc(total ? total : 1) : NULL;
    if (pass && code == NULL)
    {
      free(a);
      return ERROR_INSUFFICIENT_MEMORY;
    }
    uint64_t off = 0;
    for (uint32_t k = 0; k < n_pool; k++)
    {
      YR_AC_MATCH* m = &rules->ac_match_pool[k];
      uint32_t f = 0, b = 0;
      if ((m->string->flags & STRING_FLAGS_FAST_REGEXP) && m->forward_code != NULL)
      {
        f = _fast_code_len(m->forward_code);
        b = m->backward_code ? _fast_code_len(m->backward_code) : 0;
        if (f == 0 || (m->backward_code != NULL && b == 0)) f = b = 0;
      }
      else if (!(m->string->flags & STRING_FLAGS_LITERAL) && m->forward_code != NULL &&
               m->forward_code >= re_base && m->forward_code < re_base + re_size)
      {
        /* yr_re_exec programs: copy every instruction reachable from the start */
        int okf = yr_amd_re_code_extent(m->forward_code,
                                        (uint64_t) (re_base + re_size - m->forward_code), &f);
        int okb = ERROR_SUCCESS;
        if (m->backward_code != NULL)
          okb = m->backward_code >= re_base && m->backward_code < re_base + re_size
                    ? yr_amd_re_code_extent(m->backward_code,
                                            (uint64_t) (re_base + re_size - m->backward_code), &b)
                    : ERROR_INVALID_ARGUMENT;
        if (okf != ERROR_SUCCESS || okb != ERROR_SUCCESS) f = b = 0;
      }
      if (pass)
      {
        fo[k] = (uint32_t) off;
        fl[k] = f;
        if (f) memcpy(code + off, m->forward_code, f);
        bo[k] = (uint32_t) (off + f);
        bl[k] = b;
        if (b) memcpy(code + off + f, m->backward_code, b);
      }
      off += f + b;
    }
    if (!pass)
    {
      total = off;
      continue;
    }
    int r = yr_amd_tables_set_re_code(t, n_pool, fo, fl, bo, bl, code, total);
    free(code);
    free(a);
    return r;
  }
  free(a);
  return ERROR_INTERNAL_FATAL_ERROR;
}

/* YR_STRING records for yr_amd_tables_set_strings (types.h YR_STRING). */
static int _attach_strings(YR_RULES* rules, uint32_t n_pool, yr_amd_tables* t)
{
  uint32_t n_str = rules->num_strings;
  uint64_t n_bytes = 0;
  for (uint32_t k = 0; k < n_str; k++) n_bytes += rules->strings_table[k].length;
  uint32_t* ps = (uint32_t*) malloc(sizeof(uint32_t) * (n_pool ? n_pool : 1));
  yr_amd_string* st = (yr_amd_string*) malloc(sizeof(yr_amd_string) * (n_str ? n_str : 1));
  uint8_t* blob = (uint8_t*) malloc(n_bytes ? n_bytes : 1);
  int r = ERROR_INSUFFICIENT_MEMORY;
  if (ps != NULL && st != NULL && blob != NULL)
  {
    for (uint32_t k = 0; k < n_pool; k++)
      ps[k] = (uint32_t) (rules->ac_match_pool[k].string - rules->strings_table);
    uint64_t off = 0;
    for (uint32_t k = 0; k < n_str; k++)
    {
      YR_STRING* s = &rules->strings_table[k];
      st[k].flags = s->flags;
      st[k].length = (uint32_t) s->length;
      st[k].fixed_offset = s->fixed_offset;
      st[k].bytes_offset = off;
      if (s->length > 0) memcpy(blob + off, s->string, s->length);
      off += s->length;
    }
    r = yr_amd_tables_set_strings(t, ps, n_pool, st, n_str, blob, n_bytes, yr_lowercase);
  }
  free(ps);
  free(st);
  free(blob);
  return r;
}

/* The device tables of one YR_RULES on one device (or host-only, device < 0). */
static int _create_tables(YR_RULES* rules, int device, yr_amd_tables** out)
{
  *out = NULL;
  /* table sizes exactly as yr_rules_get_stats computes them (rules.c:442) */
  uint32_t n_slots = (uint32_t) (yr_arena_get_current_offset(
                                     rules->arena, YR_AC_TRANSITION_TABLE) /
                                 sizeof(YR_AC_TRANSITION));
  uint32_t n_pool = (uint32_t) (yr_arena_get_current_offset(
                                    rules->arena, YR_AC_STATE_MATCHES_POOL) /
                                sizeof(YR_AC_MATCH));

  uint32_t* nx = (uint32_t*) malloc(sizeof(uint32_t) * (n_pool ? n_pool : 1));
  uint16_t* bt = (uint16_t*) malloc(sizeof(uint16_t) * (n_pool ? n_pool : 1));
  if (nx == NULL || bt == NULL)
  {
    free(nx);
    free(bt);
    return ERROR_INSUFFICIENT_MEMORY;
  }
  for (uint32_t k = 0; k < n_pool; k++)
  {
    YR_AC_MATCH* m = &rules->ac_match_pool[k];
    nx[k] = m->next ? (uint32_t) (m->next - rules->ac_match_pool) + 1 : 0;
    bt[k] = m->backtrack;
  }
  yr_amd_tables* t = NULL;
  int r = yr_amd_tables_create(
      rules->ac_transition_table,
      rules->ac_match_table,
      n_slots,
      nx,
      bt,
      n_pool,
      device,
      &t);
  free(nx);
  free(bt);
  if (r == ERROR_SUCCESS && device >= 0) r = _attach_strings(rules, n_pool, t);
  if (r == ERROR_SUCCESS && device >= 0) r = _attach_re_code(rules, n_pool, t);
#ifdef YR_PROFILING_ENABLED
  /* libyara counts every verify call past its early returns: pre-verification
   * reports the dropped ones as count-only records (_count_only) */
  if (r == ERROR_SUCCESS && device >= 0) r = yr_amd_tables_set_profiling(t, 1);
#endif
  if (r != ERROR_SUCCESS)
  {
    yr_amd_tables_destroy(t);
    return r;
  }
  *out = t;
  return ERROR_SUCCESS;
}

int yr_gpu_rules_create_multi(
    YR_RULES* rules,
    const int* devices,
    int n_devices,
    YR_GPU_RULES** out)
{
  *out = NULL;
  if (devices == NULL || n_devices < 1 || n_devices > YR_AMD_MAX_DEVICES)
    return ERROR_INVALID_ARGUMENT;
  if (n_devices > 1)
    for (int k = 0; k < n_devices; k++)
      if (devices[k] < 0) return ERROR_INVALID_ARGUMENT;
  YR_GPU_RULES* g = (YR_GPU_RULES*) calloc(1, sizeof(YR_GPU_RULES));
  if (g == NULL) return ERROR_INSUFFICIENT_MEMORY;
  int r = ERROR_SUCCESS;
  for (int k = 0; k < n_devices && r == ERROR_SUCCESS; k++)
  {
    r = _create_tables(rules, devices[k], &g->dev_tables[k]);
    if (r == ERROR_SUCCESS) g->n_devices++;
  }
  if (r != ERROR_SUCCESS)
  {
    yr_gpu_rules_destroy(g);
    return r;
  }
  g->tables = g->dev_tables[0];
  g->rules = rules;
  *out = g;
  return ERROR_SUCCESS;
}

int yr_gpu_rules_create(YR_RULES* rules, int device, YR_GPU_RULES** out)
{
  return yr_gpu_rules_create_multi(rules, &device, 1, out);
}

void yr_gpu_rules_destroy(YR_GPU_RULES* g)
{
  if (g == NULL) return;
  for (uint32_t k = 0; k < g->n_devices; k++) yr_amd_tables_destroy(g->dev_tables[k]);
  free(g);
}

/* The copy that moves a block into the library's pinned staging
 * (yr_amd_copy_fn): memcpy inside YR_TRYCATCH on whichever thread runs it --
 * the caller's or one of the library's helpers -- so a block that faults while
 * it is copied (a file mapping truncated underneath) fails the copy, and the
 * scan returns ERROR_COULD_NOT_MAP_FILE exactly as scanner.c:493-496 maps a
 * fault of the walk, instead of SIGBUS on a helper thread. */
/* YR_TRYCATCH (exception.h:150-185) saves the SIGBUS/SIGSEGV actions it finds
 * and restores them when it ends.  Several helpers copying at once would
 * restore each other's handler in any order -- one helper's exit can uninstall
 * the handler while another still copies.  So the copies share one counted
 * installation of libyara's exception_handler: the first copy in installs it,
 * the last one out restores what was there, and the handler is installed only
 * while some copy runs (not across the GPU work that follows the copies). */
static pthread_mutex_t _sig_mu = PTHREAD_MUTEX_INITIALIZER;
static int _sig_users = 0;
static struct sigaction _sig_old_bus, _sig_old_segv;

static void _sig_install(struct sigaction* old_bus, struct sigaction* old_segv)
{
  struct sigaction act;
  memset(&act, 0, sizeof(act));
  act.sa_handler = exception_handler;
  act.sa_flags = 0;
  sigfillset(&act.sa_mask);
  sigaction(SIGBUS, &act, old_bus);
  sigaction(SIGSEGV, &act, old_segv);
}

static int _sig_is_ours(void)
{
  struct sigaction bus, segv;
  sigaction(SIGBUS, NULL, &bus);
  sigaction(SIGSEGV, NULL, &segv);
  return bus.sa_handler == exception_handler && segv.sa_handler == exception_handler;
}

static void _sig_enter(void)
{
  pthread_mutex_lock(&_sig_mu);
  if (_sig_users++ == 0)
    _sig_install(&_sig_old_bus, &_sig_old_segv);
  else if (!_sig_is_ours())
    /* a stock YR_TRYCATCH on another thread ended meanwhile and restored
     * what it had saved: install ours again for this copy (the saved actions
     * stay those found by the first copy in) */
    _sig_install(NULL, NULL);
  pthread_mutex_unlock(&_sig_mu);
}

static void _sig_leave(void)
{
  pthread_mutex_lock(&_sig_mu);
  /* the last copy out restores what the first one found -- unless the
   * handler is no longer ours: then the application (or another YR_TRYCATCH)
   * installed its own meanwhile, and that one stays */
  if (--_sig_users == 0 && _sig_is_ours())
  {
    sigaction(SIGBUS, &_sig_old_bus, NULL);
    sigaction(SIGSEGV, &_sig_old_segv, NULL);
  }
  pthread_mutex_unlock(&_sig_mu);
}

static int _guarded_copy(void* user, void* dst, const void* src, size_t n)
{
  YR_GPU_SCANNER* gs = (YR_GPU_SCANNER*) user;
  if (!gs->trycatch)
  {
    memcpy(dst, src, n);
    return 0;
  }
  volatile int result = 0;
  sigjmp_buf jb;
  _sig_enter();
  /* exception_handler jumps to the buffer this thread stored (TLS) */
  yr_thread_storage_set_value(&yr_trycatch_trampoline_tls, &jb);
  if (sigsetjmp(jb, 1) == 0)
    memcpy(dst, src, n);
  else
    result = 1;
  yr_thread_storage_set_value(&yr_trycatch_trampoline_tls, NULL);
  _sig_leave();
  return result;
}

int yr_gpu_scanner_create(YR_GPU_RULES* g, YR_GPU_SCANNER** out)
{
  *out = NULL;
  YR_GPU_SCANNER* s = (YR_GPU_SCANNER*) calloc(1, sizeof(YR_GPU_SCANNER));
  if (s == NULL) return ERROR_INSUFFICIENT_MEMORY;
  s->multi_min = YR_GPU_MULTI_MIN_BLOCK;
  s->trycatch = 1;
  int r = yr_amd_scanner_create(g->tables, NULL, &s->scanner);
  if (r == ERROR_SUCCESS)
  {
    /* several devices: one pipeline over all of them -- blocks of at least
     * multi_min split across the devices, smaller ones whole to one device
     * (round-robin), all in one ordered stream, so a large block never waits
     * for the blocks in flight to drain */
    s->depth = 2;
    r = g->n_devices > 1
            ? yr_amd_pipeline_create_multi(g->dev_tables, g->n_devices, s->depth, &s->pipe)
            : yr_amd_pipeline_create(g->tables, s->depth, &s->pipe);
    if (r == ERROR_SUCCESS) r = yr_amd_pipeline_set_copy(s->pipe, _guarded_copy, s);
    if (r == ERROR_SUCCESS && g->n_devices > 1)
      r = yr_amd_pipeline_set_split_min(s->pipe, s->multi_min);
    if (r != ERROR_SUCCESS)
    {
      yr_amd_pipeline_destroy(s->pipe);
      yr_amd_scanner_destroy(s->scanner);
    }
  }
  if (r == ERROR_SUCCESS && g->n_devices > 1)
  {
    r = yr_amd_multi_create(g->dev_tables, g->n_devices, &s->multi);
    if (r == ERROR_SUCCESS) r = yr_amd_multi_set_copy(s->multi, _guarded_copy, s);
    if (r != ERROR_SUCCESS)
    {
      yr_amd_multi_destroy(s->multi);
      yr_amd_pipeline_destroy(s->pipe);
      yr_amd_scanner_destroy(s->scanner);
    }
  }
  if (r != ERROR_SUCCESS)
  {
    free(s);
    return r;
  }
  s->gpu_rules = g;
  s->preverify = 1;
  *out = s;
  return ERROR_SUCCESS;
}

void yr_gpu_scanner_set_preverify(YR_GPU_SCANNER* s, int enable)
{
  s->preverify = enable != 0;
}

void yr_gpu_scanner_set_multi_min_block(YR_GPU_SCANNER* s, uint64_t bytes)
{
  s->multi_min = bytes;
  if (s->multi != NULL) yr_amd_pipeline_set_split_min(s->pipe, bytes);
}

uint64_t yr_gpu_scanner_multi_blocks(const YR_GPU_SCANNER* s)
{
  return s->multi_blocks;
}

static double _now(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

void yr_gpu_scanner_timing(const YR_GPU_SCANNER* s, double t[3])
{
  t[0] = s->t_copy;
  t[1] = s->t_gpu;
  t[2] = s->t_replay;
}

void yr_gpu_scanner_destroy(YR_GPU_SCANNER* s)
{
  if (s == NULL) return;
  yr_amd_multi_destroy(s->multi);
  yr_amd_pipeline_destroy(s->pipe);
  yr_amd_scanner_destroy(s->scanner);
  free(s->staging);
  free(s);
}

/* Timeout checks at the block positions the reference walk checks them
 * (scanner.c:74-81): at the top of the loop for every i < size with
 * i % 4096 == 0, i.e. before the verify calls dispatched at i.  The GPU path
 * reaches position `pos` of the block when it replays the first call
 * dispatched at a position >= pos; every check of the reference up to pos that
 * has not been made yet is made then (one clock read: the clock is monotonic,
 * so a later read fires whenever an earlier one would have).  *next is the
 * first position not yet checked. */
static int _timeout_upto(YR_SCANNER* scanner, uint64_t* next, uint64_t pos, size_t size)
{
  if (scanner->timeout <= 0 || size == 0) return ERROR_SUCCESS;
  if (pos > size - 1) pos = size - 1;
  if (*next > pos) return ERROR_SUCCESS;
  *next = (pos / 4096 + 1) * 4096;
  if (yr_stopwatch_elapsed_ns(&scanner->stopwatch) > scanner->timeout)
    return ERROR_SCAN_TIMEOUT;
  return ERROR_SUCCESS;
}

typedef struct
{
  YR_SCANNER* scanner;
  const uint8_t* data;
  size_t size;
  uint64_t base;
  uint64_t next_check; /* _timeout_upto */
} verify_ctx;

/* The reference's own call, scanner.c:111-117 / :153-159, after the timeout
 * checks the walk makes before reaching the call's position. */
static int _verify(void* user, uint32_t pool_index, uint64_t offset)
{
  verify_ctx* c = (verify_ctx*) user;
  YR_AC_MATCH* m = &c->scanner->rules->ac_match_pool[pool_index];
  FAIL_ON_ERROR(_timeout_upto(c->scanner, &c->next_check, offset + m->backtrack, c->size));
  return yr_scan_verify_match(c->scanner, m, c->data, c->size, c->base, (size_t) offset);
}

#ifdef YR_PROFILING_ENABLED
/* A count-only record (YR_AMD_REC_COUNT_ONLY: a call pre-verification dropped
 * that still passes yr_scan_verify_match's early returns): the reference's own
 * tests in its order (scan.c:1013-1027) on the host state at this point of
 * the call sequence, then its atom_matches count (scan.c:1083) -- nothing
 * else of the call can have an effect. */
static void _count_only(YR_SCANNER* scanner, YR_AC_MATCH* m, size_t size, uint64_t base,
                        uint64_t offset)
{
  YR_STRING* string = m->string;
  if (size - offset <= 0) return;
  if (yr_bitmask_is_set(scanner->strings_temp_disabled, string->idx)) return;
  if (scanner->flags & SCAN_FLAGS_FAST_MODE && STRING_IS_SINGLE_MATCH(string) &&
      scanner->matches[string->idx].head != NULL)
    return;
  if (STRING_IS_FIXED_OFFSET(string) && string->fixed_offset != base + offset) return;
  scanner->profiling_info[string->rule_idx].atom_matches++;
}
#endif

/* The effective verify calls of one block (pre-verification records), in the
 * reference's order, with the walk's timeout checks (_timeout_upto). */
static int _replay_records(
    YR_SCANNER* scanner,
    const yr_amd_verify_rec* recs,
    uint64_t n,
    const uint8_t* data,
    size_t size,
    uint64_t base,
    uint64_t next_check)
{
  verify_ctx ctx = {scanner, data, size, base, next_check};
  for (uint64_t c = 0; c < n; c++)
  {
    if (recs[c].pool_index & YR_AMD_REC_COUNT_ONLY)
    {
#ifdef YR_PROFILING_ENABLED
      YR_AC_MATCH* m = &scanner->rules->ac_match_pool[recs[c].pool_index & ~YR_AMD_REC_COUNT_ONLY];
      FAIL_ON_ERROR(_timeout_upto(scanner, &ctx.next_check, recs[c].offset + m->backtrack, size));
      _count_only(scanner, m, size, base, recs[c].offset);
#endif
      continue;
    }
    FAIL_ON_ERROR(_verify(&ctx, recs[c].pool_index, recs[c].offset));
  }
  /* the checks the walk makes after its last dispatch, up to size - 1 */
  return _timeout_upto(scanner, &ctx.next_check, size, size);
}

/* Replacement of _yr_scanner_scan_mem_block (scanner.c:45-176). */
static int _yr_gpu_scan_mem_block(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* block_data,
    YR_MEMORY_BLOCK* block)
{
  int result = ERROR_SUCCESS;
  uint64_t next_check = 0;

  /* the walk's first timeout check, position 0 (scanner.c:74-81) */
  FAIL_ON_ERROR(_timeout_upto(scanner, &next_check, 0, block->size));

  /* Block bytes may live in an mmap (filemap.c:56): copy them in the scanning
   * thread inside the trycatch so a SIGBUS/SIGSEGV maps to
   * ERROR_COULD_NOT_MAP_FILE exactly as at scanner.c:493-496. */
  if (block->size > gs->staging_size)
  {
    uint8_t* p = (uint8_t*) realloc(gs->staging, block->size);
    if (p == NULL) return ERROR_INSUFFICIENT_MEMORY;
    gs->staging = p;
    gs->staging_size = block->size;
  }
  YR_TRYCATCH(
      !(scanner->flags & SCAN_FLAGS_NO_TRYCATCH),
      { memcpy(gs->staging, block_data, block->size); },
      { result = ERROR_COULD_NOT_MAP_FILE; });
  if (result != ERROR_SUCCESS) return result;

  const uint64_t* positions = NULL;
  uint64_t count = 0;
  int all_positions = 0;
  FAIL_ON_ERROR(yr_amd_scan_block(
      gs->scanner,
      gs->staging,
      block->size,
      &positions,
      &count,
      &all_positions));

  verify_ctx ctx = {scanner, gs->staging, block->size, block->base, next_check};
  FAIL_ON_ERROR(yr_amd_replay(
      gs->gpu_rules->tables,
      gs->staging,
      block->size,
      positions,
      count,
      all_positions,
      _verify,
      &ctx));
  return _timeout_upto(scanner, &ctx.next_check, block->size, block->size);
}

/* Replay the oldest block of the pipeline: its effective verify calls, in the
 * reference's order (scanner.c:111-117 / :153-159), into the unmodified
 * yr_scan_verify_match. */
static int _replay_next(YR_SCANNER* scanner, YR_GPU_SCANNER* gs)
{
  const yr_amd_verify_rec* recs = NULL;
  uint64_t n = 0;
  const uint8_t* data = NULL;
  size_t size = 0;
  uint64_t base = 0;
  double t0 = _now();
  int result = yr_amd_pipeline_next(gs->pipe, &recs, &n, &data, &size, &base);
  double t1 = _now();
  gs->t_gpu += t1 - t0;
  gs->inflight--;
  if (result != ERROR_SUCCESS) return result;
  /* the walk of this block starts here: its position-0 timeout check */
  uint64_t next_check = 0;
  FAIL_ON_ERROR(_timeout_upto(scanner, &next_check, 0, size));
  result = _replay_records(scanner, recs, n, data, size, base, next_check);
  gs->t_replay += _now() - t1;
  return result;
}

/* One block into the pipeline; replays the oldest when `depth` are in flight. */
static int _pipeline_block(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* data,
    YR_MEMORY_BLOCK* block)
{
  int result = ERROR_SUCCESS;
  /* The block is copied into the pipeline's pinned buffer by several threads
   * at once (yr_amd_pipeline_submit_dma), each chunk through _guarded_copy:
   * a fault on any of them (a truncated mapping) fails the submission with
   * ERROR_COULD_NOT_MAP_FILE as scanner.c:493-496 does. */
  gs->trycatch = !(scanner->flags & SCAN_FLAGS_NO_TRYCATCH);
  double t0 = _now();
  result = yr_amd_pipeline_submit_dma(gs->pipe, data, block->size, block->base);
  gs->t_copy += _now() - t0;
  if (result != ERROR_SUCCESS) return result;
  gs->inflight++;
  if (gs->inflight == gs->depth) return _replay_next(scanner, gs);
  return ERROR_SUCCESS;
}

/* A block the caller keeps valid and in memory for the whole scan (the one
 * block of yr_gpu_scanner_scan_mem): no staging copy -- H2D straight from the
 * caller's buffer, pre-verification, replay of the effective calls.  Reads of
 * the block during the replay stay inside YR_TRYCATCH as in scanner.c:493-496. */
static int _direct_block(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* data,
    YR_MEMORY_BLOCK* block,
    int use_multi)
{
  int result = ERROR_SUCCESS;
  uint64_t next_check = 0;
  FAIL_ON_ERROR(_timeout_upto(scanner, &next_check, 0, block->size));
  const yr_amd_verify_rec* recs = NULL;
  uint64_t n = 0;
  gs->trycatch = !(scanner->flags & SCAN_FLAGS_NO_TRYCATCH);
  double t0 = _now();
  if (use_multi)
  {
    /* staged through pinned memory by _guarded_copy (helper threads
     * included): a fault fails the call with ERROR_COULD_NOT_MAP_FILE */
    result = yr_amd_multi_scan_block_verified(
        gs->multi, data, block->size, block->base, &recs, &n);
    if (result != ERROR_SUCCESS) return result;
  }
  else
  {
    /* The H2D below reads the caller's buffer inside the HIP runtime, where a
     * fault cannot be unwound.  Touch every page of it first, inside the
     * trycatch, so a buffer that faults (a truncated file mapping, an unmapped
     * range) yields ERROR_COULD_NOT_MAP_FILE as scanner.c:493-496 does; ~3 ms
     * per GiB of resident memory. */
    YR_TRYCATCH(
        gs->trycatch,
        {
          volatile uint8_t sink = 0;
          for (size_t o = 0; o < block->size; o += 4096) sink ^= data[o];
          if (block->size > 0) sink ^= data[block->size - 1];
          (void) sink;
        },
        { result = ERROR_COULD_NOT_MAP_FILE; });
    if (result != ERROR_SUCCESS) return result;
    FAIL_ON_ERROR(
        yr_amd_scan_block_verified(gs->scanner, data, block->size, block->base, &recs, &n));
  }
  double t1 = _now();
  gs->t_gpu += t1 - t0;
  YR_TRYCATCH(
      !(scanner->flags & SCAN_FLAGS_NO_TRYCATCH),
      { result = _replay_records(scanner, recs, n, data, block->size, block->base, next_check); },
      { result = ERROR_COULD_NOT_MAP_FILE; });
  gs->t_replay += _now() - t1;
  return result;
}

/* Can the multi-device path take a block of this size?  Every device's
 * candidate stream must fit pre-verification (yr_amd_multi_scan_block_verified
 * refuses it otherwise). */
static int _multi_fits(YR_GPU_SCANNER* gs, uint64_t size)
{
  for (uint32_t k = 0; k < gs->gpu_rules->n_devices; k++)
  {
    uint64_t b = 0, e = 0;
    if (yr_amd_multi_shard(gs->multi, size, k, &b, &e, NULL, NULL) != ERROR_SUCCESS) return 0;
    if ((e - b) + (b == 0 ? 1 : 0) > YR_AMD_VERIFY_MAX_CANDIDATES) return 0;
  }
  return 1;
}

/* One block: the replacement of the walk at scanner.c:493-496. */
static int _scan_one_block(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* data,
    YR_MEMORY_BLOCK* block)
{
  /* Pre-verification takes candidate streams of at most
   * YR_AMD_VERIFY_MAX_CANDIDATES (yr_amd_verify_device), and a block of size
   * bytes has at most size + 1 candidates (every position of a root-accepting
   * rule set, or a dense key): a block that could exceed it is replayed from
   * the GPU scan's stream instead -- after the blocks still in flight, in
   * order.  The same limit as the library's, so no block reaches a refusal. */
  int split = gs->multi != NULL && block->size >= gs->multi_min;
  int fits = split ? _multi_fits(gs, block->size)
                   : (uint64_t) block->size + 1 <= YR_AMD_VERIFY_MAX_CANDIDATES;
  int replay_block = !gs->preverify || !fits;
  while (replay_block && gs->inflight > 0) FAIL_ON_ERROR(_replay_next(scanner, gs));
  if (replay_block) return _yr_gpu_scan_mem_block(scanner, gs, data, block);
  if (split) gs->multi_blocks++;
  /* the one block of scan_mem, in place (a large one across the devices) */
  if (gs->direct) return _direct_block(scanner, gs, data, block, split);
  /* the pipeline (across the devices when split), in order behind the
   * blocks in flight */
  return _pipeline_block(scanner, gs, data, block);
}

/* The blocks still on the GPU, in order (after the iterator's last block). */
static int _finish_blocks(YR_SCANNER* scanner, YR_GPU_SCANNER* gs)
{
  while (gs->inflight > 0) FAIL_ON_ERROR(_replay_next(scanner, gs));
  return ERROR_SUCCESS;
}

static void _abort_blocks(YR_GPU_SCANNER* gs)
{
  if (gs->inflight > 0)
  {
    yr_amd_pipeline_drain(gs->pipe);
    gs->inflight = 0;
  }
}

#ifdef YR_HAVE_BLOCK_SCANNER
/* With libyara patched by integration/libyara-block-scanner.patch, the
 * unmodified driver (yr_scanner_scan_mem_blocks and every entry point above
 * it) calls these in place of its CPU walk. */
static int _bs_scan_block(
    void* ctx,
    YR_SCANNER* scanner,
    const uint8_t* data,
    YR_MEMORY_BLOCK* block)
{
  return _scan_one_block(scanner, (YR_GPU_SCANNER*) ctx, data, block);
}

static int _bs_finish(void* ctx, YR_SCANNER* scanner)
{
  return _finish_blocks(scanner, (YR_GPU_SCANNER*) ctx);
}

static void _bs_abort(void* ctx, YR_SCANNER* scanner)
{
  (void) scanner;
  _abort_blocks((YR_GPU_SCANNER*) ctx);
}

int yr_gpu_scanner_attach(YR_SCANNER* scanner, YR_GPU_SCANNER* gs)
{
  if (gs->gpu_rules->rules != scanner->rules) return ERROR_INVALID_ARGUMENT;
  gs->block_scanner.scan_block = _bs_scan_block;
  gs->block_scanner.finish = _bs_finish;
  gs->block_scanner.abort = _bs_abort;
  gs->block_scanner.ctx = gs;
  yr_scanner_set_block_scanner(scanner, &gs->block_scanner);
  return ERROR_SUCCESS;
}
#endif

/* _yr_scanner_clean_matches (scanner.c:178-203) is static: same memsets. */
static void _clean_matches(YR_SCANNER* scanner)
{
  memset(
      scanner->rule_matches_flags,
      0,
      sizeof(YR_BITMASK) * YR_BITMASK_SIZE(scanner->rules->num_rules));
  memset(
      scanner->ns_unsatisfied_flags,
      0,
      sizeof(YR_BITMASK) * YR_BITMASK_SIZE(scanner->rules->num_namespaces));
  memset(
      scanner->strings_temp_disabled,
      0,
      sizeof(YR_BITMASK) * YR_BITMASK_SIZE(scanner->rules->num_strings));
  memset(scanner->matches, 0, sizeof(YR_MATCHES) * scanner->rules->num_strings);
  memset(
      scanner->unconfirmed_matches,
      0,
      sizeof(YR_MATCHES) * scanner->rules->num_strings);
}

/* Diagnostics (not part of the drop-in API; tools/replay_profile.py): the
 * replay of one block's records on a scanner set up as for a scan, timed.
 * mode 0: the shim's replay (_replay_records: the walk's timeout checks, then
 * yr_scan_verify_match per record); 1: the shim's per-record work without the
 * libyara call; 2: yr_scan_verify_match alone, one call per record.  With
 * timeout_ns > 0 the scanner has that timeout (the checks then read the
 * clock).  The scan state is cleared afterwards, as a scan's end does. */
int yr_gpu_replay_profile(
    YR_SCANNER* scanner,
    const yr_amd_verify_rec* recs,
    uint64_t n,
    const uint8_t* data,
    size_t size,
    int mode,
    uint64_t timeout_ns,
    double* seconds)
{
  uint32_t max_match_data;
  int result = ERROR_SUCCESS;
  FAIL_ON_ERROR(yr_get_configuration_uint32(YR_CONFIG_MAX_MATCH_DATA, &max_match_data));
  FAIL_ON_ERROR(yr_notebook_create(
      1024 * (sizeof(YR_MATCH) + max_match_data), &scanner->matches_notebook));
  scanner->timeout = timeout_ns;
  yr_stopwatch_start(&scanner->stopwatch);
  double t0 = _now();
  if (mode == 0)
  {
    result = _replay_records(scanner, recs, n, data, size, 0, 0);
  }
  else if (mode == 1)
  {
    verify_ctx c = {scanner, data, size, 0, 0};
    volatile uintptr_t sink = 0;
    for (uint64_t k = 0; k < n && result == ERROR_SUCCESS; k++)
    {
      YR_AC_MATCH* m = &scanner->rules->ac_match_pool[recs[k].pool_index];
      result = _timeout_upto(scanner, &c.next_check, recs[k].offset + m->backtrack, size);
      sink ^= (uintptr_t) m ^ recs[k].offset;
    }
  }
  else
  {
    for (uint64_t k = 0; k < n && result == ERROR_SUCCESS; k++)
      result = yr_scan_verify_match(
          scanner, &scanner->rules->ac_match_pool[recs[k].pool_index], data, size, 0,
          (size_t) recs[k].offset);
  }
  *seconds = _now() - t0;
  scanner->timeout = 0;
  _clean_matches(scanner);
  yr_notebook_destroy(scanner->matches_notebook);
  scanner->matches_notebook = NULL;
  return result;
}

/* yr_scanner_scan_mem_blocks (scanner.c:417-583) with the GPU block scan. */
int yr_gpu_scanner_scan_mem_blocks(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    YR_MEMORY_BLOCK_ITERATOR* iterator)
{
  YR_RULES* rules;
  YR_RULE* rule;
  YR_MEMORY_BLOCK* block;
  int i, result = ERROR_SUCCESS;

  if (scanner->callback == NULL) return ERROR_CALLBACK_REQUIRED;

  scanner->iterator = iterator;
  rules = scanner->rules;

  if (iterator->last_error == ERROR_BLOCK_NOT_READY)
  {
    block = iterator->next(iterator);
  }
  else
  {
    uint32_t max_match_data;
    FAIL_ON_ERROR(
        yr_get_configuration_uint32(YR_CONFIG_MAX_MATCH_DATA, &max_match_data));
    result = yr_notebook_create(
        1024 * (sizeof(YR_MATCH) + max_match_data), &scanner->matches_notebook);
    if (result != ERROR_SUCCESS) goto _exit;
    yr_stopwatch_start(&scanner->stopwatch);
    block = iterator->first(iterator);
  }

  while (block != NULL)
  {
    const uint8_t* data = block->fetch_data(block);
    if (data == NULL)
    {
      block = iterator->next(iterator);
      continue;
    }
    if (scanner->entry_point == YR_UNDEFINED)
    {
      YR_TRYCATCH(
          !(scanner->flags & SCAN_FLAGS_NO_TRYCATCH),
          {
            if (scanner->flags & SCAN_FLAGS_PROCESS_MEMORY)
              scanner->entry_point = yr_get_entry_point_address(
                  data, block->size, block->base);
            else
              scanner->entry_point = yr_get_entry_point_offset(
                  data, block->size);
          },
          {});
    }

    result = _scan_one_block(scanner, gs, data, block);
    if (result != ERROR_SUCCESS) goto _exit;
    block = iterator->next(iterator);
  }

  result = _finish_blocks(scanner, gs);
  if (result != ERROR_SUCCESS) goto _exit;

  result = iterator->last_error;
  if (result != ERROR_SUCCESS) goto _exit;

  if (iterator->file_size != NULL)
    scanner->file_size = iterator->file_size(iterator);
  else
    scanner->file_size = YR_UNDEFINED;

  YR_TRYCATCH(
      !(scanner->flags & SCAN_FLAGS_NO_TRYCATCH),
      { result = yr_execute_code(scanner); },
      { result = ERROR_COULD_NOT_MAP_FILE; });
  if (result != ERROR_SUCCESS) goto _exit;

  for (i = 0, rule = rules->rules_table; !RULE_IS_NULL(rule); i++, rule++)
  {
    int message = 0;
    if (yr_bitmask_is_set(scanner->rule_matches_flags, i) &&
        yr_bitmask_is_not_set(scanner->ns_unsatisfied_flags, rule->ns->idx))
    {
      if (scanner->flags & SCAN_FLAGS_REPORT_RULES_MATCHING)
        message = CALLBACK_MSG_RULE_MATCHING;
    }
    else
    {
      if (scanner->flags & SCAN_FLAGS_REPORT_RULES_NOT_MATCHING)
        message = CALLBACK_MSG_RULE_NOT_MATCHING;
    }
    if (message != 0 && !RULE_IS_PRIVATE(rule))
    {
      switch (scanner->callback(scanner, message, rule, scanner->user_data))
      {
      case CALLBACK_ABORT:
        result = ERROR_SUCCESS;
        goto _exit;
      case CALLBACK_ERROR:
        result = ERROR_CALLBACK_ERROR;
        goto _exit;
      }
    }
  }
  scanner->callback(scanner, CALLBACK_MSG_SCAN_FINISHED, NULL, scanner->user_data);

_exit:
  _abort_blocks(gs);
  if (result != ERROR_BLOCK_NOT_READY)
  {
    _clean_matches(scanner);
    if (scanner->matches_notebook != NULL)
    {
      yr_notebook_destroy(scanner->matches_notebook);
      scanner->matches_notebook = NULL;
    }
  }
  return result;
}

static YR_MEMORY_BLOCK* _first_block(YR_MEMORY_BLOCK_ITERATOR* it)
{
  return (YR_MEMORY_BLOCK*) it->context;
}

static YR_MEMORY_BLOCK* _next_block(YR_MEMORY_BLOCK_ITERATOR* it)
{
  return NULL;
}

static uint64_t _file_size(YR_MEMORY_BLOCK_ITERATOR* it)
{
  return ((YR_MEMORY_BLOCK*) it->context)->size;
}

static const uint8_t* _fetch(YR_MEMORY_BLOCK* b)
{
  return (const uint8_t*) b->context;
}

static int _scan_mem(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* buffer,
    size_t buffer_size,
    int direct)
{
  YR_MEMORY_BLOCK block;
  YR_MEMORY_BLOCK_ITERATOR iterator;
  block.size = buffer_size;
  block.base = 0;
  block.fetch_data = _fetch;
  block.context = (void*) buffer;
  iterator.context = &block;
  iterator.first = _first_block;
  iterator.next = _next_block;
  iterator.file_size = _file_size;
  iterator.last_error = ERROR_SUCCESS;
  gs->direct = direct;
  int result = yr_gpu_scanner_scan_mem_blocks(scanner, gs, &iterator);
  gs->direct = 0;
  return result;
}

/* yr_scanner_scan_mem (scanner.c:633-671) with the GPU driver: the caller's
 * buffer is ordinary memory, valid for the whole call, so it is scanned in
 * place (no staging copy). */
int yr_gpu_scanner_scan_mem(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* buffer,
    size_t buffer_size)
{
  return _scan_mem(scanner, gs, buffer, buffer_size, 1);
}

/* yr_scanner_scan_file (scanner.c:674-688): map, scan, unmap. */
int yr_gpu_scanner_scan_file(YR_SCANNER* scanner, YR_GPU_SCANNER* gs, const char* filename)
{
  YR_MAPPED_FILE mfile;
  int result = yr_filemap_map(filename, &mfile);
  if (result == ERROR_SUCCESS)
  {
    result = _scan_mem(scanner, gs, mfile.data, mfile.size, 0);   /* mmap: copy under TRYCATCH */
    yr_filemap_unmap(&mfile);
  }
  return result;
}

/* yr_scanner_scan_fd (scanner.c:690-704). */
int yr_gpu_scanner_scan_fd(YR_SCANNER* scanner, YR_GPU_SCANNER* gs, YR_FILE_DESCRIPTOR fd)
{
  YR_MAPPED_FILE mfile;
  int result = yr_filemap_map_fd(fd, 0, 0, &mfile);
  if (result == ERROR_SUCCESS)
  {
    result = _scan_mem(scanner, gs, mfile.data, mfile.size, 0);
    yr_filemap_unmap_fd(&mfile);
  }
  return result;
}

/* yr_scanner_scan_proc (scanner.c:706-722): the process's memory regions are
 * the blocks (proc/linux.c iterator), SCAN_FLAGS_PROCESS_MEMORY set. */
int yr_gpu_scanner_scan_proc(YR_SCANNER* scanner, YR_GPU_SCANNER* gs, int pid)
{
  YR_MEMORY_BLOCK_ITERATOR iterator;
  int result = yr_process_open_iterator(pid, &iterator);
  if (result == ERROR_SUCCESS)
  {
    int prev_flags = scanner->flags;
    scanner->flags |= SCAN_FLAGS_PROCESS_MEMORY;
    result = yr_gpu_scanner_scan_mem_blocks(scanner, gs, &iterator);
    scanner->flags = prev_flags;
    yr_process_close_iterator(&iterator);
  }
  return result;
}
