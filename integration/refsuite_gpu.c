/*
 * refsuite_gpu.c -- runs libyara's OWN known-answer suites through the GPU
 * scan path (test infrastructure; oracle/refsuite.mk builds it).
 *
 * The reference's tests/test-rules.c, tests/test-async.c, tests/test-api.c and
 * tests/util.c are compiled in place from the reference tree with every scan
 * entry point renamed at compile time (-Dyr_rules_scan_mem=ygt_rules_scan_mem,
 * ...; the full list is REDIRECT in oracle/refsuite.mk).  This file defines
 * those names: each is the reference function's own flow (rules.c:172-324,
 * scanner.c:417-719) with the block scan done by the libyara-side integration
 * (integration/yr_gpu_scanner.c: GPU candidate stream + on-device
 * pre-verification + replay into the unmodified yr_scan_verify_match), so every
 * assertion of those suites checks the GPU path's match sets, match counts,
 * offsets, error codes and ERROR_BLOCK_NOT_READY resumption.
 *
 *   YR_GPU_PREVERIFY=0   replay the full candidate stream (no pre-verification)
 *
 * A YR_GPU_RULES is built per YR_RULES on first use and freed by the
 * redirected yr_rules_destroy; a YR_GPU_SCANNER per YR_SCANNER, freed by the
 * redirected yr_scanner_destroy.  At exit the number of GPU block scans is
 * printed ("refsuite-gpu: ..."), so the test can tell the suite really went
 * through the GPU (and a GPU setup failure aborts loudly: there is no CPU
 * fallback).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <yara.h>
#include <yara/filemap.h>
#include <yara/proc.h>

#include "yr_gpu_scanner.h"

#define MAX_LIVE 256

static struct
{
  YR_RULES* rules;
  YR_GPU_RULES* g;
} live_rules[MAX_LIVE];

static struct
{
  YR_SCANNER* scanner;
  YR_GPU_SCANNER* gs;
} live_scanners[MAX_LIVE];

static unsigned long n_scans, n_rules_built;
static int preverify = 1;
static int initialised;

static void _report(void)
{
  fprintf(
      stderr,
      "refsuite-gpu: %lu scans through yr_gpu_scanner, %lu GPU rule sets, "
      "preverify=%d\n",
      n_scans,
      n_rules_built,
      preverify);
}

static void _init(void)
{
  if (initialised) return;
  initialised = 1;
  const char* e = getenv("YR_GPU_PREVERIFY");
  if (e != NULL && e[0] == '0') preverify = 0;
  atexit(_report);
}

static void _fatal(const char* what, int rc)
{
  fprintf(stderr, "refsuite-gpu: %s failed: %d (no CPU fallback)\n", what, rc);
  exit(3);
}

static YR_GPU_RULES* _gpu_rules(YR_RULES* rules)
{
  int free_slot = -1;
  for (int i = 0; i < MAX_LIVE; i++)
  {
    if (live_rules[i].rules == rules) return live_rules[i].g;
    if (live_rules[i].rules == NULL && free_slot < 0) free_slot = i;
  }
  if (free_slot < 0) _fatal("rules cache (too many live YR_RULES)", -1);
  YR_GPU_RULES* g = NULL;
  int rc = yr_gpu_rules_create(rules, 0, &g);
  if (rc != ERROR_SUCCESS) _fatal("yr_gpu_rules_create", rc);
  live_rules[free_slot].rules = rules;
  live_rules[free_slot].g = g;
  n_rules_built++;
  return g;
}

static YR_GPU_SCANNER* _gpu_scanner(YR_SCANNER* scanner)
{
  _init();
  int free_slot = -1;
  for (int i = 0; i < MAX_LIVE; i++)
  {
    if (live_scanners[i].scanner == scanner) return live_scanners[i].gs;
    if (live_scanners[i].scanner == NULL && free_slot < 0) free_slot = i;
  }
  if (free_slot < 0) _fatal("scanner cache (too many live YR_SCANNERs)", -1);
  YR_GPU_SCANNER* gs = NULL;
  int rc = yr_gpu_scanner_create(_gpu_rules(scanner->rules), &gs);
  if (rc != ERROR_SUCCESS) _fatal("yr_gpu_scanner_create", rc);
  yr_gpu_scanner_set_preverify(gs, preverify);
  live_scanners[free_slot].scanner = scanner;
  live_scanners[free_slot].gs = gs;
  return gs;
}

/* ---- YR_SCANNER entry points (scanner.c:287, :417-719) ---- */

void ygt_scanner_destroy(YR_SCANNER* scanner)
{
  for (int i = 0; i < MAX_LIVE; i++)
    if (live_scanners[i].scanner == scanner)
    {
      yr_gpu_scanner_destroy(live_scanners[i].gs);
      live_scanners[i].scanner = NULL;
      live_scanners[i].gs = NULL;
    }
  yr_scanner_destroy(scanner);
}

int ygt_scanner_scan_mem_blocks(YR_SCANNER* scanner, YR_MEMORY_BLOCK_ITERATOR* iterator)
{
  n_scans++;
  return yr_gpu_scanner_scan_mem_blocks(scanner, _gpu_scanner(scanner), iterator);
}

int ygt_scanner_scan_mem(YR_SCANNER* scanner, const uint8_t* buffer, size_t buffer_size)
{
  n_scans++;
  return yr_gpu_scanner_scan_mem(scanner, _gpu_scanner(scanner), buffer, buffer_size);
}

int ygt_scanner_scan_file(YR_SCANNER* scanner, const char* filename)
{
  n_scans++;
  return yr_gpu_scanner_scan_file(scanner, _gpu_scanner(scanner), filename);
}

int ygt_scanner_scan_fd(YR_SCANNER* scanner, YR_FILE_DESCRIPTOR fd)
{
  n_scans++;
  return yr_gpu_scanner_scan_fd(scanner, _gpu_scanner(scanner), fd);
}

int ygt_scanner_scan_proc(YR_SCANNER* scanner, int pid)
{
  n_scans++;
  return yr_gpu_scanner_scan_proc(scanner, _gpu_scanner(scanner), pid);
}

/* ---- YR_RULES entry points (rules.c:172-324, :515) ---- */

int ygt_rules_destroy(YR_RULES* rules)
{
  for (int i = 0; i < MAX_LIVE; i++)
    if (live_scanners[i].scanner != NULL && live_scanners[i].scanner->rules == rules)
      _fatal("yr_rules_destroy with a live scanner", -1);
  for (int i = 0; i < MAX_LIVE; i++)
    if (live_rules[i].rules == rules)
    {
      yr_gpu_rules_destroy(live_rules[i].g);
      live_rules[i].rules = NULL;
      live_rules[i].g = NULL;
    }
  return yr_rules_destroy(rules);
}

/* One scanner per call, exactly as rules.c:180-193 / :214-225 do. */
typedef int (*scan_fn)(YR_SCANNER*, void*);

static int _with_scanner(
    YR_RULES* rules,
    int flags,
    YR_CALLBACK_FUNC callback,
    void* user_data,
    int timeout,
    scan_fn fn,
    void* arg)
{
  YR_SCANNER* scanner;
  FAIL_ON_ERROR(yr_scanner_create(rules, &scanner));
  yr_scanner_set_callback(scanner, callback, user_data);
  yr_scanner_set_timeout(scanner, timeout);
  yr_scanner_set_flags(scanner, flags);
  int result = fn(scanner, arg);
  ygt_scanner_destroy(scanner);
  return result;
}

typedef struct
{
  const uint8_t* buffer;
  size_t size;
} mem_arg;

static int _scan_mem_fn(YR_SCANNER* s, void* a)
{
  mem_arg* m = (mem_arg*) a;
  return ygt_scanner_scan_mem(s, m->buffer, m->size);
}

static int _scan_blocks_fn(YR_SCANNER* s, void* a)
{
  return ygt_scanner_scan_mem_blocks(s, (YR_MEMORY_BLOCK_ITERATOR*) a);
}

static int _scan_file_fn(YR_SCANNER* s, void* a)
{
  return ygt_scanner_scan_file(s, (const char*) a);
}

static int _scan_fd_fn(YR_SCANNER* s, void* a)
{
  return ygt_scanner_scan_fd(s, *(YR_FILE_DESCRIPTOR*) a);
}

static int _scan_proc_fn(YR_SCANNER* s, void* a)
{
  return ygt_scanner_scan_proc(s, *(int*) a);
}

int ygt_rules_scan_mem_blocks(
    YR_RULES* rules,
    YR_MEMORY_BLOCK_ITERATOR* iterator,
    int flags,
    YR_CALLBACK_FUNC callback,
    void* user_data,
    int timeout)
{
  return _with_scanner(rules, flags, callback, user_data, timeout, _scan_blocks_fn, iterator);
}

int ygt_rules_scan_mem(
    YR_RULES* rules,
    const uint8_t* buffer,
    size_t buffer_size,
    int flags,
    YR_CALLBACK_FUNC callback,
    void* user_data,
    int timeout)
{
  mem_arg m = {buffer, buffer_size};
  return _with_scanner(rules, flags, callback, user_data, timeout, _scan_mem_fn, &m);
}

int ygt_rules_scan_file(
    YR_RULES* rules,
    const char* filename,
    int flags,
    YR_CALLBACK_FUNC callback,
    void* user_data,
    int timeout)
{
  return _with_scanner(
      rules, flags, callback, user_data, timeout, _scan_file_fn, (void*) filename);
}

int ygt_rules_scan_fd(
    YR_RULES* rules,
    YR_FILE_DESCRIPTOR fd,
    int flags,
    YR_CALLBACK_FUNC callback,
    void* user_data,
    int timeout)
{
  return _with_scanner(rules, flags, callback, user_data, timeout, _scan_fd_fn, &fd);
}

int ygt_rules_scan_proc(
    YR_RULES* rules,
    int pid,
    int flags,
    YR_CALLBACK_FUNC callback,
    void* user_data,
    int timeout)
{
  /* rules.c:287-313: the process iterator, SCAN_FLAGS_PROCESS_MEMORY */
  return _with_scanner(
      rules, flags | SCAN_FLAGS_PROCESS_MEMORY, callback, user_data, timeout, _scan_proc_fn, &pid);
}
