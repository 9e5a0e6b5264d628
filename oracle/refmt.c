// Multi-threaded STOCK libyara scan rate (test / measurement infrastructure,
// never product code): bench.py's cpu_baseline "stock, nproc threads" leg.
//
// One YR_SCANNER per thread, each scanning its own contiguous slice of one
// buffer with yr_scanner_scan_mem -- the way the reference CLI runs one scanner
// per scanning thread (cli/yara.c:1564-1608: yr_scanner_create +
// yr_scanner_set_callback per thread), except that the unit of work is a slice
// of one block instead of a file, and the thread count is not capped at the
// CLI's YR_MAX_THREADS (limits.h:50): the library itself does not limit it.
// A slice restarts the walk 4 bytes early (YR_MAX_ATOM_LENGTH, limits.h:68),
// as SURVEY.md §8d prescribes for the "nproc threads, one walker per slice"
// CPU comparator.  Every pass re-scans every slice; passes repeat until
// `min_seconds` of wall time have elapsed.
//
// Built against oracle/_ref/libyara_ref.so by oracle/ref.mk; called from
// bench.py through ctypes (the GIL is released for the call).
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <yara.h>

typedef struct {
  YR_SCANNER* scanner;
  const uint8_t* data;
  size_t lo, hi;   // bytes [lo, hi) of the buffer
  int rc;
  volatile int* go;
  volatile int* stop;
  volatile uint64_t passes;
} Worker;

static int refmt_callback(YR_SCAN_CONTEXT* ctx, int msg, void* msg_data, void* user) {
  (void)ctx;
  (void)msg;
  (void)msg_data;
  (void)user;
  return CALLBACK_CONTINUE;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void* worker_main(void* arg) {
  Worker* w = (Worker*)arg;
  while (!*w->go) sched_yield();
  while (!*w->stop) {
    const int rc = yr_scanner_scan_mem(w->scanner, w->data + w->lo, w->hi - w->lo);
    if (rc != ERROR_SUCCESS) {
      w->rc = rc;
      break;
    }
    ++w->passes;
  }
  return NULL;
}

// Returns 0 and fills *gbps (owned bytes scanned per second, decimal GB/s,
// over the passes every thread completed) and *passes (minimum completed
// passes over the threads), or a libyara error code / -1.
static int scan_initialized(const char* rules_src, const uint8_t* data, size_t n, int threads,
                            double min_seconds, double* gbps, uint64_t* passes, double* seconds) {
  int rc;
  YR_COMPILER* comp = NULL;
  YR_RULES* rules = NULL;
  rc = yr_compiler_create(&comp);
  if (rc != ERROR_SUCCESS) return rc;
  if (yr_compiler_add_string(comp, rules_src, NULL) != 0) {
    yr_compiler_destroy(comp);
    return -1;
  }
  rc = yr_compiler_get_rules(comp, &rules);
  yr_compiler_destroy(comp);
  if (rc != ERROR_SUCCESS) return rc;

  Worker* w = (Worker*)calloc((size_t)threads, sizeof(Worker));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  volatile int go = 0, stop = 0;
  int made = 0;
  for (int k = 0; k < threads && rc == ERROR_SUCCESS; ++k) {
    const size_t b = n / threads * k, e = k == threads - 1 ? n : n / threads * (k + 1);
    w[k].data = data;
    w[k].lo = b >= 4 ? b - 4 : 0;   // 4-byte warm-up (limits.h:68)
    w[k].hi = e;
    w[k].go = &go;
    w[k].stop = &stop;
    rc = yr_scanner_create(rules, &w[k].scanner);
    if (rc != ERROR_SUCCESS) break;
    yr_scanner_set_callback(w[k].scanner, refmt_callback, NULL);
    if (pthread_create(&th[k], NULL, worker_main, &w[k]) != 0) {
      yr_scanner_destroy(w[k].scanner);
      rc = -1;
      break;
    }
    ++made;
  }
  if (made < threads) stop = 1;   // the created threads leave without scanning
  const double t0 = now_s();
  go = 1;
  if (made == threads) {
    // until min_seconds have passed and every thread has finished a pass
    for (;;) {
      struct timespec d = {0, 20 * 1000 * 1000};
      nanosleep(&d, NULL);
      int all = 1;
      for (int k = 0; k < threads; ++k) all &= w[k].passes >= 1 || w[k].rc != 0;
      if (all && now_s() - t0 >= min_seconds) break;
    }
    stop = 1;
  }
  for (int k = 0; k < made; ++k) pthread_join(th[k], NULL);
  const double dt = now_s() - t0;
  uint64_t min_p = UINT64_MAX;
  double bytes = 0;
  for (int k = 0; k < made; ++k) {
    if (w[k].rc != 0 && rc == ERROR_SUCCESS) rc = w[k].rc;
    const size_t own = w[k].hi - (k == 0 ? 0 : w[k].lo + 4);
    bytes += (double)own * (double)w[k].passes;
    if (w[k].passes < min_p) min_p = w[k].passes;
    yr_scanner_destroy(w[k].scanner);
  }
  free(w);
  free(th);
  yr_rules_destroy(rules);
  if (rc == ERROR_SUCCESS) {
    *gbps = bytes / dt / 1e9;
    *passes = min_p;
    *seconds = dt;
  }
  return rc;
}

// yr_initialize / yr_finalize are paired on every call (libyara counts them,
// libyara.c), so repeated bench legs leave no global state behind.
int refmt_scan(const char* rules_src, const uint8_t* data, size_t n, int threads, double min_seconds,
               double* gbps, uint64_t* passes, double* seconds) {
  if (threads < 1 || n == 0) return -1;
  int rc = yr_initialize();
  if (rc != ERROR_SUCCESS) return rc;
  rc = scan_initialized(rules_src, data, n, threads, min_seconds, gbps, passes, seconds);
  yr_finalize();
  return rc;
}
