/*
 * ac_oracle.c -- CPU restatement of libyara's Aho-Corasick block scan.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the HIP path: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (yara_amd/, libyara_amd.so) never links or calls it.
 *
 * Pinned against the reference itself: tests/test_oracle_golden.py checks every
 * stream produced here against the verify-call streams recorded from the stock
 * libyara build (oracle/refdump + oracle/refhook.c, fixtures in tests/golden/).
 *
 * Reference followed (HoundThe/yara, libyara 4.2.1):
 *   - walk + per-position match-list dispatch: libyara/scanner.c:45-176
 *       dispatch before each byte (:98-122), transition with failure loop
 *       (:124-141), final dispatch at i == size (:144-163), backtrack filter
 *       `match->backtrack <= i` (:109, :151)
 *   - transition encoding: libyara/include/yara/ahocorasick.h:37-50
 *       slot = (target_slot << 9) | code, code = byte + 1, T[S] = failure link
 *   - match list: 1-based index into ac_match_pool, 0 = none
 *       (libyara/ahocorasick.c:611-618, types.h:596-607)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define AC_SLOT_OFFSET_BITS 9
#define AC_NEXT_STATE(t) ((t) >> AC_SLOT_OFFSET_BITS)
#define AC_INVALID(t, c) (((t) &0x1FFu) != (c))

/* One transition of the reference walk (scanner.c:124-141). */
static inline uint32_t ac_step(const uint32_t* T, uint32_t state, uint8_t byte)
{
  uint32_t index = (uint32_t) byte + 1;
  uint32_t t = T[state + index];
  while (AC_INVALID(t, index))
  {
    if (state != 0)
    {
      state = AC_NEXT_STATE(T[state]);
      t = T[state + index];
    }
    else
    {
      t = 0;
      break;
    }
  }
  return AC_NEXT_STATE(t);
}

uint32_t oracle_step(const uint32_t* T, uint32_t state, uint8_t byte)
{
  return ac_step(T, state, byte);
}

/*
 * Full reference walk over one block.  Every call the reference would make to
 * yr_scan_verify_match(scanner, &pool[k], data, n, base, i - backtrack) is
 * recorded as (i, k).  Returns the number of calls; writes at most `cap`.
 */
int64_t oracle_walk_verify(
    const uint32_t* T,
    const uint32_t* M,
    const uint32_t* pool_next,
    const uint16_t* pool_backtrack,
    const uint8_t* data,
    uint64_t n,
    uint64_t* out_pos,
    uint32_t* out_idx,
    int64_t cap)
{
  int64_t count = 0;
  uint32_t state = 0;
  uint64_t i = 0;
  for (;;)
  {
    uint32_t head = M[state];
    if (head != 0)
    {
      for (uint32_t k = head; k != 0; k = pool_next[k - 1])
      {
        if (pool_backtrack[k - 1] <= i)
        {
          if (count < cap)
          {
            out_pos[count] = i;
            out_idx[count] = k - 1;
          }
          count++;
        }
      }
    }
    if (i >= n) break;
    state = ac_step(T, state, data[i++]);
  }
  return count;
}

/* Positions i in [0, n] where M[state_i] != 0 (the candidate stream). */
int64_t oracle_candidates(
    const uint32_t* T,
    const uint32_t* M,
    const uint8_t* data,
    uint64_t n,
    uint64_t* out,
    int64_t cap)
{
  int64_t count = 0;
  uint32_t state = 0;
  uint64_t i = 0;
  for (;;)
  {
    if (M[state] != 0)
    {
      if (count < cap) out[count] = i;
      count++;
    }
    if (i >= n) break;
    state = ac_step(T, state, data[i++]);
  }
  return count;
}

/*
 * Candidate count over positions (lo, hi] of a block of n bytes, starting the
 * walk at root on byte max(0, lo - warm).  With warm >= the trie depth (4 for
 * libyara, limits.h:68) the state stream equals the full walk's.  Used by the
 * multi-threaded CPU baseline (one walker per contiguous slice).
 */
int64_t oracle_count_slice(
    const uint32_t* T,
    const uint32_t* M,
    const uint8_t* data,
    uint64_t lo,
    uint64_t hi,
    uint32_t warm)
{
  uint64_t i = lo > warm ? lo - warm : 0;
  uint32_t state = 0;
  int64_t count = 0;
  if (lo == 0 && M[0] != 0) count++;
  while (i < hi)
  {
    state = ac_step(T, state, data[i++]);
    if (i > lo && M[state] != 0) count++;
  }
  return count;
}

typedef struct
{
  const uint32_t* T;
  const uint32_t* M;
  const uint8_t* data;
  uint64_t lo, hi;
  int64_t count;
} slice_job;

static void* slice_worker(void* arg)
{
  slice_job* j = (slice_job*) arg;
  j->count = oracle_count_slice(j->T, j->M, j->data, j->lo, j->hi, 4);
  return NULL;
}

/* nthreads contiguous slices + 4-byte warm-up (SURVEY.md §8d CPU mode 2). */
int64_t oracle_count_parallel(
    const uint32_t* T,
    const uint32_t* M,
    const uint8_t* data,
    uint64_t n,
    int nthreads)
{
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = calloc(nthreads, sizeof(pthread_t));
  slice_job* jobs = calloc(nthreads, sizeof(slice_job));
  for (int t = 0; t < nthreads; t++)
  {
    jobs[t].T = T;
    jobs[t].M = M;
    jobs[t].data = data;
    jobs[t].lo = n * t / nthreads;
    jobs[t].hi = n * (t + 1) / nthreads;
    pthread_create(&th[t], NULL, slice_worker, &jobs[t]);
  }
  int64_t total = 0;
  for (int t = 0; t < nthreads; t++)
  {
    pthread_join(th[t], NULL);
    total += jobs[t].count;
  }
  free(th);
  free(jobs);
  return total;
}

/* SURVEY.md Appendix A canonical buffer generator (xorshift64, byte = x>>24). */
void oracle_xorshift_fill(uint8_t* buf, uint64_t n, uint64_t seed)
{
  uint64_t x = 0x9E3779B97F4A7C15ull * seed;
  for (uint64_t i = 0; i < n; i++)
  {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    buf[i] = (uint8_t) (x >> 24);
  }
}
