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
 * The walk's debug trace (scanner.c:83-96 at YR_DEBUG_VERBOSITY 2, plus the
 * final state at i == n, scanner.c:145): every position i in [0, n] whose
 * state is not the root, with the state and M[state].  The sequential walk
 * from the block start, as the reference runs it.
 */
int64_t oracle_trace(
    const uint32_t* T,
    const uint32_t* M,
    const uint8_t* data,
    uint64_t n,
    uint64_t* pos,
    uint32_t* states,
    uint32_t* matches,
    int64_t cap)
{
  int64_t count = 0;
  uint32_t state = 0;
  uint64_t i = 0;
  for (;;)
  {
    if (state != 0)
    {
      if (count < cap)
      {
        pos[count] = i;
        states[count] = state;
        matches[count] = M[state];
      }
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

/* The same generator continued from *state (updated): chunked generation of
 * multi-GiB inputs (tests/golden/make_config_d.py). */
void oracle_xorshift_continue(uint8_t* buf, uint64_t n, uint64_t* state)
{
  uint64_t x = *state;
  for (uint64_t i = 0; i < n; i++)
  {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    buf[i] = (uint8_t) (x >> 24);
  }
  *state = x;
}

/*
 * Literal pre-verification oracle.  For every
 * call (position i, pool index k) of a verify-call stream, decide whether
 * yr_scan_verify_match(ctx, &pool[k], data, size, base, i - backtrack[k]) can
 * have an effect, restating:
 *   - yr_scan_verify_match early outs (libyara/scan.c:1013 offset == size,
 *     :1023-1025 FIXED_OFFSET mismatch), literal vs re.c dispatch (:1036-1046);
 *   - _yr_scan_verify_literal_match (scan.c:887-990): FITS_IN_ATOM ->
 *     forward_matches = backtrack; NO_CASE -> ascii icompare then wide
 *     wicompare; else ascii compare, wide wcompare, then (XOR) wide xor then
 *     xor; no effect iff forward_matches == 0 (:974-975);
 *   - the comparisons _yr_scan_compare / icompare / wcompare / wicompare /
 *     xor_compare / xor_wcompare (scan.c:62-255), lowercase = yr_lowercase;
 *   - the FULL_WORD test of _yr_scan_match_callback (scan.c:672-694).
 * Base64 literal strings are not restated: always kept (as on the device).
 * Non-literal strings: decided by re_call_effect when the pool entry has a
 * fast-exec program (re_kind[k] == 1, tests/golden tables v2), else kept.
 * out[c] = 1 keep, 0 no effect.
 */
#define SF_NO_CASE 0x04u
#define SF_ASCII 0x08u
#define SF_WIDE 0x10u
#define SF_FULL_WORD 0x80u
#define SF_LITERAL 0x400u
#define SF_FITS_IN_ATOM 0x800u
#define SF_FIXED_OFFSET 0x8000u
#define SF_XOR 0x80000u
#define SF_BASE64_ANY (0x200000u | 0x400000u)

/* yr_isalnum (strutils.c:240-244) */
static int re_is_alnum(uint8_t c)
{
  return (c >= 0x30 && c <= 0x39) || (c >= 0x41 && c <= 0x5a) || (c >= 0x61 && c <= 0x7a);
}

static uint64_t fwd_plain(const uint8_t* d, uint64_t avail, const uint8_t* s, uint32_t n,
                          const uint8_t* low)
{
  if (avail < n) return 0;
  uint32_t i = 0;
  while (i < n && (low ? low[d[i]] == low[s[i]] : d[i] == s[i])) i++;
  return i == n ? n : 0;
}

static uint64_t fwd_wide(const uint8_t* d, uint64_t avail, const uint8_t* s, uint32_t n,
                         const uint8_t* low)
{
  if (avail < 2ull * n) return 0;
  uint32_t i = 0;
  while (i < n && (low ? low[d[2 * i]] == low[s[i]] : d[2 * i] == s[i]) && d[2 * i + 1] == 0) i++;
  return i == n ? 2ull * n : 0;
}

static uint64_t fwd_xor(const uint8_t* d, uint64_t avail, const uint8_t* s, uint32_t n, int wide)
{
  if (avail < (wide ? 2ull * n : (uint64_t) n)) return 0;
  uint8_t k = d[0] ^ s[0];
  uint32_t i = 0;
  if (wide)
    while (i < n && d[2 * i] == (uint8_t) (s[i] ^ k) && (uint8_t) (d[2 * i + 1] ^ k) == 0) i++;
  else
    while (i < n && d[i] == (uint8_t) (s[i] ^ k)) i++;
  return i == n ? (wide ? 2ull * n : n) : 0;
}

/*
 * Fast-exec regex restatement (hex strings, STRING_FLAGS_FAST_REGEXP): the
 * program is the linear opcode sequence yr_re_fast_exec runs (re.c:2150-2391).
 * The reference keeps a list of input positions and applies one opcode per
 * round to all of them; here the same rounds run over the SET of
 * bytes_matched values (a bitset over [0, YR_RE_SCAN_LIMIT]):
 *   ANY / LITERAL / NOT_LITERAL / MASKED_(NOT_)LITERAL: b -> b + 1 if
 *     b < max_bytes_matched and the byte at distance b (forward: input[b],
 *     backward: input[-1-b]) passes;
 *   REPEAT_ANY_UNGREEDY {min, max}: b -> b + min (if b < max_bytes_matched),
 *     and b + j for min < j <= max while b + j < max_bytes_matched;
 *   MATCH: a match iff the set is non-empty.
 * max_bytes_matched = min(available bytes in that direction, 4096)
 * (limits.h:163).  Returns 1 if a match is reachable, 0 otherwise.  (The set
 * is exact "exists a path" semantics, a superset of what the reference's
 * de-duplicating position list can reach: never says 0 where the reference
 * would match.)
 */
#define RE_SCAN_LIMIT 4096
#define RE_SET_WORDS ((RE_SCAN_LIMIT + 1 + 31) / 32 + 1)

static int fast_re_reachable(const uint8_t* code, uint32_t len, const uint8_t* input,
                             uint64_t avail, int backwards)
{
  uint32_t cur[RE_SET_WORDS], nxt[RE_SET_WORDS];
  int maxb = (int) (avail < RE_SCAN_LIMIT ? avail : RE_SCAN_LIMIT);
  memset(cur, 0, sizeof(cur));
  cur[0] = 1; /* bytes_matched = 0 */
  uint32_t ip = 0;
  while (ip < len)
  {
    uint8_t op = code[ip];
    if (op == 0xAD) /* MATCH */
    {
      for (int w = 0; w < RE_SET_WORDS; w++)
        if (cur[w]) return 1;
      return 0;
    }
    memset(nxt, 0, sizeof(nxt));
    int any = 0;
    for (int b = 0; b <= RE_SCAN_LIMIT; b++)
    {
      if (!((cur[b >> 5] >> (b & 31)) & 1)) continue;
      if (b >= maxb) continue; /* every opcode here needs b < max_bytes_matched */
      uint8_t c = backwards ? input[-1 - (int64_t) b] : input[b];
      int pass = 0;
      switch (op)
      {
      case 0xA0: pass = 1; break;
      case 0xA2: pass = c == code[ip + 1]; break;
      case 0xAE: pass = c != code[ip + 1]; break;
      case 0xA4: pass = (c & code[ip + 2]) == code[ip + 1]; break;
      case 0xAF: pass = (c & code[ip + 2]) != code[ip + 1]; break;
      case 0xB5:
      {
        int mn = code[ip + 1] | (code[ip + 2] << 8);
        int mx = code[ip + 3] | (code[ip + 4] << 8);
        if (b + mn <= RE_SCAN_LIMIT) nxt[(b + mn) >> 5] |= 1u << ((b + mn) & 31);
        for (int j = mn + 1; j <= mx && b + j < maxb; j++)
          nxt[(b + j) >> 5] |= 1u << ((b + j) & 31);
        any = 1;
        continue;
      }
      default: return 1; /* not a fast program: cannot rule a match out */
      }
      if (pass)
      {
        nxt[(b + 1) >> 5] |= 1u << ((b + 1) & 31);
        any = 1;
      }
    }
    if (!any) return 0;
    memcpy(cur, nxt, sizeof(cur));
    ip += op == 0xA0 ? 1 : (op == 0xA2 || op == 0xAE) ? 2 : (op == 0xA4 || op == 0xAF) ? 3 : 5;
  }
  return 1;
}

/*
 * yr_re_exec programs (re.c:1693-2072), same over-approximating question as
 * the product's general_re_reachable (verify.hip) and the same search order,
 * stack limit (16 open choices) and step budget (1000 < RE_MAX_FIBERS, so an
 * exec that would fail with ERROR_TOO_MANY_RE_FIBERS, re.c:1228, always runs
 * out): exhausting either, or unknown code, answers 2 = keep the call.
 * 0 = no path reaches MATCH, 1 = some path does.  Exact character tests: LITERAL (case-folded with `lower` under
 * NO_CASE), NOT/MASKED literals, CLASS (+ ASCII case swap under NO_CASE,
 * negation), ANY (newline unless DOT_ALL); every consumed character needs
 * bytes_matched < max_bytes_matched and, wide, a zero high byte.  SPLIT
 * branches, REPEAT_START (min 0: skip) / REPEAT_END (loop or leave),
 * REPEAT_ANY ranges, boundary/anchor assertions and \w\s\d are unconstrained.
 */
static int re_sz(uint8_t op)
{
  if (op == 0xA0 || (op >= 0xA7 && op <= 0xAD) || (op >= 0xB0 && op <= 0xB3)) return 1;
  if (op == 0xA2 || op == 0xAE) return 2;
  if (op == 0xA4 || op == 0xAF) return 3;
  if (op == 0xA5) return 34;
  if (op == 0xB4 || op == 0xB5) return 5;
  if (op == 0xC0 || op == 0xC1) return 4;
  if (op == 0xC2) return 3;
  if (op >= 0xC3 && op <= 0xC6) return 9;
  return 0;
}

/* _yr_re_is_word_char (re.c:114-122) with yr_isalnum (strutils.c:240-244) */
static int re_is_word(const uint8_t* ch, int cs)
{
  uint8_t c = ch[0];
  int w = (c >= 0x30 && c <= 0x39) || (c >= 0x41 && c <= 0x5a) || (c >= 0x61 && c <= 0x7a) ||
          c == '_';
  return cs == 2 ? (w && ch[1] == 0) : w;
}

/*
 * yr_re_exec (re.c:1693-2072) as "can some path reach MATCH": every opcode
 * with the reference's semantics -- character tests incl. \w \s \d, the
 * prolog, REPEAT_ANY ranges whose repeated characters pass ANY's test, counted
 * REPEAT_START/END loops with the fiber's counter stack (re.c:1533-1582), the
 * \b \B ^ $ assertions (re.c:1937-1981), both SPLIT branches.  Returns 0 (no
 * path), 1 (a path), 2 (budget of 1000 steps / 16 choices / 4 nested loops
 * exceeded, or unknown code: keep the call).  fwd/bwd = the input sizes
 * yr_re_exec receives (data_size - offset, offset; scan.c:820-876).
 */
static int general_reachable(const uint8_t* code, uint32_t len, const uint8_t* input,
                             uint64_t fwd, uint64_t bwd, int backwards, int wide, int nocase,
                             int dotall, const uint8_t* lower)
{
  struct { int32_t ip; int b, j, jmax, step, sp; uint16_t cnt[4]; } st[16];
  int csp = 0;
  int cs = wide ? 2 : 1;
  uint64_t avail = backwards ? bwd : fwd;
  int maxb = (int) (avail < RE_SCAN_LIMIT ? avail : RE_SCAN_LIMIT);
  maxb -= maxb % cs;
  int32_t ip = 0;
  int b = 0, sp = -1;
  uint16_t cnt[4] = {0, 0, 0, 0};
#define AT(bb) (backwards ? input - cs - (bb) : input + (bb))
#define PUSH(cip, cb, cj, cjmax, cstep)                                   \
  do {                                                                  \
    if (csp == 16) return 2;                                            \
    st[csp].ip = (cip); st[csp].b = (cb); st[csp].j = (cj);             \
    st[csp].jmax = (cjmax); st[csp].step = (cstep); st[csp].sp = sp;    \
    memcpy(st[csp].cnt, cnt, sizeof cnt);                               \
    csp++;                                                              \
  } while (0)
  for (int steps = 0; steps < 1000; steps++)
  {
    if (ip < 0 || (uint32_t) ip >= len) return 2;
    uint8_t op = code[ip];
    int alive = 1;
    if (op == 0xAD) return 1;
    if (op == 0xC2) { ip += (int16_t) (code[ip + 1] | (code[ip + 2] << 8)); continue; }
    if (op == 0xC0 || op == 0xC1)
    {
      PUSH(ip + (int16_t) (code[ip + 2] | (code[ip + 3] << 8)), b, 0, 0, 0);
      ip += 4;
      continue;
    }
    if (op >= 0xC3 && op <= 0xC6)
    {
      int32_t off = (int32_t) ((uint32_t) code[ip + 5] | ((uint32_t) code[ip + 6] << 8) |
                               ((uint32_t) code[ip + 7] << 16) | ((uint32_t) code[ip + 8] << 24));
      int mn = code[ip + 1] | (code[ip + 2] << 8), mx = code[ip + 3] | (code[ip + 4] << 8);
      if (op == 0xC3 || op == 0xC5)   /* REPEAT_START, re.c:1533-1553 */
      {
        if (mn == 0) PUSH(ip + off, b, 0, 0, 0);
        if (sp + 1 >= 4) return 2;
        cnt[++sp] = 0;
        ip += 9;
        continue;
      }
      /* REPEAT_END, re.c:1555-1582 */
      if (sp < 0) return 2;
      cnt[sp]++;
      if (cnt[sp] < mn) { ip += off; continue; }
      if (cnt[sp] < mx) PUSH(ip + off, b, 0, 0, 0);
      sp--;
      ip += 9;
      continue;
    }
    if (op == 0xB2 || op == 0xB3)   /* \b \B, re.c:1937-1965 */
    {
      int m;
      if (b == 0 && bwd < (uint64_t) cs) m = 1;
      else if (b >= maxb) m = 1;
      else
      {
        const uint8_t* cur = AT(b);
        m = re_is_word(cur, cs) != re_is_word(backwards ? cur + cs : cur - cs, cs);
      }
      if (op == 0xB3) m = !m;
      alive = m;
      ip += 1;
    }
    else if (op == 0xB1)   /* ^, re.c:1967-1974 */
    {
      alive = backwards ? !(bwd > (uint64_t) b) : !(bwd > 0 || b != 0);
      ip += 1;
    }
    else if (op == 0xB0)   /* $, re.c:1976-1981 */
    {
      alive = !(backwards || fwd > (uint64_t) b);
      ip += 1;
    }
    else if (op == 0xB4 || op == 0xB5)   /* REPEAT_ANY, re.c:1810-1821, :1584-1641 */
    {
      int mn = code[ip + 1] | (code[ip + 2] << 8), mx = code[ip + 3] | (code[ip + 4] << 8);
      int k = 0;
      while (k < mx)
      {
        int bb = b + k * cs;
        if (bb >= maxb) break;
        const uint8_t* ch = AT(bb);
        if ((wide && ch[1] != 0) || (!dotall && ch[0] == 0x0A)) break;
        k++;
      }
      if (k < mn) alive = 0;
      else
      {
        if (mn < k) PUSH(ip + 5, b, mn + 1, k, cs);
        b += mn * cs;
        ip += 5;
        continue;
      }
    }
    else
    {
      int sz = re_sz(op);
      if (sz == 0) return 2;
      if (b >= maxb) alive = 0;
      else
      {
        const uint8_t* ch = AT(b);
        if (wide && ch[1] != 0) alive = 0;
        else
        {
          uint8_t c = ch[0];
          int ok = 1;
          switch (op)
          {
          case 0xA0: ok = dotall || c != 0x0A; break;
          case 0xA2: ok = nocase ? lower[c] == lower[code[ip + 1]] : c == code[ip + 1]; break;
          case 0xAE: ok = c != code[ip + 1]; break;
          case 0xA4: ok = (c & code[ip + 2]) == code[ip + 1]; break;
          case 0xAF: ok = (c & code[ip + 2]) != code[ip + 1]; break;
          case 0xA5:
          {
            const uint8_t* bm = code + ip + 2;
            int in = (bm[c / 8] >> (c % 8)) & 1;
            if (nocase)
            {
              uint8_t a = (c >= 'a' && c <= 'z') ? c - 32 : (c >= 'A' && c <= 'Z') ? c + 32 : c;
              in = in || ((bm[a / 8] >> (a % 8)) & 1);
            }
            ok = code[ip + 1] ? !in : in;
            break;
          }
          case 0xA7: ok = re_is_word(ch, cs); break;
          case 0xA8: ok = !re_is_word(ch, cs); break;
          case 0xA9:
          case 0xAA:
          {
            int s_ = c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f';
            ok = op == 0xA9 ? s_ : !s_;
            break;
          }
          case 0xAB: ok = c >= '0' && c <= '9'; break;
          case 0xAC: ok = !(c >= '0' && c <= '9'); break;
          default: ok = 1;
          }
          if (!ok) alive = 0;
          else { b += cs; ip += sz; continue; }
        }
      }
    }
    if (alive) continue;
    if (csp == 0) return 0;
    ip = st[csp - 1].ip;
    b = st[csp - 1].b + st[csp - 1].j * st[csp - 1].step;
    sp = st[csp - 1].sp;
    memcpy(cnt, st[csp - 1].cnt, sizeof cnt);
    if (++st[csp - 1].j > st[csp - 1].jmax) csp--;
  }
#undef AT
#undef PUSH
  return 2;
}

/*
 * Does a yr_re_exec regex call have a possible effect?  _yr_scan_verify_re_match
 * (scan.c:817-848): the ascii attempt runs for ASCII / base64 strings, the wide
 * one for WIDE non-base64 strings when the ascii one found nothing, the
 * backward program with the flags of the attempt that matched.  Since a "1"
 * forward answer may be a reference miss, every attempt is tried; an answer of
 * 2 (search exhausted) keeps the call.
 */
static int general_call_effect(uint32_t flags, const uint8_t* fwd, uint32_t fl, const uint8_t* bwd,
                               uint32_t bl, const uint8_t* data, uint64_t size, uint64_t off,
                               const uint8_t* lower)
{
  /* scan.c:817-848: ascii attempt for ASCII/base64 strings, wide attempt for
   * WIDE non-base64 strings; the backward program with the matching flags */
  int nocase = (flags & SF_NO_CASE) != 0, dotall = (flags & 0x20000u) != 0;
  int try_ascii = (flags & (SF_ASCII | SF_BASE64_ANY)) != 0;
  int try_wide = (flags & SF_WIDE) && !(flags & SF_BASE64_ANY);
  for (int w = 0; w < 2; w++)
  {
    if (w == 0 ? !try_ascii : !try_wide) continue;
    int f = general_reachable(fwd, fl, data + off, size - off, off, 0, w, nocase, dotall, lower);
    if (f == 2) return 1;
    if (f == 0) continue;
    if (bl == 0 ||
        general_reachable(bwd, bl, data + off, size - off, off, 1, w, nocase, dotall, lower) != 0)
      return 1;
  }
  return 0;
}

/*
 * FAST (hex) strings, _yr_scan_verify_re_match (scan.c:778-880) with
 * yr_re_fast_exec: the forward program from `off` must match
 * (forward_matches != -1); with a backward program its MATCHes are what reach
 * _yr_scan_match_callback; forward_matches == 0 without one returns early.
 * Only ascii hex strings are decided.
 */
static int re_call_effect(uint32_t flags, const uint8_t* fwd, uint32_t fl, const uint8_t* bwd,
                          uint32_t bl, const uint8_t* data, uint64_t size, uint64_t off)
{
  if (!(flags & 0x40u) || !(flags & SF_ASCII) || (flags & (SF_WIDE | SF_BASE64_ANY)))
    return 1;
  if (fl == 1) /* forward program = MATCH: forward_matches = 0 */
    return bl > 0 ? fast_re_reachable(bwd, bl, data + off, off, 1) : 0;
  if (!fast_re_reachable(fwd, fl, data + off, size - off, 0)) return 0;
  if (bl > 0 && !fast_re_reachable(bwd, bl, data + off, off, 1)) return 0;
  return 1;
}

int64_t oracle_literal_effect(
    const uint64_t* pos, const uint32_t* pool_idx, uint64_t n_calls,
    const uint16_t* backtrack, const uint32_t* pool_string,
    const uint32_t* str_flags, const uint32_t* str_len, const int64_t* str_fixed,
    const uint64_t* str_off, const uint8_t* blob, const uint8_t* lowercase,
    const uint8_t* data, uint64_t size, uint64_t base, uint8_t* out,
    const uint8_t* re_kind, const uint32_t* re_fwd_off, const uint32_t* re_fwd_len,
    const uint32_t* re_bwd_off, const uint32_t* re_bwd_len, const uint8_t* re_code)
{
  int64_t kept = 0;
  for (uint64_t c = 0; c < n_calls; c++)
  {
    uint32_t k = pool_idx[c];
    uint64_t off = pos[c] - backtrack[k];
    uint32_t s = pool_string[k];
    uint32_t f = str_flags[s];
    uint64_t fm = 1; /* forward_matches != 0, or "not decided here" */
    if (off == size)
      fm = 0;
    else if ((f & SF_FIXED_OFFSET) && str_fixed[s] != (int64_t) (base + off))
      fm = 0;
    else if ((f & SF_LITERAL) && !(f & SF_BASE64_ANY))
    {
      const uint8_t* d = data + off;
      uint64_t avail = size - off;
      const uint8_t* str = blob + str_off[s];
      uint32_t n = str_len[s];
      if (f & SF_FITS_IN_ATOM)
        fm = backtrack[k];
      else if (f & SF_NO_CASE)
      {
        fm = 0;
        if (f & SF_ASCII) fm = fwd_plain(d, avail, str, n, lowercase);
        if ((f & SF_WIDE) && fm == 0) fm = fwd_wide(d, avail, str, n, lowercase);
      }
      else
      {
        fm = 0;
        if (f & SF_ASCII) fm = fwd_plain(d, avail, str, n, NULL);
        if ((f & SF_WIDE) && fm == 0) fm = fwd_wide(d, avail, str, n, NULL);
        if ((f & SF_XOR) && fm == 0)
        {
          if (f & SF_WIDE) fm = fwd_xor(d, avail, str, n, 1);
          if (fm == 0) fm = fwd_xor(d, avail, str, n, 0);
        }
      }
      /* _yr_scan_match_callback (scan.c:672-694): a FULL_WORD match touching an
       * alphanumeric character (yr_isalnum, strutils.c:240-244) is dropped;
       * wide (forward_matches == 2 * length, scan.c:977-978): an alphanumeric
       * followed by 0x00 */
      if (fm != 0 && (f & SF_FULL_WORD))
      {
        if (fm == 2ull * n)
        {
          if (off >= 2 && data[off - 1] == 0 && re_is_alnum(data[off - 2])) fm = 0;
          else if (off + fm + 1 < size && data[off + fm + 1] == 0 && re_is_alnum(data[off + fm]))
            fm = 0;
        }
        else
        {
          if (off >= 1 && re_is_alnum(data[off - 1])) fm = 0;
          else if (off + fm < size && re_is_alnum(data[off + fm])) fm = 0;
        }
      }
    }
    else if (!(f & SF_LITERAL) && re_kind != NULL && re_kind[k] == 1)
    {
      fm = re_call_effect(f, re_code + re_fwd_off[k], re_fwd_len[k], re_code + re_bwd_off[k],
                          re_bwd_len[k], data, size, off);
    }
    else if (!(f & SF_LITERAL) && re_kind != NULL && re_kind[k] == 2)
    {
      fm = general_call_effect(f, re_code + re_fwd_off[k], re_fwd_len[k], re_code + re_bwd_off[k],
                               re_bwd_len[k], data, size, off, lowercase);
    }
    out[c] = fm != 0;
    kept += fm != 0;
  }
  return kept;
}
