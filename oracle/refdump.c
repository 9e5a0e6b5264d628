/*
 * refdump -- golden-vector generator driven by the REFERENCE libyara
 * (test infrastructure only; links oracle/_ref/libyara_ref_hooked.so).
 *
 *   refdump tables <rules.yar> <out.bin>
 *       Compile with the stock compiler (compiler.c:632/703) and dump the
 *       Aho-Corasick tables exactly as YR_RULES exposes them (rules.c:356-363):
 *       T = ac_transition_table, M = ac_match_table, and the YR_AC_MATCH pool
 *       (types.h:324-344) with `next` turned into a 1-based pool index.  Also
 *       dumps the YR_STRING records (types.h:238-287) the verifier uses and,
 *       for FAST_REGEXP strings (hex strings), each pool entry's forward and
 *       backward RE code (re.c fast-exec opcodes, decoded linearly up to
 *       RE_OPCODE_MATCH).
 *
 *   refdump scan <rules.yar> <data> <out_prefix> [block_size overlap]
 *       <data> is a file path, "xs:<seed>:<size>" (SURVEY.md App. A
 *       xorshift64 generator) or "xst:<state>:<size>" (the same generator
 *       continued from a raw state, e.g. oracle.xorshift_state(seed, offset):
 *       bytes [offset, offset + size) of the seed's stream).  Runs stock yr_rules_scan_mem (or
 *       yr_rules_scan_mem_blocks with the tests/util.c-style overlapping block
 *       iterator) and records
 *         <out>.verify   every call the hot loop makes to yr_scan_verify_match:
 *                        {u64 block_base, u64 position i, u32 pool index}
 *         <out>.matches  the final match set, every string, private included:
 *                        {u32 string idx, i64 base+offset, i32 len, u32 xor}
 *         <out>.rules    one byte per rule: 1 = RULE_MATCHING
 *
 * Output is little-endian packed binary parsed by tests/golden/make_golden.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <yara.h>
#include <yara/arena.h>
#include <yara/compiler.h>
#include <yara/types.h>

typedef void (*yr_refhook_fn)(void* user, const YR_AC_MATCH* m, size_t offset);
extern yr_refhook_fn yr_refhook_cb;
extern void* yr_refhook_user;

static void die(const char* msg, int code)
{
  fprintf(stderr, "refdump: %s (%d)\n", msg, code);
  exit(2);
}

static void compiler_cb(
    int error_level,
    const char* file_name,
    int line_number,
    const YR_RULE* rule,
    const char* message,
    void* user_data)
{
  if (error_level == YARA_ERROR_LEVEL_ERROR)
    fprintf(stderr, "refdump: %s:%d: %s\n", file_name ? file_name : "-",
            line_number, message);
}

static YR_RULES* compile_rules(const char* path)
{
  YR_COMPILER* c;
  YR_RULES* rules;
  FILE* f = fopen(path, "r");
  if (!f) die("cannot open rules", 0);
  int r = yr_compiler_create(&c);
  if (r != ERROR_SUCCESS) die("compiler_create", r);
  yr_compiler_set_callback(c, compiler_cb, NULL);
  if (yr_compiler_add_file(c, f, NULL, path) != 0) die("compile errors", 0);
  fclose(f);
  r = yr_compiler_get_rules(c, &rules);
  if (r != ERROR_SUCCESS) die("get_rules", r);
  yr_compiler_destroy(c);
  return rules;
}

static uint32_t n_slots_of(YR_RULES* rules)
{
  return (uint32_t) (yr_arena_get_current_offset(
                         rules->arena, YR_AC_TRANSITION_TABLE) /
                     sizeof(YR_AC_TRANSITION));
}

static uint32_t n_pool_of(YR_RULES* rules)
{
  return (uint32_t) (yr_arena_get_current_offset(
                         rules->arena, YR_AC_STATE_MATCHES_POOL) /
                     sizeof(YR_AC_MATCH));
}

/* Length (incl. the final MATCH) of a linear fast-exec program (the opcodes
 * yr_re_fast_exec accepts, re.c:2150-2391), or 0 if `code` is not one. */
static uint32_t fast_code_len(const uint8_t* code)
{
  uint32_t n = 0;
  while (n < 65536)
  {
    switch (code[n])
    {
    case 0xA0: n += 1; break;             /* ANY */
    case 0xA2: case 0xAE: n += 2; break;  /* LITERAL, NOT_LITERAL */
    case 0xA4: case 0xAF: n += 3; break;  /* MASKED_LITERAL, MASKED_NOT_LITERAL */
    case 0xB5: n += 5; break;             /* REPEAT_ANY_UNGREEDY {u16 min, u16 max} */
    case 0xAD: return n + 1;              /* MATCH */
    default: return 0;
    }
  }
  return 0;
}

/* Size of one regexp instruction (re.h:65-92 opcodes, re.c:65-87 operands), 0 if unknown. */
static uint32_t re_insn_size(uint8_t op)
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

/* Extent of a yr_re_exec program: furthest end of an instruction reachable
 * from its start (jumps, splits, repeat back/forward offsets), 0 if invalid. */
static uint32_t general_code_len(const uint8_t* code, size_t avail)
{
  if (avail == 0 || avail > (1u << 20)) avail = avail ? (1u << 20) : 0;
  if (avail == 0) return 0;
  uint8_t* seen = calloc(avail, 1);
  int64_t* todo = malloc(sizeof(int64_t) * (avail + 1));
  size_t nt = 0;
  uint64_t end = 0;
  int ok = 1;
  todo[nt++] = 0;
  while (nt > 0 && ok)
  {
    int64_t ip = todo[--nt];
    for (;;)
    {
      if (ip < 0 || (uint64_t) ip >= avail) { ok = 0; break; }
      if (seen[ip]) break;
      seen[ip] = 1;
      uint8_t op = code[ip];
      uint32_t sz = re_insn_size(op);
      if (sz == 0 || (uint64_t) ip + sz > avail) { ok = 0; break; }
      if ((uint64_t) ip + sz > end) end = ip + sz;
      if (op == 0xAD) break;
      if (op == 0xC2) { ip += (int16_t) (code[ip + 1] | (code[ip + 2] << 8)); continue; }
      if ((op == 0xC0 || op == 0xC1) && nt < avail)
        todo[nt++] = ip + (int16_t) (code[ip + 2] | (code[ip + 3] << 8));
      if (op >= 0xC3 && op <= 0xC6 && nt < avail)
      {
        int32_t off = (int32_t) ((uint32_t) code[ip + 5] | ((uint32_t) code[ip + 6] << 8) |
                                 ((uint32_t) code[ip + 7] << 16) | ((uint32_t) code[ip + 8] << 24));
        todo[nt++] = ip + off;
      }
      ip += sz;
    }
  }
  free(seen);
  free(todo);
  return ok ? (uint32_t) end : 0;
}

static void w32(FILE* f, uint32_t v) { fwrite(&v, 4, 1, f); }
static void w64(FILE* f, uint64_t v) { fwrite(&v, 8, 1, f); }

static int cmd_tables(const char* rules_path, const char* out)
{
  YR_RULES* rules = compile_rules(rules_path);
  uint32_t ns = n_slots_of(rules), np = n_pool_of(rules);
  FILE* f = fopen(out, "wb");
  if (!f) die("cannot open output", 0);
  fwrite("YRTB", 4, 1, f);
  w32(f, 2);
  w32(f, ns);
  w32(f, np);
  w32(f, rules->num_strings);
  w32(f, rules->num_rules);
  fwrite(rules->ac_transition_table, 4, ns, f);
  fwrite(rules->ac_match_table, 4, ns, f);
  for (uint32_t k = 0; k < np; k++)
  {
    YR_AC_MATCH* m = &rules->ac_match_pool[k];
    w32(f, m->next ? (uint32_t) (m->next - rules->ac_match_pool) + 1 : 0);
    w32(f, m->string->idx);
    w32(f, m->backtrack);
  }
  for (uint32_t k = 0; k < rules->num_strings; k++)
  {
    YR_STRING* s = &rules->strings_table[k];
    w32(f, s->flags);
    w32(f, s->rule_idx);
    w32(f, (uint32_t) s->length);
    w32(f, s->chained_to ? s->chained_to->idx : 0xFFFFFFFFu);
    w32(f, (uint32_t) s->chain_gap_min);
    w32(f, (uint32_t) s->chain_gap_max);
    w64(f, (uint64_t) s->fixed_offset);
    fwrite(s->string, 1, s->length, f);
    static const uint8_t pad[4] = {0, 0, 0, 0};
    fwrite(pad, 1, (4 - (s->length & 3)) & 3, f);
  }
  /* v2: per pool entry {u32 kind, u32 fwd_len, u32 bwd_len, fwd, bwd, pad};
   * kind 1 = FAST_REGEXP string with linear forward (and, if bwd_len > 0,
   * backward) programs; kind 2 = other regexp string, every instruction of its
   * yr_re_exec programs reachable from their start; kind 0 = anything else. */
  const uint8_t* re_base = yr_arena_get_ptr(rules->arena, YR_RE_CODE_SECTION, 0);
  size_t re_size = yr_arena_get_current_offset(rules->arena, YR_RE_CODE_SECTION);
  for (uint32_t k = 0; k < np; k++)
  {
    YR_AC_MATCH* m = &rules->ac_match_pool[k];
    uint32_t kind = 0, fl = 0, bl = 0;
    if ((m->string->flags & STRING_FLAGS_FAST_REGEXP) && m->forward_code != NULL)
    {
      fl = fast_code_len(m->forward_code);
      bl = m->backward_code ? fast_code_len(m->backward_code) : 0;
      kind = fl > 0 && (m->backward_code == NULL || bl > 0);
      if (!kind) fl = bl = 0;
    }
    else if (!(m->string->flags & STRING_FLAGS_LITERAL) && m->forward_code != NULL &&
             m->forward_code >= re_base && m->forward_code < re_base + re_size)
    {
      fl = general_code_len(m->forward_code, re_base + re_size - m->forward_code);
      bl = 0;
      if (m->backward_code != NULL)
        bl = m->backward_code >= re_base && m->backward_code < re_base + re_size
                 ? general_code_len(m->backward_code, re_base + re_size - m->backward_code)
                 : 0;
      kind = fl > 0 && (m->backward_code == NULL || bl > 0) ? 2 : 0;
      if (!kind) fl = bl = 0;
    }
    w32(f, kind);
    w32(f, fl);
    w32(f, bl);
    if (fl) fwrite(m->forward_code, 1, fl, f);
    if (bl) fwrite(m->backward_code, 1, bl, f);
    static const uint8_t pad[4] = {0, 0, 0, 0};
    fwrite(pad, 1, (4 - ((fl + bl) & 3)) & 3, f);
  }
  fclose(f);
  printf("slots=%u pool=%u strings=%u rules=%u\n", ns, np, rules->num_strings,
         rules->num_rules);
  yr_rules_destroy(rules);
  return 0;
}

/* SURVEY.md Appendix A canonical buffer generator. */
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

static void xorshift_continue(uint8_t* buf, size_t n, uint64_t x)
{
  for (size_t i = 0; i < n; i++)
  {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    buf[i] = (uint8_t) (x >> 24);
  }
}

static uint8_t* load_data(const char* spec, size_t* size)
{
  if (strncmp(spec, "xst:", 4) == 0)
  {
    unsigned long long state, n;
    if (sscanf(spec + 4, "%llu:%llu", &state, &n) != 2) die("bad xst spec", 0);
    uint8_t* b = malloc(n ? n : 1);
    if (!b) die("oom", 0);
    xorshift_continue(b, n, state);
    *size = n;
    return b;
  }
  if (strncmp(spec, "xs:", 3) == 0)
  {
    unsigned long long seed, n;
    if (sscanf(spec + 3, "%llu:%llu", &seed, &n) != 2) die("bad xs spec", 0);
    uint8_t* b = malloc(n ? n : 1);
    if (!b) die("oom", 0);
    xorshift_fill(b, n, seed);
    *size = n;
    return b;
  }
  FILE* f = fopen(spec, "rb");
  if (!f) die("cannot open data", 0);
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* b = malloc(n ? n : 1);
  if (fread(b, 1, n, f) != (size_t) n) die("short read", 0);
  fclose(f);
  *size = (size_t) n;
  return b;
}

typedef struct
{
  YR_RULES* rules;
  FILE* verify;
  uint64_t block_base;
  uint64_t n_calls;
} hook_state;

static void on_verify(void* user, const YR_AC_MATCH* m, size_t offset)
{
  hook_state* h = (hook_state*) user;
  uint64_t pos = (uint64_t) offset + m->backtrack;
  uint32_t idx = (uint32_t) (m - h->rules->ac_match_pool);
  w64(h->verify, h->block_base);
  w64(h->verify, pos);
  w32(h->verify, idx);
  h->n_calls++;
}

typedef struct
{
  FILE* matches;
  uint8_t* rule_flags;
  YR_RULES* rules;
  int dumped;
} scan_state;

static void dump_all_matches(YR_SCAN_CONTEXT* ctx, scan_state* s)
{
  for (uint32_t k = 0; k < s->rules->num_strings; k++)
  {
    for (YR_MATCH* m = ctx->matches[k].head; m != NULL; m = m->next)
    {
      w32(s->matches, k);
      w64(s->matches, (uint64_t) (m->base + m->offset));
      w32(s->matches, (uint32_t) m->match_length);
      w32(s->matches, m->xor_key);
    }
  }
}

static int scan_cb(YR_SCAN_CONTEXT* ctx, int msg, void* data, void* user)
{
  scan_state* s = (scan_state*) user;
  if (msg == CALLBACK_MSG_RULE_MATCHING || msg == CALLBACK_MSG_RULE_NOT_MATCHING)
  {
    YR_RULE* rule = (YR_RULE*) data;
    uint32_t idx = (uint32_t) (rule - s->rules->rules_table);
    s->rule_flags[idx] = (msg == CALLBACK_MSG_RULE_MATCHING);
    if (!s->dumped)
    {
      /* Match lists are final once the report loop starts (scanner.c:524). */
      dump_all_matches(ctx, s);
      s->dumped = 1;
    }
  }
  return CALLBACK_CONTINUE;
}

/* Overlapping fixed-size block iterator, the semantics of tests/util.c:136-209
 * (each block is scanned independently, base = its offset in the buffer). */
typedef struct
{
  const uint8_t* data;
  size_t size, bsize, overlap, next_base;
  YR_MEMORY_BLOCK blk;
  hook_state* hook;
} blk_iter;

static const uint8_t* blk_fetch(YR_MEMORY_BLOCK* b)
{
  blk_iter* it = (blk_iter*) b->context;
  it->hook->block_base = b->base;
  return it->data + b->base;
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
  it->next_base = base + len >= it->size ? it->size
                                          : base + len - it->overlap;
  return &it->blk;
}

static YR_MEMORY_BLOCK* blk_first(YR_MEMORY_BLOCK_ITERATOR* iter)
{
  blk_iter* it = (blk_iter*) iter->context;
  it->next_base = 0;
  if (it->size == 0)
  {
    it->blk.base = 0;
    it->blk.size = 0;
    it->blk.context = it;
    it->blk.fetch_data = blk_fetch;
    it->next_base = 1;
    return &it->blk;
  }
  return blk_next(iter);
}

static int cmd_scan(int argc, char** argv)
{
  const char* rules_path = argv[2];
  const char* spec = argv[3];
  const char* prefix = argv[4];
  size_t bsize = argc > 5 ? strtoull(argv[5], NULL, 10) : 0;
  size_t overlap = argc > 6 ? strtoull(argv[6], NULL, 10) : 0;

  YR_RULES* rules = compile_rules(rules_path);
  size_t n;
  uint8_t* data = load_data(spec, &n);

  char path[4096];
  snprintf(path, sizeof(path), "%s.verify", prefix);
  hook_state hook = {rules, fopen(path, "wb"), 0, 0};
  snprintf(path, sizeof(path), "%s.matches", prefix);
  scan_state ss = {fopen(path, "wb"), calloc(rules->num_rules + 1, 1), rules, 0};
  if (!hook.verify || !ss.matches) die("cannot open outputs", 0);

  yr_refhook_user = &hook;
  yr_refhook_cb = on_verify;
  int r;
  if (bsize == 0)
  {
    r = yr_rules_scan_mem(rules, data, n, 0, scan_cb, &ss, 0);
  }
  else
  {
    blk_iter it = {data, n, bsize, overlap, 0};
    it.hook = &hook;
    YR_MEMORY_BLOCK_ITERATOR iter;
    iter.context = &it;
    iter.first = blk_first;
    iter.next = blk_next;
    iter.file_size = NULL;
    iter.last_error = ERROR_SUCCESS;
    r = yr_rules_scan_mem_blocks(rules, &iter, 0, scan_cb, &ss, 0);
  }
  yr_refhook_cb = NULL;
  fclose(hook.verify);
  fclose(ss.matches);
  snprintf(path, sizeof(path), "%s.rules", prefix);
  FILE* f = fopen(path, "wb");
  fwrite(ss.rule_flags, 1, rules->num_rules, f);
  fclose(f);
  printf("rc=%d size=%zu verify_calls=%llu\n", r, n,
         (unsigned long long) hook.n_calls);
  free(data);
  yr_rules_destroy(rules);
  return r;
}

int main(int argc, char** argv)
{
  if (argc < 4)
  {
    fprintf(stderr, "usage: refdump tables|scan ...\n");
    return 2;
  }
  yr_initialize();
  int r;
  if (strcmp(argv[1], "tables") == 0)
    r = cmd_tables(argv[2], argv[3]);
  else if (strcmp(argv[1], "scan") == 0 && argc >= 5)
    r = cmd_scan(argc, argv);
  else
  {
    fprintf(stderr, "bad command\n");
    r = 2;
  }
  yr_finalize();
  return r;
}
