/*
 * yara_amd.h -- C ABI of the MI355X (gfx950) Aho-Corasick atom scanner.
 *
 * Drop-in boundary for libyara's per-block AC walk.  In the reference
 * (HoundThe/yara, libyara 4.2.1) the walk is the static function
 *
 *     static int _yr_scanner_scan_mem_block(YR_SCANNER* scanner,
 *         const uint8_t* block_data, YR_MEMORY_BLOCK* block);
 *                                          -- libyara/scanner.c:45-176
 *
 * called only from yr_scanner_scan_mem_blocks (scanner.c:495).  Being static it
 * cannot be interposed; a maintainer replaces the call site with the three
 * steps below (INTEGRATION.md shows the patch and the binding):
 *
 *   1. yr_amd_tables_create   once per YR_RULES: flatten the tables the rules
 *                             compiler built (rules->ac_transition_table,
 *                             rules->ac_match_table, rules->ac_match_pool;
 *                             rules.c:356-363) into HBM-resident scan tables.
 *   2. yr_amd_scan_block      per YR_MEMORY_BLOCK: the GPU walk.  Returns the
 *                             ascending positions i in [0, size] at which the
 *                             reference loop finds ac_match_table[state] != 0
 *                             (scanner.c:98 and :144) -- the candidate stream.
 *   3. yr_amd_replay          hands every candidate, in the reference's order,
 *                             to the caller's verifier: for each i, the match
 *                             list of state_i is walked exactly like
 *                             scanner.c:105-121 and the callback receives
 *                             (pool index k, offset i - backtrack) for every
 *                             entry with backtrack <= i -- i.e. the arguments
 *                             of yr_scan_verify_match (scan.c:992).
 *
 * Conventions follow libyara: every function returns an int error code
 * (ERROR_SUCCESS = 0; codes and values from libyara/include/yara/error.h:40-109,
 * repeated below), tables are immutable after creation and may be shared by
 * any number of scanners/threads (as YR_RULES is, docs/capi.rst:330-347), and a
 * scanner is used by one thread at a time (as YR_SCANNER is, scanner.h).
 * No torch / HIP types appear in the signatures: streams are passed as void*
 * (a hipStream_t, or NULL for the scanner's own stream).
 */
#ifndef YARA_AMD_H
#define YARA_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes: identical values to libyara/include/yara/error.h. */
#define YR_AMD_SUCCESS                0   /* ERROR_SUCCESS */
#define YR_AMD_INSUFFICIENT_MEMORY    1   /* ERROR_INSUFFICIENT_MEMORY */
#define YR_AMD_COULD_NOT_MAP_FILE     4   /* ERROR_COULD_NOT_MAP_FILE (H2D of block data failed) */
#define YR_AMD_SCAN_TIMEOUT          26   /* ERROR_SCAN_TIMEOUT */
#define YR_AMD_CALLBACK_ERROR        28   /* ERROR_CALLBACK_ERROR */
#define YR_AMD_INVALID_ARGUMENT      29   /* ERROR_INVALID_ARGUMENT */
#define YR_AMD_INTERNAL_FATAL_ERROR  31   /* ERROR_INTERNAL_FATAL_ERROR (HIP failure) */

/* Max trie depth the kernels handle: YR_MAX_ATOM_LENGTH (limits.h:68). */
#define YR_AMD_MAX_ATOM_LENGTH 4

typedef struct yr_amd_tables yr_amd_tables;
typedef struct yr_amd_scanner yr_amd_scanner;

/*
 * Build device tables from the reference's compiled AC tables.
 *
 *   transition_table  rules->ac_transition_table, n_slots entries
 *                     (YR_AC_TRANSITION = uint32, ahocorasick.h:37-50)
 *   match_table       rules->ac_match_table, n_slots entries (1-based pool
 *                     index, 0 = no matches; ahocorasick.c:611-618)
 *   pool_next         for k in [0, n_pool): 1-based pool index of
 *                     rules->ac_match_pool[k].next, 0 when next == NULL
 *   pool_backtrack    rules->ac_match_pool[k].backtrack (types.h:343)
 *   device            HIP device ordinal the tables live on, or -1 for
 *                     host-only tables (flattening + yr_amd_replay only; no
 *                     scanner can be created on them)
 *
 * n_slots = yr_arena_get_current_offset(arena, YR_AC_TRANSITION_TABLE) /
 *           sizeof(YR_AC_TRANSITION)                         (rules.c:442-444)
 * Returns YR_AMD_INVALID_ARGUMENT if the trie is deeper than
 * YR_AMD_MAX_ATOM_LENGTH or the tables are malformed.
 */
int yr_amd_tables_create(
    const uint32_t* transition_table,
    const uint32_t* match_table,
    uint32_t n_slots,
    const uint32_t* pool_next,
    const uint16_t* pool_backtrack,
    uint32_t n_pool,
    int device,
    yr_amd_tables** tables);

int yr_amd_tables_destroy(yr_amd_tables* tables);

/*
 * The same tables straight from a compiled rules file (SURVEY.md section 8f,
 * row 3): the bytes of a .yarc written by yarac / yr_rules_save (arena format
 * version 19, arena.c:543-700, sections compiler.h:58-69), parsed without
 * libyara.  With device >= 0 the string records and the strings' regex
 * programs are attached too (yr_amd_tables_set_strings with C-locale case
 * folding, yr_amd_tables_set_re_code), so pre-verification works directly.
 * YR_AMD_INVALID_ARGUMENT for anything that is not a well-formed v19 arena.
 */
int yr_amd_tables_load_yarc(
    const uint8_t* file,
    size_t file_size,
    int device,
    yr_amd_tables** tables);

/* Diagnostics of the flattened form (yr_rules_get_stats analogue, rules.c:438). */
typedef struct
{
  uint32_t n_slots;
  uint32_t n_states;           /* trie nodes incl. root */
  uint32_t max_depth;
  uint32_t states_by_depth[YR_AMD_MAX_ATOM_LENGTH + 1];
  uint32_t accepting_states;   /* states with ac_match_table != 0 */
  uint32_t keys_by_length[YR_AMD_MAX_ATOM_LENGTH + 1]; /* minimal accepting suffixes */
  uint32_t root_accepting;     /* 1: every position is a candidate */
  uint32_t filter_bits;        /* log2 of the LDS window-filter size in bits */
  uint32_t filter_set_bits;    /* populated bits of that filter */
  uint32_t exact_slots;        /* slots of the HBM exact-suffix hash table */
  uint32_t max_backtrack;      /* max YR_AC_MATCH.backtrack of the pool */
  /* Bytes a shard must hold before / after the positions it owns for
   * yr_amd_verify_device to decide every call exactly as on the whole block
   * (yr_amd_scan_window): max_backtrack + YR_RE_SCAN_LIMIT (limits.h:163)
   * before, max(YR_RE_SCAN_LIMIT, 2 * longest string) after.  Without string
   * records (candidates only): the 4-byte warm-up before, 0 after. */
  uint64_t verify_halo_before;
  uint64_t verify_halo_after;
  /* Stage-1 filter form: 0 = pair filter (every position's window), 1 =
   * even-position filter (rule sets whose keys are all 4 bytes long: the
   * windows ending at even positions only, each key's prefix and suffix),
   * 2 = the same with a hashed block index. */
  uint32_t filter_mode;
} yr_amd_tables_info;

int yr_amd_tables_get_info(const yr_amd_tables* tables, yr_amd_tables_info* info);

/*
 * A scanner owns a HIP stream and the device workspace for one scan at a time.
 * stream: a hipStream_t to run on, or NULL to create a private stream.
 */
int yr_amd_scanner_create(
    yr_amd_tables* tables,
    void* stream,
    yr_amd_scanner** scanner);

int yr_amd_scanner_destroy(yr_amd_scanner* scanner);

/*
 * Scan one block that lives in HOST memory (the _yr_scanner_scan_mem_block
 * replacement).  The block is copied to HBM, scanned, and the candidate
 * stream copied back.  On success *positions points to *count ascending
 * positions in [0, size], owned by the scanner and valid until its next scan.
 * If *all_positions is set the rules have a non-empty root match list
 * (ac_match_table[0] != 0): every position 0..size is a candidate and the
 * positions array is empty.
 */
int yr_amd_scan_block(
    yr_amd_scanner* scanner,
    const uint8_t* data,
    size_t size,
    const uint64_t** positions,
    uint64_t* count,
    int* all_positions);

/*
 * Device-resident scan (the hot path the benchmark times): data is already in
 * HBM.  Scans the bytes [byte_begin, byte_end) of a block of block_size bytes,
 * i.e. reports candidate positions i in (byte_begin, byte_end] (position 0 is
 * reported iff byte_begin == 0 and the root is accepting), reading up to
 * YR_AMD_MAX_ATOM_LENGTH bytes before byte_begin as warm-up.  Shards of one
 * block scanned this way concatenate into exactly the full block's stream.
 *
 * Asynchronous on the scanner's stream: results become available through
 * yr_amd_scan_device_result after the stream is synchronised.
 * Requirements: d_data 16-byte aligned, byte_begin % 16 == 0.
 */
int yr_amd_scan_device(
    yr_amd_scanner* scanner,
    const uint8_t* d_data,
    uint64_t block_size,
    uint64_t byte_begin,
    uint64_t byte_end);

/*
 * The same scan when the device holds only a WINDOW of the block: d_window
 * holds bytes [window_begin, window_end) of a block of block_size bytes
 * (multi-GPU shards, SURVEY.md section 8e: each GPU owns a byte range and
 * holds it plus a halo).  Scans [byte_begin, byte_end) and reads only
 * [byte_begin - min(4, byte_begin), byte_end), which must lie in the window.
 * Positions, offsets and data_base semantics are those of the whole block, so
 * the candidate stream (and yr_amd_verify_device's records, when the window
 * includes yr_amd_tables_info's verify halos) equal the whole block's restricted
 * to (byte_begin, byte_end].
 * Requirements: d_window 16-byte aligned, window_begin and byte_begin
 * multiples of 16.  yr_amd_scan_device(s, d, n, b, e) is
 * yr_amd_scan_window(s, d, 0, n, n, b, e).
 */
int yr_amd_scan_window(
    yr_amd_scanner* scanner,
    const uint8_t* d_window,
    uint64_t window_begin,
    uint64_t window_end,
    uint64_t block_size,
    uint64_t byte_begin,
    uint64_t byte_end);

/*
 * Result of the last yr_amd_scan_device: synchronises the stream, retries
 * once with exact output capacity if a segment overflowed, and returns a
 * DEVICE pointer to the ascending candidate positions (uint64) and the count.
 */
int yr_amd_scan_device_result(
    yr_amd_scanner* scanner,
    const uint64_t** d_positions,
    uint64_t* count,
    int* all_positions);

/*
 * Verified-only scans (enable = 1): the scans of this scanner serve
 * yr_amd_verify_device only -- the paths that hand libyara records
 * (yr_amd_scan_block_verified, the block pipeline and the multi-device calls
 * set it on their own scanners).  For rule sets with 1-byte keys whose calls
 * the scan can decide from the bytes next to the key (candidate classes), the
 * scan kernel itself decides them and leaves the candidates none of whose
 * calls can have an effect out of the result: yr_amd_scan_device_result then
 * returns that reduced stream, while the records of yr_amd_verify_device are
 * unchanged -- the same calls, and the candidate field still indexes the FULL
 * stream (yr_amd_scan_device_stream_length).  yr_amd_scan_device_result of
 * a verified-only scan returns as soon as the counts are known, before the
 * compaction has written the positions: they are complete in the scanner's
 * stream order (yr_amd_verify_device queues behind them), and a reader on
 * another stream or on the host must synchronise that stream first.  No
 * effect on other rule sets or with yr_amd_tables_set_profiling.  Default 0.
 */
int yr_amd_scanner_set_verified_only(yr_amd_scanner* scanner, int enable);

/*
 * Length of the full candidate stream of the last completed scan (after
 * yr_amd_scan_device_result): its count, plus the candidates a verified-only
 * scan left out.
 */
int yr_amd_scan_device_stream_length(yr_amd_scanner* scanner, uint64_t* length);

/*
 * Verification callback: the arguments the reference passes to
 * yr_scan_verify_match(scanner, &rules->ac_match_pool[pool_index], data,
 * size, base, offset) (scanner.c:111-117).  A non-zero return aborts the
 * replay and is returned by yr_amd_replay (GOTO_EXIT_ON_ERROR semantics).
 */
typedef int (*yr_amd_verify_fn)(void* user, uint32_t pool_index, uint64_t offset);

/*
 * Replay a candidate stream in the reference order.  For every candidate i
 * (or every i in [0, size] when all_positions), the AC state is recomputed on
 * the host from position max(0, i - YR_AMD_MAX_ATOM_LENGTH) (exact: the trie
 * is at most that deep), and its match list is walked as scanner.c:105-121
 * does.  Candidates whose state has no match list are a protocol error
 * (YR_AMD_INTERNAL_FATAL_ERROR).
 */
int yr_amd_replay(
    const yr_amd_tables* tables,
    const uint8_t* data,
    size_t size,
    const uint64_t* positions,
    uint64_t count,
    int all_positions,
    yr_amd_verify_fn verify,
    void* user);

/*
 * ---- Device trace of the walk (tracing) ----
 *
 * The analogue of the reference walk's YR_DEBUG_VERBOSITY == 2 trace
 * (libyara/scanner.c:83-96), computed on the GPU: one row per block position
 * i in [0, size] whose walk state (after bytes [0, i)) is not the root,
 * ascending, with the state's slot and match_table[state].  The state is
 * walked with the reference's own transition rule over the untouched
 * transition table (scanner.c:123-141), independently of the scan kernel's
 * filter path, so the rows with match != 0 are exactly the candidate stream
 * of yr_amd_scan_device over the same block (the reference prints the rows
 * i < size; the row i == size is its final check, scanner.c:145-160).
 * d_data: DEVICE pointer to the block.  Writes min(total, cap) rows into the
 * host array out (may be NULL when cap == 0); *count = total.  With
 * YR_DEBUG_VERBOSITY >= 2 in the environment every row is also printed to
 * stderr in the reference's format.  Meant for small blocks (debugging).
 */
typedef struct
{
  uint64_t position;
  uint32_t state;
  uint32_t match;  /* match_table[state]: 1-based match-list head, 0 = none */
} yr_amd_trace_rec;

int yr_amd_trace_walk(
    yr_amd_scanner* scanner,
    const uint8_t* d_data,
    size_t size,
    uint64_t data_base,
    yr_amd_trace_rec* out,
    uint64_t cap,
    uint64_t* count);

/*
 * ---- On-device literal pre-verification ----
 *
 * The string records of the rules (YR_STRING, libyara/include/yara/types.h),
 * indexed like rules->strings_table, for the on-device evaluation of
 * _yr_scan_verify_literal_match (scan.c:887-990).
 */
typedef struct
{
  uint32_t flags;          /* YR_STRING.flags (STRING_FLAGS_* values, types.h:66-88) */
  uint32_t length;         /* YR_STRING.length */
  int64_t fixed_offset;    /* YR_STRING.fixed_offset */
  uint64_t bytes_offset;   /* where YR_STRING.string starts in the byte blob */
} yr_amd_string;

/*
 * Attach the string records to the tables (once, before any scanner verifies
 * on them).  pool_string[k] = index (into strings) of
 * rules->ac_match_pool[k].string; n_pool must equal the tables' pool size.
 * lowercase = the host's yr_lowercase[256] table (libyara.c:258), so nocase
 * comparisons use exactly the host's case folding.
 */
int yr_amd_tables_set_strings(
    yr_amd_tables* tables,
    const uint32_t* pool_string,
    uint32_t n_pool,
    const yr_amd_string* strings,
    uint32_t n_strings,
    const uint8_t* bytes,
    uint64_t n_bytes,
    const uint8_t* lowercase);

/*
 * Attach the regexp programs so that calls on
 * hex strings (STRING_FLAGS_FAST_REGEXP) and other regexp strings are
 * pre-verified too.  For
 * pool entry k, forward code = code[fwd_off[k] .. + fwd_len[k]) (a copy of
 * rules->ac_match_pool[k].forward_code up to and including RE_OPCODE_MATCH),
 * backward code likewise (bwd_len[k] = 0: backward_code == NULL);
 * fwd_len[k] = 0: no program (the call is always kept).  For FAST_REGEXP
 * strings the program must be linear in the opcodes yr_re_fast_exec executes
 * (re.c:2150-2391): ANY, LITERAL, NOT_LITERAL, MASKED_LITERAL,
 * MASKED_NOT_LITERAL, REPEAT_ANY_UNGREEDY, MATCH; for other regexp strings any
 * well-formed yr_re_exec program (re.c:1693) whose reachable instructions span
 * exactly the given length (yr_amd_re_code_extent).  YR_AMD_INVALID_ARGUMENT
 * otherwise.  Requires yr_amd_tables_set_strings first.
 */
int yr_amd_tables_set_re_code(
    yr_amd_tables* tables,
    uint32_t n_pool,
    const uint32_t* fwd_off,
    const uint32_t* fwd_len,
    const uint32_t* bwd_off,
    const uint32_t* bwd_len,
    const uint8_t* code,
    uint64_t code_len);

/*
 * Extent of a regexp program starting at `code` with `avail` readable bytes:
 * the end of the furthest instruction reachable from its start through jumps,
 * splits and repeat offsets (re.h:65-92 opcodes).  YR_AMD_INVALID_ARGUMENT if
 * an unknown opcode or an out-of-range target is reachable.  Used to copy
 * YR_AC_MATCH.forward_code / backward_code for yr_amd_tables_set_re_code.
 */
int yr_amd_re_code_extent(const uint8_t* code, uint64_t avail, uint32_t* extent);

/*
 * One call of the replay that can have an effect: the host calls
 * yr_scan_verify_match(scanner, &rules->ac_match_pool[pool_index], data,
 * size, base, offset).  candidate = index of the candidate position in the
 * scan's stream that produced it.
 */
typedef struct
{
  uint64_t offset;
  uint32_t pool_index;
  uint32_t candidate;
} yr_amd_verify_rec;

/*
 * Pre-verify the candidate stream of the last completed scan of this scanner
 * (yr_amd_scan_device + yr_amd_scan_device_result, on the same block) on the
 * GPU.  Produces, in the exact order yr_amd_replay would make them, the calls
 * of the reference loop (scanner.c:105-121) minus those that provably return
 * without effect: a literal string whose comparison fails
 * (_yr_scan_verify_literal_match returns before _yr_scan_match_callback,
 * scan.c:974-975) or whose FULL_WORD match touches an alphanumeric character
 * (_yr_scan_match_callback, scan.c:672-694), a FIXED_OFFSET string at another
 * offset (scan.c:1023), offset == size (scan.c:1013), and -- with
 * yr_amd_tables_set_re_code -- a regexp string whose program provably cannot
 * match from the call's offset (_yr_scan_verify_re_match, scan.c:778-880):
 * hex strings' fast-exec programs (yr_re_fast_exec, re.c:2150-2391) in the
 * reference's position-set form; other regexps' yr_re_exec programs
 * (re.c:1693-2072) by an exact search over every opcode's semantics (keeping
 * a call where the reference's SPLIT fiber-kill rule, re.c:1482-1495, might
 * end the only path) with a 1000-step budget below RE_MAX_FIBERS, so calls
 * that could fail with ERROR_TOO_MANY_RE_FIBERS are always kept.  Base64
 * strings are always kept.  Kept calls are verified by re.c / scan.c on the
 * host.  data_base = YR_MEMORY_BLOCK.base.  After yr_amd_scan_window, a call
 * whose bytes are not all in the window is kept (never decided on missing
 * bytes).
 * On success *d_records is a DEVICE pointer owned by the scanner (valid until
 * its next verify) to *count records.  Synchronous.  The record's candidate
 * field is a 32-bit index: a candidate stream longer than
 * YR_AMD_VERIFY_MAX_CANDIDATES returns YR_AMD_INVALID_ARGUMENT.  A block (or a
 * window's byte range) of size bytes has at most size + 1 candidates, so any
 * block below 4 GiB is accepted; callers route larger ones to yr_amd_replay
 * when size + 1 exceeds the limit (integration/yr_gpu_scanner.c).
 * Requires yr_amd_tables_set_strings; YR_AMD_INVALID_ARGUMENT otherwise.
 */
#define YR_AMD_VERIFY_MAX_CANDIDATES 0x100000000ull
int yr_amd_verify_device(
    yr_amd_scanner* scanner,
    uint64_t data_base,
    const yr_amd_verify_rec** d_records,
    uint64_t* count);

/*
 * Host-block convenience: H2D, scan, pre-verify, D2H.  *records points to
 * *count host records owned by the scanner (valid until its next call).
 * Replaying them in order into yr_scan_verify_match yields the same scan
 * state as replaying the full candidate stream with yr_amd_replay.
 */
int yr_amd_scan_block_verified(
    yr_amd_scanner* scanner,
    const uint8_t* data,
    size_t size,
    uint64_t data_base,
    const yr_amd_verify_rec** records,
    uint64_t* count);

/*
 * ---- Block pipeline ----
 *
 * The block driver of libyara (yr_scanner_scan_mem_blocks, scanner.c:417-583;
 * files via filemap.c, processes via proc/linux.c) scans one
 * YR_MEMORY_BLOCK at a time.  A pipeline keeps up to `depth` blocks in flight
 * (each: copy to a pinned buffer, H2D, scan, on-device pre-verification on
 * its own HIP stream and worker thread) while the caller replays the oldest
 * one, so end-to-end scans of many blocks overlap PCIe, GPU and host replay.
 * Requires yr_amd_tables_set_strings.  One pipeline per YR_SCANNER.
 */
typedef struct yr_amd_pipeline yr_amd_pipeline;

/* depth: blocks in flight, 1..8 (2 double-buffers). */
int yr_amd_pipeline_create(yr_amd_tables* tables, uint32_t depth, yr_amd_pipeline** pipeline);

/* Waits for the workers to finish, frees everything. */
int yr_amd_pipeline_destroy(yr_amd_pipeline* pipeline);

/*
 * Copy a block (the caller's buffer may be reused on return; the copy runs in
 * the calling thread, so a fault on an mmap'ed block surfaces in the caller,
 * inside its YR_TRYCATCH) and start its GPU work.  At most `depth` blocks may
 * be in flight: YR_AMD_INVALID_ARGUMENT otherwise (call yr_amd_pipeline_next).
 * base = YR_MEMORY_BLOCK.base.
 */
int yr_amd_pipeline_submit(
    yr_amd_pipeline* pipeline,
    const uint8_t* data,
    size_t size,
    uint64_t base);

/*
 * The same at link rate: the block is copied into the slot's pinned host
 * buffer by several threads at once (the caller's and a small pool; the
 * buffer may be reused on return) and moved to the device by plain DMA, with
 * no second host pass in the runtime's pageable staging.  The pinned copy is
 * what yr_amd_pipeline_next hands back for the replay.  Every page of the
 * block must be readable: a fault in a helper thread cannot unwind through
 * the caller's YR_TRYCATCH, so a libyara caller first touches each page
 * inside it (integration/yr_gpu_scanner.c).
 */
int yr_amd_pipeline_submit_dma(
    yr_amd_pipeline* pipeline,
    const uint8_t* data,
    size_t size,
    uint64_t base);

/*
 * Wait for the oldest submitted block.  Returns its scan status; on success
 * *records / *count are its effective verify calls (yr_amd_scan_block_verified
 * semantics) and *data / *size / *base its pipeline-owned bytes, all valid
 * until the next yr_amd_pipeline_next / _drain / _destroy.  Blocks come back
 * in submission order.
 */
int yr_amd_pipeline_next(
    yr_amd_pipeline* pipeline,
    const yr_amd_verify_rec** records,
    uint64_t* count,
    const uint8_t** data,
    size_t* size,
    uint64_t* base);

/* Wait for and discard every block in flight (error paths). */
int yr_amd_pipeline_drain(yr_amd_pipeline* pipeline);

/*
 * The copy that moves a caller's block into pipeline / multi-device staging
 * memory: copy n bytes from src to dst, return 0, or nonzero if the source
 * could not be read.  It may run on the caller's thread and on the library's
 * helper threads, several at once on disjoint pieces.  A libyara caller passes
 * one that runs memcpy inside YR_TRYCATCH (exception.h:150-185) on the thread
 * that calls it, so a block that faults while being copied (a file mapping
 * truncated underneath) fails the submission with YR_AMD_COULD_NOT_MAP_FILE
 * -- scanner.c:493-496's mapping of the walk's fault -- instead of raising
 * SIGBUS on a thread with no handler.  Default (NULL): memcpy, and every page
 * of a block must be readable.
 */
typedef int (*yr_amd_copy_fn)(void* user, void* dst, const void* src, size_t n);
int yr_amd_pipeline_set_copy(yr_amd_pipeline* pipeline, yr_amd_copy_fn fn, void* user);

/*
 * A pipeline whose blocks are split across n devices:
 * tables[k] as for yr_amd_multi_create.  Each block is copied once into a
 * pinned buffer (yr_amd_pipeline_submit_dma: in parallel; _submit: in the
 * caller's thread), every device DMAs its window of it (its byte range plus
 * the verify halos, yr_amd_multi_shard's bounds) and scans and pre-verifies it;
 * yr_amd_pipeline_next returns the devices' records concatenated in order --
 * exactly the single-device record stream of the block.  Blocks overlap as in
 * the single-device pipeline (block k+1's copy and DMA while block k is
 * scanned or replayed).  n = 1 is yr_amd_pipeline_create.  A block whose
 * device ranges could exceed YR_AMD_VERIFY_MAX_CANDIDATES candidates fails
 * in yr_amd_pipeline_next with YR_AMD_INVALID_ARGUMENT (callers route such
 * blocks to the host replay first, as integration/yr_gpu_scanner.c does).
 */
int yr_amd_pipeline_create_multi(yr_amd_tables* const* tables, uint32_t n, uint32_t depth,
                                 yr_amd_pipeline** pipeline);

/* Blocks smaller than `bytes` are not split: each goes whole to one device,
 * round-robin (default 0: every block is split). */
int yr_amd_pipeline_set_split_min(yr_amd_pipeline* pipeline, uint64_t bytes);

/*
 * ---- Multi-device block scans ----
 *
 * One process, n devices (n <= YR_AMD_MAX_DEVICES; a device may repeat: n
 * logical devices on fewer GPUs).  A block is split into n byte ranges, equal
 * 1 MiB-aligned slices with the last taking the rest (yara_amd/dist.py
 * shard_bounds); device k holds only its WINDOW of the block -- its range plus
 * the tables' verify halos (yr_amd_tables_info) -- scans it
 * (yr_amd_scan_window) and pre-verifies its own candidates
 * (yr_amd_verify_device), each device on its own stream and host thread.
 * Records are block-global: their concatenation in device order is exactly
 * yr_amd_scan_block_verified's on the whole block, candidate indices rebased
 * onto the whole block's stream.  The input buffers shard across the GPUs of
 * a node with no data-path exchange (the north star's 8-GPU layout inside one
 * libyara process; torch.distributed ranks use the same windows, dist.py).
 */
#define YR_AMD_MAX_DEVICES 64
typedef struct yr_amd_multi yr_amd_multi;

/* tables[k]: the same rule set built on device k (yr_amd_tables_create +
 * yr_amd_tables_set_strings [+ _set_re_code]), one per device; owned by the
 * caller and kept alive while the multi scanner exists.  One multi scanner per
 * thread (like yr_amd_scanner). */
int yr_amd_multi_create(yr_amd_tables* const* tables, uint32_t n, yr_amd_multi** multi);
int yr_amd_multi_destroy(yr_amd_multi* multi);

/* Device k's byte range [*begin, *end) of a block of `size` bytes and the
 * window [*window_begin, *window_end) it holds (any pointer may be NULL). */
int yr_amd_multi_shard(const yr_amd_multi* multi, uint64_t size, uint32_t k, uint64_t* begin,
                       uint64_t* end, uint64_t* window_begin, uint64_t* window_end);

/* yr_amd_scan_block_verified across the devices: *records / *count are host
 * records owned by the multi scanner (valid until its next call).  A device
 * whose range could exceed YR_AMD_VERIFY_MAX_CANDIDATES candidates (range + 1
 * > the limit) makes it return YR_AMD_INVALID_ARGUMENT before any work: use
 * the single-device replay (yr_amd_scan_block + yr_amd_replay) then.  The
 * block is staged through two pinned 256 MiB buffers (copied in parallel
 * through the copy function of yr_amd_multi_set_copy, DMA'd to every device
 * whose window overlaps them); a failed copy returns
 * YR_AMD_COULD_NOT_MAP_FILE. */
int yr_amd_multi_set_copy(yr_amd_multi* multi, yr_amd_copy_fn fn, void* user);
int yr_amd_multi_scan_block_verified(
    yr_amd_multi* multi,
    const uint8_t* data,
    size_t size,
    uint64_t data_base,
    const yr_amd_verify_rec** records,
    uint64_t* count);

/* The device a table set lives on (-1: host-only tables). */
int yr_amd_tables_device(const yr_amd_tables* tables);

/*
 * Profiling-counter parity (libyara built with YR_PROFILING_ENABLED).
 * yr_scan_verify_match counts profiling_info[rule].atom_matches for every
 * call that passes its early returns (scan.c:1013-1027, :1077-1083), whether or
 * not the string matches.  With profiling enabled on a table set,
 * pre-verification (yr_amd_verify_device and everything built on it) also
 * emits every dropped call past those returns as a COUNT-ONLY record: its
 * pool_index carries YR_AMD_REC_COUNT_ONLY, and the host counts it -- after
 * the same temp-disabled / fast-mode tests, which depend on host state at that
 * point of the call order -- without calling the verifier
 * (integration/yr_gpu_scanner.c).  Default off.
 */
#define YR_AMD_REC_COUNT_ONLY 0x80000000u
int yr_amd_tables_set_profiling(yr_amd_tables* tables, int enable);

/*
 * Kernel timing (measurement support): when enabled, the scanner records HIP
 * events around its scan kernel on its own stream; yr_amd_scanner_kernel_ms
 * returns the duration of the last scan kernel launch (after the scan result
 * was collected), yr_amd_scanner_scan_ms that of the scan and its compaction
 * into the position list (the candidate classes included).
 */
int yr_amd_scanner_set_timing(yr_amd_scanner* scanner, int enable);
int yr_amd_scanner_kernel_ms(yr_amd_scanner* scanner, float* ms);
int yr_amd_scanner_scan_ms(yr_amd_scanner* scanner, float* ms);

/*
 * Benchmark/test utility (not part of the libyara path): fill a device buffer
 * with bytes [offset, offset + n) of the canonical synthetic input of
 * SURVEY.md Appendix A (xorshift64, byte = (uint8_t)(x >> 24),
 * x0 = 0x9E3779B97F4A7C15 * seed), generated in parallel on the GPU with GF(2)
 * jump-ahead.  stream: hipStream_t or NULL.
 */
int yr_amd_fill_xorshift64(void* d_buf, uint64_t n, uint64_t seed, uint64_t offset, void* stream);

/* Library version string, e.g. "yara_amd 0.1.0 (gfx950)". */
const char* yr_amd_version(void);

#ifdef __cplusplus
}
#endif

#endif
