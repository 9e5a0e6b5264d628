/*
 * yr_gpu_scanner.h -- libyara-side integration of the MI355X atom scanner
 * (see yr_gpu_scanner.c and INTEGRATION.md).  Include after <yara.h>.
 */
#ifndef YR_GPU_SCANNER_H
#define YR_GPU_SCANNER_H

#include <yara.h>

#include "../include/yara_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct YR_GPU_RULES YR_GPU_RULES;     /* device tables of one YR_RULES */
typedef struct YR_GPU_SCANNER YR_GPU_SCANNER; /* one per YR_SCANNER / thread */

int yr_gpu_rules_create(YR_RULES* rules, int device, YR_GPU_RULES** out);

/* Device tables on n_devices devices (a device may repeat).  Scanners of these
 * rules split every block of at least YR_GPU_MULTI_MIN_BLOCK bytes (see
 * yr_gpu_scanner_set_multi_min_block) across the devices: each holds only its
 * shard of the block plus the rule set's verify halos, scans and pre-verifies
 * it (yr_amd_multi_*), and the records are replayed in block order -- the
 * same match set as one device.  Smaller blocks run on devices[0]. */
#define YR_GPU_MULTI_MIN_BLOCK (256ull << 20)
int yr_gpu_rules_create_multi(
    YR_RULES* rules,
    const int* devices,
    int n_devices,
    YR_GPU_RULES** out);
void yr_gpu_rules_destroy(YR_GPU_RULES* g);
int yr_gpu_scanner_create(YR_GPU_RULES* g, YR_GPU_SCANNER** out);
void yr_gpu_scanner_destroy(YR_GPU_SCANNER* s);

/* On-device literal pre-verification + block pipeline (default on): blocks
 * are copied, scanned and pre-verified two at a time on the GPU while the
 * host replays the previous one, and only the verify calls that can have an
 * effect reach yr_scan_verify_match.  Off: one block at a time, every call of
 * the reference loop replayed (yr_amd_scan_block + yr_amd_replay). */
void yr_gpu_scanner_set_preverify(YR_GPU_SCANNER* s, int enable);

/* Smallest block the multi-device path takes (rules from
 * yr_gpu_rules_create_multi; default YR_GPU_MULTI_MIN_BLOCK). */
void yr_gpu_scanner_set_multi_min_block(YR_GPU_SCANNER* s, uint64_t bytes);
/* How many blocks this scanner has split across its devices. */
uint64_t yr_gpu_scanner_multi_blocks(const YR_GPU_SCANNER* s);

/* Where a GPU scan's wall time goes (seconds, cumulative over the scanner's
 * scans; measurement support -- tools/e2e_rate.sh): t[0] host copy of blocks
 * into the pipeline's pinned staging, t[1] waiting for the GPU (H2D, scan,
 * on-device pre-verification and the records' D2H of blocks not yet done when
 * their replay is due, and the whole of the direct single-block path), t[2]
 * the host replay of the records into yr_scan_verify_match (scan.c / re.c). */
void yr_gpu_scanner_timing(const YR_GPU_SCANNER* s, double t[3]);

/* Drop-in counterparts of yr_scanner_scan_mem_blocks / yr_scanner_scan_mem
 * (scanner.c:417, :633): same arguments, callbacks, flags and error codes. */
int yr_gpu_scanner_scan_mem_blocks(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    YR_MEMORY_BLOCK_ITERATOR* iterator);
int yr_gpu_scanner_scan_mem(
    YR_SCANNER* scanner,
    YR_GPU_SCANNER* gs,
    const uint8_t* buffer,
    size_t buffer_size);

#ifdef YR_HAVE_BLOCK_SCANNER
/* libyara patched with integration/libyara-block-scanner.patch: make the
 * scanner's own driver (yr_scanner_scan_mem / _mem_blocks / _file / _fd /
 * _proc, yr_rules_* above them) use the GPU for every block.  gs must be
 * created on the scanner's rules; one gs per scanner. */
int yr_gpu_scanner_attach(YR_SCANNER* scanner, YR_GPU_SCANNER* gs);
#endif

/* ... and of yr_scanner_scan_file / _fd / _proc (scanner.c:674-722). */
int yr_gpu_scanner_scan_file(YR_SCANNER* scanner, YR_GPU_SCANNER* gs, const char* filename);
int yr_gpu_scanner_scan_fd(YR_SCANNER* scanner, YR_GPU_SCANNER* gs, YR_FILE_DESCRIPTOR fd);
int yr_gpu_scanner_scan_proc(YR_SCANNER* scanner, YR_GPU_SCANNER* gs, int pid);

#ifdef __cplusplus
}
#endif

#endif
