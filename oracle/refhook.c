/*
 * Verify-call probe for the REFERENCE build (test infrastructure only).
 *
 * libyara's hot loop (_yr_scanner_scan_mem_block, reference
 * libyara/scanner.c:45-176) is static, so its only observable output is the
 * sequence of calls it makes to yr_scan_verify_match (scanner.c:111, :153).
 * oracle/ref.mk compiles the reference scanner.c a second time with
 * -Dyr_scan_verify_match=yr_refhook_verify_match, so every such call lands here,
 * is recorded, and is then forwarded to the real, unmodified verifier
 * (reference libyara/scan.c:992).  The recorded (position, pool index) stream
 * is the golden the in-repo oracle and the HIP path must reproduce exactly.
 */
#include <yara.h>
#include <yara/scan.h>

typedef void (*yr_refhook_fn)(void* user, const YR_AC_MATCH* m, size_t offset);

yr_refhook_fn yr_refhook_cb = NULL;
void* yr_refhook_user = NULL;

int yr_refhook_verify_match(
    YR_SCAN_CONTEXT* context,
    YR_AC_MATCH* ac_match,
    const uint8_t* data,
    size_t data_size,
    uint64_t data_base,
    size_t offset)
{
  if (yr_refhook_cb != NULL)
    yr_refhook_cb(yr_refhook_user, ac_match, offset);
  return yr_scan_verify_match(
      context, ac_match, data, data_size, data_base, offset);
}
