/* Test infrastructure only: a CPU stand-in for edverify.h edv_stage_put, so the
 * native scan's staged mode (hostpack.cpp, defer = 2) can be exercised without a
 * GPU.  ctx is the address of a host "staging" buffer; the put is a memcpy (the
 * scan's workers call it concurrently on disjoint ranges). */
#include <stdint.h>
#include <string.h>

int stage_double_put(void *ctx, const void *src, uint64_t nbytes, uint64_t off) {
  if (!ctx || (nbytes && !src)) return -1;
  memcpy((char *)ctx + off, src, nbytes);
  return 0;
}
