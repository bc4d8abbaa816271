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

/* A CPU stand-in for edverify.h edv_verify_staged_part (test infrastructure only): the staged
 * scan's copier calls it for each part of a speculative batch.  It snapshots the part's key ids
 * and spans (what the library DMAs at that moment) into the caller's part_double_t, checks that
 * the parts come in order and 64-aligned, and can be told to fail at its k-th call. */
typedef struct {
  uint32_t *keys;   /* n snapshots */
  uint64_t *spans;  /* starts[n] then ends[n] snapshots */
  uint64_t n, covered, calls, fail_at, bad, slot_off;
} part_double_t;

int stage_double_part(void *ctx, const void *keys, uint64_t slot_off, uint64_t msg_base, const uint64_t *spans,
                      uint64_t n, uint64_t lo, uint64_t hi) {
  part_double_t *c = (part_double_t *)ctx;
  (void)msg_base;
  c->calls++;
  c->slot_off = slot_off;
  if (!c || n != c->n || lo > hi || hi > n || (lo & 63) || lo != c->covered) {
    c->bad++;
    return -1;
  }
  if (c->fail_at && c->calls == c->fail_at) return -2;
  memcpy(c->keys + lo, (const uint32_t *)keys + lo, 4 * (hi - lo));
  memcpy(c->spans + lo, spans + lo, 8 * (hi - lo));
  memcpy(c->spans + n + lo, spans + n + lo, 8 * (hi - lo));
  c->covered = hi;
  return 0;
}
