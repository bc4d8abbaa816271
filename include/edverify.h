/*
 * edverify.h -- C ABI of libplenum_edverify.so, the MI355X (gfx950) batched
 * Ed25519 request-signature engine behind Plenum's client authenticator.
 *
 * What it replaces (reference interfaces, /root/reference):
 *   stp_core/crypto/nacl_wrappers.py:232-242  Verifier.verify(signature, msg) -> bool
 *   stp_core/crypto/nacl_wrappers.py:100-108  VerifyKey.verify(sig + msg) ->
 *                                             libnacl.crypto_sign_open(sm, pk)
 *   (libsodium 1.0.18 crypto_sign_open / crypto_sign_verify_detached:
 *    int crypto_sign_verify_detached(const unsigned char *sig,
 *        const unsigned char *m, unsigned long long mlen, const unsigned char *pk);
 *    0 = accept, -1 = reject)
 *   called once per request from NaclAuthNr.authenticate
 *   (plenum/server/client_authn.py:99-102); here one call covers a batch.
 *
 *   plenum/server/quorums.py:15-32 + plenum/server/models.py:21-37
 *   (Quorums thresholds, TrackedMsgs distinct-voter sets) -> edv_tally_*.
 *
 * Conventions
 *   - Every function returns 0 on success or a negative EDV_E* code; the
 *     message for the last failure on the calling thread is edv_last_error().
 *     No C++ exception crosses this boundary.  A call either completes or
 *     fails as a whole (no partial results).
 *   - Host-pointer entry points (no _device suffix): the caller owns its
 *     buffers; the library stages them through its own device buffers and
 *     returns when the result is in the caller's buffer.
 *   - _device entry points take device pointers and an optional hipStream_t
 *     (NULL = the context's stream, a blocking stream ordered after work on
 *     the legacy NULL stream) and are asynchronous.
 *   - Bitmasks: bit i of the mask is bit (i % 8) of byte (i / 8), i.e.
 *     little-endian 64-bit words of wave ballots.  1 = libsodium returns 0.
 *   - Threading: one context per GPU; calls on one context are serialised by
 *     the caller (Plenum's node is single-threaded asyncio).
 *
 * Stability.  STABLE: the drop-in's contract, what plenum_amd's authenticator
 * binds -- context, verify (host-pointer, keyed, one-request, staged, submit /
 * collect), the key store, pinned host memory, request digests, the tally and
 * BLS.  Every tuning knob is one edv_options struct read and written whole
 * (edv_set_options checks every field before applying any; the authenticator
 * never changes them); measurements are one edv_stats struct.  DIAGNOSTIC
 * (benches and tests, not the drop-in): edv_get_stats, the *_device forms,
 * the synthetic-load signer (edv_seed_keypair_batch, edv_sign_*), and
 * edv_bls_sign_batch / edv_bls_keygen_batch.  tests/test_abi.py fails on any
 * exported edv_* symbol this header does not declare.
 */
#ifndef PLENUM_EDVERIFY_H
#define PLENUM_EDVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EDV_OK 0
#define EDV_EINVAL -1   /* bad argument (NULL pointer, n too large, ...) */
#define EDV_EHIP -2     /* HIP runtime error (message has the hipError string) */
#define EDV_ENOMEM -3   /* device or host allocation failed */
#define EDV_ENODEV -4   /* no gfx950 device / device index out of range */
#define EDV_EBUSY -5    /* the staging set holds an uncollected submission (collect it, or use the other set) */

typedef struct edv_ctx edv_ctx;

/* Library/version info. */
const char *edv_version(void);
/* Window of the base-point comb table built by edv_create (rows =
 * ceil(254 / w) mixed additions per [S]B): the bench's roofline prices the
 * comb kernel's work from it. */
int edv_base_window(void);
const char *edv_last_error(void);
int edv_device_count(void);

/* Create a context bound to HIP device `device` (one stream, lazily grown
 * device staging buffers).  Returns NULL on failure (see edv_last_error()). */
edv_ctx *edv_create(int device);
void edv_destroy(edv_ctx *ctx);
/* Block until all work queued on the context stream has finished. */
int edv_synchronize(edv_ctx *ctx);

/* ------------------------------------------------------------ options (STABLE)
 * Every tuning knob of a context.  edv_default_options fills what a fresh
 * context has; edv_set_options validates every field before applying any (a
 * refused call changes nothing). */
typedef struct edv_options {
  /* sub-batches per 2^20-request chunk, 1..4 (default 1: each kernel alone on the GPU; 2-4 alternate
   * two streams so a sub-batch's encode overlaps the next one's hash -- within 1 % at 1M) */
  int32_t pipeline;
  /* hash lanes in SHA-512 block-count order (a stable descending radix sort of the block counts, one
   * 6-bit rocPRIM pass, ~50 us per 1M): 0 off, 1 on, 2 auto (default: host-offset calls sort when
   * unsorted waves would run > 1.25x the batch's blocks; device-pointer calls cannot see the lengths
   * and treat auto as off), 3 sorted + packed (north_star (1): each 64-lane group's messages written
   * as padded big-endian SHA-512 stream words, lane-interleaved, into the unit arena; groups that do
   * not fit are read in place).  configs[3]: hash 4.72 -> 1.50 ms per 1M with sorting. */
  int32_t length_buckets;
  /* key order of the comb on the key-table path: 0 off, 1 on, 2 auto (default: sub-batches of 4,096+
   * requests at key windows >= 15 with < 16,384 keys).  A counting sort makes one key's requests
   * neighbours, so a wave gathers from one key's rows (W = 16, random key order: comb 1.70 -> 1.02 ms
   * per 1M); the accept bits do not change. */
  int32_t key_sort;
  /* edv_verify_one's resident kernel: 1 on (default; 0 when EDV_RESIDENT=0 at edv_create), 0 off
   * (every single request launches edv_verify_small_kernel) */
  int32_t resident;
  /* keyed host-pointer batches of at most this many requests run one workgroup of three waves per
   * request (hash | base comb rows | R decode side by side) for latency (default 256, at most 65536;
   * 0 = never) */
  uint64_t small_batch;
  /* the unit arena of length_buckets = 3, in bytes (default 1.25 GiB = 1,280 B per lane of a chunk) */
  uint64_t unit_arena_bytes;
  /* BLS: verify batches of at most this many checks take two lanes per check (each Miller loop on
   * its own lane), of at most half of it four lanes (default 32768; 0 = always one lane) */
  uint64_t bls_pair_lanes;
  /* BLS: verify batches of at most this many checks run one wave per check (the check as a
   * straight-line program over the wave's lanes, bls_program.h: ~3 ms for a COMMIT round's ~25;
   * checks it cannot decide re-run on the four-lane kernel) (default 8192; 0 = never) */
  uint64_t bls_wave_checks;
} edv_options;
void edv_default_options(edv_options *out);
int edv_get_options(edv_ctx *ctx, edv_options *out);
int edv_set_options(edv_ctx *ctx, const edv_options *opt);

/* ------------------------------------------------------- statistics (DIAGNOSTIC)
 * The roofline's kernel times and the last host-pointer call, in one read.
 * The verify pipeline is four kernels: hash (prechecks + SHA-512 + mod L),
 * table (decode -A, [1..8](-A); empty on the key-table path), dsm or comb
 * ([h](-A) + [S]B), encode (batched inversion, encode, compare with R,
 * ballot); a call over more than 2^20 requests runs in chunks and the phase
 * times cover the last one.  Waits for the last timed launch's events. */
typedef struct edv_stats {
  double phase_ms[4];        /* hash, table, dsm/comb, encode: per phase the SUM over the last chunk's
                                sub-batch launches, HIP events on the launch streams (a small-kernel
                                launch counts as the comb phase) */
  int32_t launch_count;      /* sub-batches (launches per phase) of that chunk */
  int32_t phases_valid;      /* 1 once a timed verify has run on the context */
  uint64_t chunk_items;      /* requests in that chunk */
  double host_call_ms;       /* the last host-pointer verify: wall time of the call */
  double host_stage_ms;      /*   CPU copies into pinned staging (0 when every input was pinned) */
  uint64_t host_h2d_bytes;   /*   bytes copied host -> device */
  uint32_t host_direct;      /*   inputs DMA'd straight from pinned memory: bit 0 signatures, 1 keys,
                                  2 messages, 3 offsets */
  uint32_t reserved;
  uint64_t resident_launches; /* edv_verify_one: resident kernels launched, requests they served */
  uint64_t resident_served;
  double resident_service_us;  /* the last request's time in the resident kernel, from seeing it to its
                                  verdict (100 MHz wall clock); the engine call's rest is PCIe and host */
} edv_stats;
int edv_get_stats(edv_ctx *ctx, edv_stats *out);

/* ---------------------------------------------------------------- verify */

/* libsodium crypto_sign_verify_detached over a batch.
 *   sig64   : n * 64 bytes (R || S per item)
 *   pk32    : n * 32 bytes
 *   msgs    : concatenated messages; item i is msgs[msg_off[i] .. msg_off[i+1])
 *   msg_off : n + 1 offsets (msg_off[0] need not be 0)
 *   accept_bits : (n + 7) / 8 bytes out.
 * Replaces n calls of Verifier.verify (nacl_wrappers.py:232-242). */
int edv_verify_batch(edv_ctx *ctx, const uint8_t *sig64, const uint8_t *pk32, const uint8_t *msgs,
                     const uint64_t *msg_off, uint64_t n, uint8_t *accept_bits);

/* libsodium crypto_sign_open semantics over a batch of signed messages
 * sm_i = sm[sm_off[i] .. sm_off[i+1]): len < 64 -> reject, otherwise split
 * at byte 64 (signature || message).  This is exactly what
 * VerifyKey.verify(signature + msg) does (nacl_wrappers.py:100-108), so a
 * base58-decoded signature of any length keeps the reference's behaviour. */
int edv_sign_open_batch(edv_ctx *ctx, const uint8_t *sm, const uint64_t *sm_off, const uint8_t *pk32, uint64_t n,
                        uint8_t *accept_bits);

/* Device-resident verify (inputs already in HBM).  d_accept_words receives
 * ceil(n / 64) little-endian uint64 words.  d_msgs must be readable up to the
 * 4-byte-aligned word containing its last message byte. */
int edv_verify_batch_device(edv_ctx *ctx, const void *d_sig64, const void *d_pk32, const void *d_msgs,
                            const void *d_msg_off, uint64_t n, void *d_accept_words, void *stream);


/* ------------------------------------------------------ key-table path */

/* Register public keys (the verkeys SimpleAuthNr.addIdr holds,
 * plenum/server/client_authn.py:133-140).  For each key the library decodes
 * -A once, records libsodium's key checks (canonical y, not small order, on
 * the curve) and builds the fixed-base comb table (j+1) * 2^(W*i) * (-A),
 * i < ceil(253/W), j < 2^(W-1), as affine niels points in HBM.  The key
 * window W trades HBM for additions per verify:
 *   W = 4:  64 KiB per key, 64 additions  (1M keys =  64 GiB)
 *   W = 6: 172 KiB per key, 43 additions  (1M keys = 172 GiB)
 *   W = 8: 512 KiB per key, 32 additions  (500k keys = 256 GiB)
 *   W = 10: 1.6 MiB per key, 26 additions (context default)
 *   W = 12 / 13 / 14 / 16: 5.5 / 10 / 19 / 64 MiB per key, 22 / 20 / 19 / 16
 *   additions (bench.py headline: 14, 1,000 keys = 19 GiB)
 * Tables are stored row-major over keys (row r of every key in one slab), so
 * lanes verifying different keys gather from one slab at a time.
 * Key ids are consecutive from *first_id.  Host / device-pointer forms. */
int edv_keys_add(edv_ctx *ctx, const uint8_t *pk32, uint64_t nkeys, uint64_t *first_id);
int edv_keys_add_device(edv_ctx *ctx, const void *d_pk32, uint64_t nkeys, uint64_t *first_id, void *stream);
/* Re-register slots [first_id, first_id + nkeys) with new keys (all < the
 * registered count): the caller's LRU eviction.  Waits for in-flight work on
 * the device first, so no verify reads a half-rebuilt table. */
int edv_keys_set(edv_ctx *ctx, uint64_t first_id, const uint8_t *pk32, uint64_t nkeys);
/* Asynchronous forms, for registrations made on the request path (a key that
 * earned a slot by use, an addIdr key): the pk upload and the table builds
 * are queued on the context's build stream and the call returns at once with
 * a ticket (tickets complete in order).  The ids are assigned immediately,
 * but a keyed verify of an id whose build has not finished reads a
 * half-built table: the caller routes those requests to the general path
 * (edv_verify_batch / edv_sign_open_batch, same verdicts) until
 * edv_keys_ready(ticket) returns 1.  edv_keys_set_async's rebuild starts
 * after the work already queued on the context's own streams (a verify still
 * reading the old table); the host never waits for it.  Replaces the
 * synchronous registration inside plenum/server/client_authn.py:133-140's
 * addIdr path (SimpleAuthNr keeps its dict; the tables are this library's). */
int edv_keys_add_async(edv_ctx *ctx, const uint8_t *pk32, uint64_t nkeys, uint64_t *first_id, uint64_t *ticket);
int edv_keys_set_async(edv_ctx *ctx, uint64_t first_id, const uint8_t *pk32, uint64_t nkeys, uint64_t *ticket);
/* edv_keys_set_async for scattered slots: key ids[k] (distinct, registered) becomes pk32[k], all
 * nkeys in one upload (through the library's pinned staging: the host returns without waiting for
 * the builds already queued) and one build launch -- the key store's evictions of a batch. */
int edv_keys_set_many_async(edv_ctx *ctx, const uint32_t *ids, const uint8_t *pk32, uint64_t nkeys,
                            uint64_t *ticket);
/* 1 when every build up to `ticket` has finished, 0 while one still runs, < 0 on error. */
int edv_keys_ready(edv_ctx *ctx, uint64_t ticket);
/* Wait for every queued build. */
int edv_keys_sync(edv_ctx *ctx);
uint64_t edv_keys_count(edv_ctx *ctx);
/* Forget all registered keys (device memory is kept for reuse; waits for queued builds). */
int edv_keys_reset(edv_ctx *ctx);
/* Set the key window (4, 6, 8, 10, 12, 13, 14 or 16; environment EDV_KEY_WINDOW sets the
 * context default).  Only with no keys registered; frees the key store. */
int edv_keys_set_window(edv_ctx *ctx, int w);
int edv_keys_window(edv_ctx *ctx);

/* Verify against registered keys: item i uses key id key_idx[i] (uint32);
 * an id >= edv_keys_count() is rejected (never read out of bounds).
 * Same verdicts as edv_verify_batch with pk32[i] = that key's encoding. */
int edv_verify_batch_keyed(edv_ctx *ctx, const uint8_t *sig64, const uint32_t *key_idx, const uint8_t *msgs,
                           const uint64_t *msg_off, uint64_t n, uint8_t *accept_bits);
int edv_verify_batch_keyed_device(edv_ctx *ctx, const void *d_sig64, const void *d_key_idx, const void *d_msgs,
                                  const void *d_msg_off, uint64_t n, void *d_accept_words, void *stream);
/* One request against registered key key_id (*accept = 1 iff libsodium accepts; an id >=
 * edv_keys_count() rejects): the per-message authenticate() that missed the verify-ahead cache
 * (plenum/server/client_authn.py:99-100 -> nacl_wrappers.py:232-242 Verifier.verify for one
 * message).  Latency form: a workgroup of edv_resident_kernel stays resident and takes the request
 * from a mailbox in pinned host memory -- no launch, copy or completion event on the path -- and
 * leaves after 200 us without a request or as soon as any other call on the context queues GPU
 * work (it is relaunched by the next edv_verify_one).  Messages over 4 KiB, or a context with the
 * resident path off (EDV_RESIDENT=0), take one launch of edv_verify_small_kernel.  Same verdicts as
 * edv_verify_batch_keyed. */
int edv_verify_one(edv_ctx *ctx, const uint8_t *sig64, uint32_t key_id, const uint8_t *msg, uint64_t mlen,
                   uint8_t *accept);

/* Staged inputs: the caller DMAs its inputs piece by piece while it is still
 * producing the rest (the authenticator's batch scan queues each 4k-request
 * chunk's signature slots and messages as soon as its workers have written
 * them, so the PCIe transfer runs under the host work instead of after it).
 *   edv_stage_reserve(ctx, bytes): a device staging buffer of >= bytes (kept
 *     across calls; clears the put error state).
 *   edv_stage_put(ctx, src, nbytes, off): queue the copy of nbytes of pinned
 *     memory (edv_host_alloc) to staging offset off; returns at once; any
 *     thread (serialized inside); src must not change until the verify.
 *   edv_verify_staged(ctx, keyed, keys, slot_off, msg_base, msg_start,
 *     msg_end, n, accept_bits): n EDV_SIG_SLOT96 signature slots at staging
 *     offset slot_off, message i at staging msg_base + [msg_start[i],
 *     msg_end[i]) (any order, any gaps), keys as edv_verify_batch_keyed /
 *     edv_verify_batch (host arrays): waits for every put queued before it,
 *     then the same kernels and verdicts as the slot forms.  Fails if any put
 *     since the last reserve failed. */
int edv_stage_reserve(edv_ctx *ctx, uint64_t bytes);
int edv_stage_put(edv_ctx *ctx, const void *src, uint64_t nbytes, uint64_t off);
int edv_verify_staged(edv_ctx *ctx, int keyed, const uint8_t *keys, uint64_t slot_off, uint64_t msg_base,
                      const uint64_t *msg_start, const uint64_t *msg_end, uint64_t n, uint8_t *accept_bits);
/* Two batches in flight (a pipeline of staged batches): edv_stage_select(ctx, set) makes
 * staging set 0 or 1 current for the next edv_stage_reserve / edv_stage_put /
 * edv_verify_staged_submit; each set has its own staging buffer and verdict buffers, so batch
 * k + 1 is staged into one set while batch k's kernels still read the other.
 * edv_verify_staged_submit queues the verify of the staged batch and returns a ticket at once;
 * edv_verify_staged_collect(ctx, ticket, accept_bits) waits for it and writes the bits.
 * A set holding an uncollected submission refuses reserve and submit (EDV_EBUSY).
 * edv_verify_staged == submit + collect.  Replaces, like edv_verify_staged, libsodium's
 * crypto_sign_open per request (nacl_wrappers.py:108). */
int edv_stage_select(edv_ctx *ctx, int set);
int edv_verify_staged_submit(edv_ctx *ctx, int keyed, const uint8_t *keys, uint64_t slot_off, uint64_t msg_base,
                             const uint64_t *msg_start, const uint64_t *msg_end, uint64_t n, uint64_t *ticket);
int edv_verify_staged_collect(edv_ctx *ctx, uint64_t ticket, uint8_t *accept_bits);
/* A staged batch verified in parts while it is still being produced (the authenticator's
 * synchronous batch: its kernels run under its own scan, with key ids the scan takes from the
 * previous batches' identifiers and the authenticator checks after it).
 *   edv_verify_staged_begin(ctx, keyed, n, ticket): the current set for an n-item batch (its
 *     buffers sized here), held until edv_verify_staged_collect(ctx, ticket, bits).
 *   edv_verify_staged_part(ctx, keys, slot_off, msg_base, spans, n, lo, hi): items [lo, hi)
 *     (lo a multiple of 64) -- keys (n uint32 ids, or n x 32-byte keys) and spans (starts[n]
 *     then ends[n]) in edv_host_alloc memory, written for those items; their slots and
 *     messages put -- are copied and verified (edv_verify_staged's kernels) after every put
 *     queued before the call.  Any thread, one call at a time.
 *   edv_verify_staged_end(ctx): the verdicts' copy after the last part; a failed part is
 *     reported here (the set still needs its collect).
 * Items no part covered are rejected.  Replaces, like edv_verify_staged, libsodium's
 * crypto_sign_open per request (nacl_wrappers.py:108). */
int edv_verify_staged_begin(edv_ctx *ctx, int keyed, uint64_t n, uint64_t *ticket);
int edv_verify_staged_part(edv_ctx *ctx, const void *keys, uint64_t slot_off, uint64_t msg_base,
                           const uint64_t *spans, uint64_t n, uint64_t lo, uint64_t hi);
int edv_verify_staged_end(edv_ctx *ctx);
/* Items of the last staged batch again, on the general path: after edv_verify_staged (or a
 * collected edv_verify_staged_submit) of the current set, verify its items idx[j] (< that
 * batch's n) with the key bytes pk32[j] (32 each), accept bit j of accept_bits[(m + 7) / 8].
 * The batch's decoded signatures, spans and messages are still in HBM, so only the indices and
 * keys cross PCIe -- the authenticator's mixed batches (signers whose keys have no table: a
 * keyed verify of the whole batch, then these items by their key bytes).  Refused once the set
 * is reserved or begun again.  Replaces, like edv_verify_staged, libsodium's crypto_sign_open per
 * request (nacl_wrappers.py:108). */
int edv_verify_staged_subset(edv_ctx *ctx, const uint32_t *idx, const uint8_t *pk32, uint64_t m,
                             uint8_t *accept_bits);

/* Signature slots: the host-pointer verifies below take, instead of sig64,
 * n slots of EDV_SIG_SLOT96 bytes, so that the base58 decode of the request
 * signature (client_authn.py:89, b58decode) runs on the GPU:
 *   slot[95] = t > 0 : slot[0 .. t) is the signature's base58 text, which the
 *                      caller has checked decodes to exactly 64 bytes (value
 *                      < 2^512; the split of sig || ser at byte 64 then is the
 *                      plain one);
 *   slot[95] = 0     : slot[0 .. 64) is R || S, decoded by the caller.
 * Same verdicts as the sig64 forms on the decoded signatures. */
#define EDV_SIG_SLOT96 96
int edv_verify_batch_slots(edv_ctx *ctx, const uint8_t *sig_slots, const uint8_t *pk32, const uint8_t *msgs,
                           const uint64_t *msg_off, uint64_t n, uint8_t *accept_bits);
int edv_verify_batch_keyed_slots(edv_ctx *ctx, const uint8_t *sig_slots, const uint32_t *key_idx, const uint8_t *msgs,
                                 const uint64_t *msg_off, uint64_t n, uint8_t *accept_bits);

/* Asynchronous form of the host-pointer verifies (the authenticator overlaps
 * its scan of the next part of a batch with the GPU work of this one).
 * edv_verify_submit queues the copies, kernels and bitmask read-back and
 * returns a ticket; inputs outside edv_host_alloc memory are copied before it
 * returns, inputs inside it are read by DMA later and must stay unchanged
 * until edv_verify_collect(ticket) has returned, which waits and writes the
 * (n + 7) / 8 accept bytes.  keyed: keys = uint32 key ids, else n * 32 key
 * bytes; sig_format: 64 (R || S) or EDV_SIG_SLOT96.  Submissions complete in
 * order; every ticket should be collected (the 64 most recent are kept). */
int edv_verify_submit(edv_ctx *ctx, int keyed, const uint8_t *sig, int sig_format, const uint8_t *keys,
                      const uint8_t *msgs, const uint64_t *msg_off, uint64_t n, uint64_t *ticket);
int edv_verify_collect(edv_ctx *ctx, uint64_t ticket, uint8_t *accept_bits);

/* Pinned host memory (hipHostMalloc, portable to every device).  A host-
 * pointer verify whose inputs (signatures, keys, messages, offsets) lie in
 * such blocks copies them to the device straight from there, with no CPU
 * staging copy -- the authenticator's batch scan writes its output into them.
 * edv_host_free only after the verifies reading the block have returned. */
int edv_host_alloc(edv_ctx *ctx, uint64_t bytes, void **out);
int edv_host_free(void *p);

/* Either path with message spans instead of contiguous offsets: item i's
 * message is d_msgs[d_msg_start[i] .. d_msg_end[i]) (uint64 each), so the k
 * signatures of a multi-signature request (authenticate_multi, configs[3])
 * share one copy of the serialized message.  keyed = 0: d_keys is n * 32 key
 * bytes; keyed = 1: n uint32 registered key ids. */
int edv_verify_spans_device(edv_ctx *ctx, const void *d_sig64, const void *d_keys, int keyed, const void *d_msgs,
                            const void *d_msg_start, const void *d_msg_end, uint64_t n, void *d_accept_words,
                            void *stream);

/* ------------------------------------------------- signing (synthetic load) */

/* crypto_sign_seed_keypair for n seeds (32 bytes each): pk32_out n*32,
 * sk64_out n*64 (= seed || pk).  Host pointers. */
int edv_seed_keypair_batch(edv_ctx *ctx, const uint8_t *seeds32, uint64_t n, uint8_t *pk32_out, uint8_t *sk64_out);

/* Deterministic Ed25519 signatures (crypto_sign_detached), device pointers:
 * item i is signed with key d_sk64[key_idx[i]] over its message. */
int edv_sign_batch_device(edv_ctx *ctx, const void *d_sk64, const void *d_key_idx, const void *d_msgs,
                          const void *d_msg_off, uint64_t n, void *d_sig64_out, void *stream);

/* Signer with message spans (d_msg_start / d_msg_end, as edv_verify_spans_device). */
int edv_sign_spans_device(edv_ctx *ctx, const void *d_sk64, const void *d_key_idx, const void *d_msgs,
                          const void *d_msg_start, const void *d_msg_end, uint64_t n, void *d_sig64_out,
                          void *stream);

/* Host-pointer convenience form of edv_sign_batch_device. */
int edv_sign_batch(edv_ctx *ctx, const uint8_t *sk64, const uint32_t *key_idx, const uint8_t *msgs,
                   const uint64_t *msg_off, uint64_t n, uint8_t *sig64_out);

/* ---------------------------------------------------- request digests */

/* Request.digest = sha256(serialize_msg_for_signing(signingState))
 * (plenum/common/request.py:51-52), computed for every request at
 * construction: SHA-256 of each message, 32 bytes per item.  For a request
 * with no top-level keys besides identifier / reqId / operation /
 * protocolVersion / signature its signing bytes ARE the signingState bytes,
 * so the verify batch's message buffer serves both. */
int edv_sha256_spans_device(edv_ctx *ctx, const void *d_msgs, const void *d_msg_start, const void *d_msg_end,
                            uint64_t n, void *d_out32, void *stream);
int edv_sha256_batch(edv_ctx *ctx, const uint8_t *msgs, const uint64_t *msg_off, uint64_t n, uint8_t *out32);

/* ------------------------------------------------------ quorum vote tally */

/* Votes are (key, voter, phase) triples with an accept flag; the tally keeps
 * the reference's distinct-voter set semantics (models.py:21-37: a duplicate
 * vote counts once) and compares against Quorums(n_validators)
 * (quorums.py:15-32: f = (n-1)//3 for n >= 4 else 0; prepare = n-f-1,
 * commit = n-f).
 * A PREPARE from the primary of its key's view never counts: the replica
 * rejects it as SuspiciousNode(PR_FRM_PRIMARY) before Prepares.addVote
 * (plenum/server/replica.py:1289-1291).
 *   d_key, d_voter, d_phase, d_valid : n_votes entries (uint32, uint8, uint8, uint8)
 *   d_primary: n_keys bytes, the primary's voter index per key (0xff = none),
 *              or NULL (no primary rejection)
 *   d_ballot : n_keys * n_validators * 2 bytes of scratch/output, zeroed here;
 *              ballot[(k * 2 + phase) * n_validators + v] = 1 if a valid vote
 *   d_counts : n_keys * 2 uint32 (distinct voters per key and phase)
 *   d_quorum : n_keys bytes: bit0 = prepare quorum, bit1 = commit quorum. */
int edv_tally_device(edv_ctx *ctx, const void *d_key, const void *d_voter, const void *d_phase, const void *d_valid,
                     const void *d_primary, uint64_t n_votes, uint32_t n_keys, uint32_t n_validators, void *d_ballot, void *d_counts,
                     void *d_quorum, void *stream);

/* Second half of the tally alone: counts + quorum flags from a ballot array
 * (used after an all-reduce(max) of ballots across GPUs). */
int edv_tally_finish_device(edv_ctx *ctx, const void *d_ballot, uint32_t n_keys, uint32_t n_validators,
                            void *d_counts, void *d_quorum, void *stream);

/* Host-pointer convenience form of edv_tally_device. */
int edv_tally(edv_ctx *ctx, const uint32_t *key, const uint8_t *voter, const uint8_t *phase, const uint8_t *valid,
              const uint8_t *primary, uint64_t n_votes, uint32_t n_keys, uint32_t n_validators, uint32_t *counts_out, uint8_t *quorum_out);

/* ------------------------------------------------ BLS multi-signatures
 * The COMMIT / state-proof BLS check, replacing indy-crypto
 * 0.1.6 under crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:59-90 over
 * AMCL BN254 (algorithm: oracle/bls_bn254_oracle.py).  Wire forms: G1
 * (signatures) 128 bytes 0x04 | x | y | 63 zero bytes; G2 (generator,
 * verkeys) 128 bytes x.a | x.b | y.a | y.b; 32-byte big-endian coordinates.
 * A G1/G2 encoding that is off the curve decodes to the point at infinity.
 * One GPU lane per check, or two / four for small batches
 * (edv_options.bls_pair_lanes; a COMMIT round's ~25 see the latency, not the
 * throughput); host-pointer calls, synchronous. */

/* BlsCryptoVerifierIndyCrypto.verify_sig (:59-70) over a batch: item i
 * accepts iff e(sig_i, gen) == e(H(m_i), vk_i), H = indy-crypto Bls::_hash.
 * vk_off == NULL: one verkey per item (vk128[i]); else verify_multi_sig
 * (:72-84): item i's verkey is the sum of vk128[vk_off[i] .. vk_off[i+1]).
 * msg_off[n + 1] as edv_verify_batch.  accept_bits: ceil(n/8) bytes. */
int edv_bls_verify_batch(edv_ctx *ctx, const uint8_t *sig128, const uint8_t *msgs, const uint64_t *msg_off,
                         const uint8_t *vk128, const uint64_t *vk_off, const uint8_t *gen128, uint64_t n,
                         uint8_t *accept_bits);
/* BlsCryptoVerifierIndyCrypto.create_multi_sig (:86-90) over a batch:
 * out128[i] = sum of sig128[sig_off[i] .. sig_off[i+1]) (MultiSignature.new). */
int edv_bls_aggregate(edv_ctx *ctx, const uint8_t *sig128, const uint64_t *sig_off, uint64_t m, uint8_t *out128);
/* Test / bench data: sig128[i] = [sk_i] H(m_i) (BlsCryptoSignerIndyCrypto.sign,
 * :112-114), vk128[i] = [sk_i] gen (VerKey.new); sk 32 bytes big-endian < r.
 * (indy-crypto derives sk from a seed with AMCL's RAND; that derivation is
 * not restated.) */
int edv_bls_sign_batch(edv_ctx *ctx, const uint8_t *sk32, const uint8_t *msgs, const uint64_t *msg_off, uint64_t n,
                       uint8_t *sig128);
int edv_bls_keygen_batch(edv_ctx *ctx, const uint8_t *sk32, const uint8_t *gen128, uint64_t n, uint8_t *vk128);

#ifdef __cplusplus
}
#endif

#endif /* PLENUM_EDVERIFY_H */
