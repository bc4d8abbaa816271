// edverify.hip -- libplenum_edverify.so: batched Ed25519 verification for
// Plenum's request authenticator on MI355X (gfx950), behind the C ABI in
// include/edverify.h.
//
// Kernels (one HIP stream per context):
//   general path (any 32-byte key per request):
//     edv_hash_kernel    prechecks + SHA-512(R||A||M) mod L, one lane per request
//     edv_dedup_*        distinct keys of the sub-batch (hash table in HBM)
//     edv_table_kernel   per distinct key: decode -A, cached [1..8](-A) (AoS);
//                        4 tables [1..8]2^(64t)(-A) for keys with >= 4 requests
//     edv_dsm_kernel     [h](-A) + [S]B: signed radix-16 windows over the
//                        lane's cached multiples, [S]B from the base comb (HBM)
//   key-table path (registered keys, comb.h):
//     edv_hash_keyed_kernel, edv_comb_kernel<W>  fixed-base combs, no doublings
//   both paths end in
//     edv_encode_kernel<M>  M results per lane share one inversion
//                           (batch_encode.h), byte compare with R, wave
//                           ballot into the accept bitmask.
//   edv_sign_kernel / edv_keypair_kernel   deterministic Ed25519 signer
//   edv_tally_*          distinct-voter ballots -> counts -> quorum flags.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <mutex>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <thread>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "../../include/edverify.h"
#include "edv_internal.h"
#include "host_pool.h"
#include "batch_encode.h"
#include "comb.h"
#include "fe_lanes.h"
#include "sha256.h"
#include "verify_core.h"

using namespace edv;

#define EDV_VERSION "plenum-edverify 0.1.0 (gfx950)"

namespace {

constexpr int kBlock = 256;
constexpr uint64_t kMaxLanes = 1ull << 20;  // scratch lanes (grid-stride beyond)
constexpr int kTableWords = 9 * 4 * 10;     // [1..8](-A) cached + the identity (slot 8), u32 limbs

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) return set_err(EDV_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------ accessors

// Per-lane cached multiples [1..8](-A) (+ the identity in slot 8), AoS per
// lane: lane t of a 256-lane block owns kTableWords contiguous words in the
// block's region, entry j at word 40 j (YplusX | YminusX | Z | T2d).  A lane
// reads its own 160-B entry with 10 dwordx4 loads, i.e. 1-2 cache lines per
// entry.  (The former SoA layout -- word w of every lane in one 1 KiB row --
// made each per-lane random entry index touch 40 different lines: 88 KB of
// FETCH per request against ~12 KB of entries, profiles/r01m.)
constexpr uint32_t kRegionBytes = kTableWords * kBlock * 4;
struct DevTableA {
  uint32_t* __restrict__ base;  // this lane's 9 entries
  __device__ DevTableA(uint32_t* scratch, uint32_t block, uint32_t lane)
      : base((uint32_t*)((char*)scratch + (uint64_t)block * kRegionBytes) + lane * kTableWords) {}
  __device__ DevTableA(uint32_t* scratch, uint64_t slot) : base(scratch + slot * kTableWords) {}
  __device__ void store(int j, const ge_cached& c) const {
    uint4* p = (uint4*)(base + j * 40);
    uint32_t w[40];
#pragma unroll
    for (int l = 0; l < 10; ++l) {
      w[l] = c.YplusX.v[l];
      w[10 + l] = c.YminusX.v[l];
      w[20 + l] = c.Z.v[l];
      w[30 + l] = c.T2d.v[l];
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  }
  __device__ void load(int j, ge_cached& c) const {  // j = -1: the identity (slot 8)
    const uint4* p = (const uint4*)(base + (j >= 0 ? j : 8) * 40);
    uint32_t w[40];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const uint4 v = p[k];
      w[4 * k] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int l = 0; l < 10; ++l) {
      c.YplusX.v[l] = w[l];
      c.YminusX.v[l] = w[10 + l];
      c.Z.v[l] = w[20 + l];
      c.T2d.v[l] = w[30 + l];
    }
  }
};

// K tables of one distinct key, consecutive slots (u * K + t) of the scratch
struct DevTableSplit {
  uint32_t* __restrict__ base;
  __device__ DevTableSplit(uint32_t* scratch, uint64_t first_slot) : base(scratch + first_slot * kTableWords) {}
  __device__ void store(int t, int j, const ge_cached& c) const {
    DevTableA a(base, (uint64_t)t);
    a.store(j, c);
  }
  __device__ void load(int t, int j, ge_cached& c) const {
    const DevTableA a(base, (uint64_t)t);
    a.load(j, c);
  }
};

__device__ __forceinline__ void load_words(uint32_t* dst, const uint8_t* src, int nwords) {
  // src is 16-byte aligned for the sig/pk arrays (64 / 32 byte records)
  const uint4* s = (const uint4*)src;
  for (int k = 0; k < nwords / 4; ++k) {
    uint4 v = s[k];
    dst[4 * k] = v.x;
    dst[4 * k + 1] = v.y;
    dst[4 * k + 2] = v.z;
    dst[4 * k + 3] = v.w;
  }
}

// ---------------------------------------------------------------- kernels

// ---- split pipeline: hash -> table -> dsm (each kernel gets its own
// register budget; intermediates are SoA in the context scratch).

#ifndef EDV_HASH_MIN_WAVES
#define EDV_HASH_MIN_WAVES 4  // 94 VGPRs = 5 waves / SIMD; 6 (80 VGPRs + 36 B spill) measured no faster (profiles/r03a_ab_hash_occupancy)
#endif

// Length buckets: the lanes of a wave should hash messages of equal SHA-512
// block count, or every lane runs as many blocks as the longest message of
// its wave (configs[3], 64 B - 4 KiB log-uniform: 3.2x the VALU work).
// edv_len_key_kernel writes each request's block count (capped at 63) and a
// stable descending radix sort over those 6 bits (rocPRIM onesweep, one
// pass) yields perm: lane t hashes request perm[t], longest first.  Equal
// block counts keep request order (stability), so a batch of one length gets
// the identity permutation and keeps its coalesced loads.
constexpr int kLenKeyBits = 6;  // block counts 0..62; 63 = longer
__device__ __forceinline__ uint64_t hash_lane_request(uint64_t t, const uint32_t* __restrict__ perm) {
  return perm ? perm[t] : t;
}

// ---- signature slots (edverify.h EDV_SIG_SLOT96): the authenticator's
// base58 decode of the request signature (client_authn.py:89) moved off the
// host.  Slot i is 96 bytes; byte 95 = t > 0: bytes 0..t-1 are the base58
// text of a signature that the host checked decodes to exactly 64 bytes
// (hostpack.cpp b58_len64), so its value is < 2^512 and the decode is the
// 512-bit big-endian value of the text; t == 0: bytes 0..63 are R || S
// (decoded on the host: other lengths, which move bytes across the split at
// 64).  HBM: 96 B read + 64 B written per request.
__device__ __forceinline__ uint32_t b58_digit(uint32_t c) {
  // '1'-'9' 0-8, 'A'-'H' 9-16, 'J'-'N' 17-21, 'P'-'Z' 22-32, 'a'-'k' 33-43, 'm'-'z' 44-57
  uint32_t d = c - '1';
  d = c >= 'A' ? c - 'A' + 9 - (c > 'H') - (c > 'N') : d;
  d = c >= 'a' ? c - 'a' + 33 - (c > 'k') : d;
  return d;
}

constexpr uint32_t kPow58[6] = {1u, 58u, 3364u, 195112u, 11316496u, 656356768u};

__global__ __launch_bounds__(kBlock) void edv_b58_sig_kernel(const uint8_t* __restrict__ slots, uint64_t n,
                                                            uint8_t* __restrict__ sig64) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[24];
  load_words(w, slots + 96 * i, 24);
  const uint32_t t = w[23] >> 24;
  uint32_t out[16];
  if (t == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) out[j] = w[j];
  } else {
    // Horner over groups of five digits (58^5 < 2^32): acc = acc * 58^k + chunk,
    // k = the group's digits inside the text (0..5, per lane)
    uint32_t acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0;
#pragma unroll
    for (int g = 0; g < 19; ++g) {
      uint32_t chunk = 0, k = 0;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int p = 5 * g + q;
        if (p < 95 && (uint32_t)p < t) {
          chunk = chunk * 58u + b58_digit((w[p >> 2] >> (8 * (p & 3))) & 0xffu);
          ++k;
        }
      }
      const uint32_t mul = k == 5 ? kPow58[5] : k == 4 ? kPow58[4] : k == 3 ? kPow58[3] : k == 2 ? kPow58[2]
                         : k == 1 ? kPow58[1] : kPow58[0];
      uint64_t carry = chunk;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint64_t v = (uint64_t)acc[j] * mul + carry;
        acc[j] = (uint32_t)v;
        carry = v >> 32;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) out[j] = __builtin_bswap32(acc[15 - j]);  // big-endian bytes
  }
  uint4* o = (uint4*)(sig64 + 64 * i);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = make_uint4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
}

// Message i = msgs[ms[i] .. me[i]): me = msg_off + 1 for contiguous offsets,
// separate arrays for spans (several signatures over one message).
__global__ __launch_bounds__(kBlock) void edv_len_key_kernel(const uint64_t* __restrict__ ms,
                                                            const uint64_t* __restrict__ me, uint64_t n,
                                                            uint8_t* __restrict__ key) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t blocks = (me[i] - ms[i] + 64 + 17 + 127) / 128;  // SHA-512 blocks of R||A||M
  constexpr uint64_t cap = (1u << kLenKeyBits) - 1;
  key[i] = (uint8_t)(blocks < cap ? blocks : cap);
}

// ---- Packed (SoA) message layout, edv_options.length_buckets = 3 (north_star
// (1)): after the block-count sort, each 64-lane group of sorted hash lanes
// owns a region of the context's unit arena, units(longest message of the
// group) x 64 lanes x 16 B, unit p of lane l at region + p * 64 + l
// (sha512.h pack_lane_units: padded big-endian stream words after R || A).
// edv_group_units_kernel sizes the groups, an exclusive scan places them,
// edv_pack_units_kernel fills them (coalesced 1 KiB stores per wave) and the
// hash kernels read them with coalesced 1 KiB loads and no byte shuffling.
// A group whose region would pass the arena's end is read in place (AoS).
struct UnitArena {
  Chunk16* __restrict__ base;            // null: no packing
  const uint64_t* __restrict__ gunits;   // units per lane of group g
  const uint64_t* __restrict__ goff;     // exclusive prefix sum of gunits
  uint64_t cap;                          // arena size in units
  // lane t's unit 0, or null if its group is not packed
  __device__ __forceinline__ Chunk16* lane(uint64_t t) const {
    if (!base) return nullptr;
    const uint64_t g = t >> 6;
    const uint64_t o = goff[g];
    return (o + gunits[g]) * 64 <= cap ? base + o * 64 + (t & 63) : nullptr;
  }
};

__global__ __launch_bounds__(kBlock) void edv_group_units_kernel(const uint64_t* __restrict__ ms,
                                                                const uint64_t* __restrict__ me, uint64_t n,
                                                                const uint32_t* __restrict__ perm,
                                                                uint64_t* __restrict__ gunits) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t u = 0;
  if (t < n) {
    const uint64_t i = perm[t];
    u = sha512_units64(me[i] - ms[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {  // every lane of the wave takes part (no early return above)
    const uint64_t v = __shfl_xor(u, o, 64);
    u = v > u ? v : u;
  }
  if ((threadIdx.x & 63) == 0 && t < n) gunits[t >> 6] = u;
}

__global__ __launch_bounds__(kBlock) void edv_pack_units_kernel(const uint8_t* __restrict__ msgs,
                                                               const uint64_t* __restrict__ ms,
                                                               const uint64_t* __restrict__ me, uint64_t n,
                                                               const uint32_t* __restrict__ perm, UnitArena ua) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  Chunk16* u = ua.lane(t);
  if (!u) return;
  const uint64_t i = perm[t];
  pack_lane_units(u, 64, msgs + ms[i], me[i] - ms[i]);
}

template <bool kUnits>
__global__ __launch_bounds__(kBlock, EDV_HASH_MIN_WAVES) void edv_hash_kernel(const uint8_t* __restrict__ sig64,
                                                         const uint8_t* __restrict__ pk32,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ ms,
                                                         const uint64_t* __restrict__ me, uint64_t n,
                                                         uint32_t* __restrict__ h_soa, uint8_t* __restrict__ flags,
                                                         uint64_t stride, const uint32_t* __restrict__ perm,
                                                         UnitArena ua) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = hash_lane_request(t, perm);
  uint32_t sig[16], pk[8], h[8];
  load_words(sig, sig64 + 64 * i, 16);
  load_words(pk, pk32 + 32 * i, 8);
  const uint64_t o0 = ms[i], o1 = me[i];
  const Chunk16* units = kUnits ? ua.lane(t) : nullptr;
  const bool ok = units ? verify_phase_hash_units(h, sig, pk, units, 64, o1 - o0)
                        : verify_phase_hash(h, sig, pk, msgs + o0, o1 - o0);
#pragma unroll
  for (int k = 0; k < 8; ++k) h_soa[k * stride + i] = h[k];
  flags[i] = ok ? 1 : 0;
}

#ifndef EDV_TABLE_MIN_WAVES
#define EDV_TABLE_MIN_WAVES 2  // 168 VGPRs (+spill) beats 256+256 AGPRs at 1 wave: table -8%
#endif
// ---- general path, distinct keys of a sub-batch: the table kernel decodes
// each distinct 32-byte key once (a batch of 1M requests from 1,000 signers
// builds 1,000 tables, not 1M).  Open-addressing hash table over the
// sub-batch: slot = request index of the key's representative (0xffffffff =
// empty); the full 32 bytes are compared, so distinct keys never share a
// table whatever their hash.  Which request becomes the representative
// depends on the order of the atomics; the table -- a function of the key
// bytes only -- does not.
constexpr uint32_t kEmptySlot = 0xffffffffu;
__device__ __forceinline__ uint32_t key_hash(const uint32_t pk[8]) {
  uint32_t h = pk[0] * 0x9e3779b1u;
  h ^= pk[1] * 0x85ebca77u;
  h ^= (pk[2] ^ pk[5]) * 0xc2b2ae3du;
  h ^= (pk[3] ^ pk[7]) * 0x27d4eb2fu;
  return h ^ (h >> 15);
}
__device__ __forceinline__ bool same_key(const uint8_t* __restrict__ pk32, uint64_t a, const uint32_t pk[8]) {
  uint32_t w[8];
  load_words(w, pk32 + 32 * a, 8);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) eq = eq && w[k] == pk[k];
  return eq;
}
// slot of request i's key (inserting i as the representative if new)
__device__ uint32_t dedup_slot(const uint8_t* __restrict__ pk32, uint64_t i, uint32_t* __restrict__ slots,
                               uint32_t nslots, bool insert) {
  uint32_t pk[8];
  load_words(pk, pk32 + 32 * i, 8);
  uint32_t h = key_hash(pk) % nslots;
  for (uint32_t probe = 0; probe < nslots; ++probe) {
    uint32_t s = __atomic_load_n(&slots[h], __ATOMIC_RELAXED);
    if (s == kEmptySlot) {
      if (!insert) return kEmptySlot;  // unreachable after the insert pass
      s = atomicCAS(&slots[h], kEmptySlot, (uint32_t)i);
      if (s == kEmptySlot) return h;
    }
    if (s == (uint32_t)i || same_key(pk32, s, pk)) return h;
    h = h + 1 == nslots ? 0 : h + 1;
  }
  return kEmptySlot;  // table full: impossible with nslots = 2n
}
// every request records its key's slot
__global__ __launch_bounds__(kBlock) void edv_dedup_insert_kernel(const uint8_t* __restrict__ pk32, uint64_t n,
                                                                 uint32_t* __restrict__ slots, uint32_t nslots,
                                                                 uint32_t* __restrict__ req_slot) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  req_slot[i] = dedup_slot(pk32, i, slots, nslots, true);
}
// representative -> compact key index u (reps[u] = its request)
__global__ __launch_bounds__(kBlock) void edv_dedup_assign_kernel(uint64_t n, const uint32_t* __restrict__ slots,
                                                                 const uint32_t* __restrict__ req_slot,
                                                                 uint32_t* __restrict__ slot_u,
                                                                 uint32_t* __restrict__ reps,
                                                                 uint32_t* __restrict__ count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t h = req_slot[i];
  if (slots[h] == (uint32_t)i) {
    const uint32_t u = atomicAdd(count, 1u);
    slot_u[h] = u;
    reps[u] = (uint32_t)i;
  }
}

// Tables per distinct key: K = 8 with at least 16 requests per distinct key
// in the sub-batch, K = 4 with at least 4, else 1.  The K tables of all keys
// then fit the sub-batch's scratch (K * count <= n), and the 256 (K-1)/K
// extra doublings per key cost at most 256 (K-1)/K^2 per request against
// 256 (K-1)/K saved in every ladder.  Decided on the device from the
// distinct-key count, identically by the table and ladder kernels.
__device__ __forceinline__ int split_of(uint32_t count, uint64_t n) {
  return 16ull * count <= n ? 8 : 4ull * count <= n ? 4 : 1;
}

// Tables of distinct key u (u < *count): decode -A of request reps[u]'s key,
// the K tables into slots u*K.., key_ok[u] = the key decodes.
__global__ __launch_bounds__(kBlock, EDV_TABLE_MIN_WAVES) void edv_table_kernel(const uint8_t* __restrict__ pk32,
                                                          uint64_t n, const uint32_t* __restrict__ reps,
                                                          const uint32_t* __restrict__ count,
                                                          uint32_t* __restrict__ table, uint8_t* __restrict__ key_ok) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cnt = *count;
  if (u >= cnt) return;
  uint32_t pk[8];
  load_words(pk, pk32 + 32 * (uint64_t)reps[u], 8);
  bool ok;
  const int k = split_of(cnt, n);
  if (k == 8) {
    const DevTableSplit tas(table, 8 * u);
    ok = verify_phase_table_split<8>(pk, tas);
  } else if (k == 4) {
    const DevTableSplit tas(table, 4 * u);
    ok = verify_phase_table_split<4>(pk, tas);
  } else {
    DevTableA ta(table, u);
    ok = verify_phase_table(pk, ta);
  }
  key_ok[u] = ok ? 1 : 0;
}

// Result points R' = (X : Y : Z), SoA [30][stride]: word w of request i at
// w * stride + i (coalesced stores here and loads in edv_encode_kernel).
__device__ __forceinline__ void store_point_soa(uint32_t* __restrict__ pt, uint64_t stride, uint64_t i,
                                                const ge_p3& Q) {
#pragma unroll
  for (int l = 0; l < 10; ++l) {
    pt[(0 + l) * stride + i] = Q.X.v[l];
    pt[(10 + l) * stride + i] = Q.Y.v[l];
    pt[(20 + l) * stride + i] = Q.Z.v[l];
  }
}

__device__ __forceinline__ void load_niels(ge_niels& nb, const uint32_t* __restrict__ p) {
  const uint4* q = (const uint4*)p;
  uint32_t w[32];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 v = q[k];
    w[4 * k] = v.x;
    w[4 * k + 1] = v.y;
    w[4 * k + 2] = v.z;
    w[4 * k + 3] = v.w;
  }
#pragma unroll
  for (int l = 0; l < 10; ++l) {
    nb.ypx.v[l] = w[l];
    nb.ymx.v[l] = w[10 + l];
    nb.xy2d.v[l] = w[20 + l];
  }
}

// A comb table in global memory (comb.h layout: row-major, 32-word entries).
template <int W>
struct DevComb {
  const uint32_t* __restrict__ tab;    // entry 0 of row 0
  const uint32_t* __restrict__ ident;  // kEntryWords-word identity entry (global memory)
  // words from row r to row r + 1: one table's row for the base table; for
  // the key store (row-major over keys) key_cap tables' rows
  uint64_t row_words = (uint64_t)Window<W>::kEntries * kEntryWords;
  __device__ const uint32_t* entry(int row, int j) const {
    return j >= 0 ? tab + (uint64_t)(uint32_t)row * row_words + (uint32_t)j * kEntryWords : ident;
  }
  __device__ void load(int row, int j, ge_niels& nb) const { load_niels(nb, entry(row, j)); }
  __device__ uint32_t touch(int row, int j) const {  // comb_mul_add's line prefetch
    return *(const volatile uint32_t*)entry(row, j);
  }
};

#ifndef EDV_DSM_MIN_WAVES
#define EDV_DSM_MIN_WAVES 2
#endif
__global__ __launch_bounds__(kBlock, EDV_DSM_MIN_WAVES) void edv_dsm_kernel(const uint8_t* __restrict__ sig64, uint64_t n,
                                                        const uint32_t* __restrict__ h_soa,
                                                        uint32_t* __restrict__ table, uint64_t stride,
                                                        const uint32_t* __restrict__ btab_comb,
                                                        const uint32_t* __restrict__ ident,
                                                        uint32_t* __restrict__ pt,
                                                        const uint32_t* __restrict__ req_slot,
                                                        const uint32_t* __restrict__ slot_u,
                                                        const uint32_t* __restrict__ count,
                                                        const uint8_t* __restrict__ key_ok,
                                                        uint8_t* __restrict__ flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t S[8], h[8];
  load_words(S, sig64 + 64 * i + 32, 8);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = h_soa[k * stride + i];
  const uint32_t u = slot_u[req_slot[i]];
  if (!key_ok[u]) flags[i] = 0;  // the key does not decode: reject (the table is still written, so the ladder runs)
  const DevComb<kBaseW> cb{btab_comb, ident};
  ge_p3 Q;
  uint32_t sink;
  const int split = split_of(*count, n);
  if (split == 8) {
    const DevTableSplit tas(table, 8ull * u);
    sink = verify_phase_dsm_split_point<8>(Q, h, S, tas, cb);
  } else if (split == 4) {
    const DevTableSplit tas(table, 4ull * u);
    sink = verify_phase_dsm_split_point<4>(Q, h, S, tas, cb);
  } else {
    const DevTableA ta(table, (uint64_t)u);
    sink = verify_phase_dsm_point(Q, h, S, ta, cb);
  }
  store_point_soa(pt, stride, i, Q);
  if (sink == 0x9e3779b9u && stride == 0) pt[i] = sink;  // keeps the prefetches live
}

// Batched encode + compare + ballot.  Lane l of wave v owns requests
// v*64*M + 64*j + l (j < M): every j is one coalesced 64-request word.
// With perm (the comb ran in key-sorted order): slot r of pt / pre is request
// perm[r], whose R and flags are read there and whose verdict goes to
// ok8[perm[r]] (edv_ok_pack_kernel makes the words).
struct DevEncode {
  const uint32_t* __restrict__ pt;
  uint32_t* __restrict__ pre;
  const uint8_t* __restrict__ sig64;
  const uint8_t* __restrict__ flags;
  unsigned long long* __restrict__ words;
  uint64_t stride, n, base, wbase;  // base = this lane's request for j = 0; wbase = word for j = 0
  uint32_t lane;
  const uint32_t* __restrict__ perm;
  uint8_t* __restrict__ ok8;
  __device__ uint64_t req(int j) const { return base + 64ull * j; }
  __device__ bool valid(int j) const { return req(j) < n; }
  __device__ void z(int j, fe& f) const {
    const uint64_t r = req(j);
#pragma unroll
    for (int l = 0; l < 10; ++l) f.v[l] = pt[(20 + l) * stride + r];
  }
  __device__ void xy(int j, fe& X, fe& Y) const {
    const uint64_t r = req(j);
#pragma unroll
    for (int l = 0; l < 10; ++l) {
      X.v[l] = pt[l * stride + r];
      Y.v[l] = pt[(10 + l) * stride + r];
    }
  }
  __device__ void put_pre(int j, const fe& f) const {
    if (!valid(j)) return;
    const uint64_t r = req(j);
#pragma unroll
    for (int l = 0; l < 10; ++l) pre[l * stride + r] = f.v[l];
  }
  __device__ void get_pre(int j, fe& f) const {
    fe_1(f);
    if (!valid(j)) return;
    const uint64_t r = req(j);
#pragma unroll
    for (int l = 0; l < 10; ++l) f.v[l] = pre[l * stride + r];
  }
  __device__ void emit(int j, const uint32_t enc[8], bool zero_z) const {
    bool ok = false;
    uint64_t r = 0;
    if (valid(j)) {
      r = perm ? perm[req(j)] : req(j);
      const uint4* R = (const uint4*)(sig64 + 64 * r);
      const uint4 a = R[0], b = R[1];
      ok = !zero_z && flags[r] && enc[0] == a.x && enc[1] == a.y && enc[2] == a.z && enc[3] == a.w &&
           enc[4] == b.x && enc[5] == b.y && enc[6] == b.z && enc[7] == b.w;
    }
    if (perm) {
      if (valid(j)) ok8[r] = ok ? 1 : 0;
      return;
    }
    const unsigned long long bits = __ballot(ok);
    if (lane == 0 && valid(j)) words[wbase + j] = bits;
  }
};

#ifndef EDV_ENCODE_M
#define EDV_ENCODE_M 16
#endif
constexpr int kEncodeM = EDV_ENCODE_M;

template <int M>
__global__ __launch_bounds__(kBlock) void edv_encode_kernel(const uint8_t* __restrict__ sig64, uint64_t n,
                                                           const uint32_t* __restrict__ pt,
                                                           uint32_t* __restrict__ pre,
                                                           const uint8_t* __restrict__ flags,
                                                           unsigned long long* __restrict__ accept_words,
                                                           uint64_t stride, const uint32_t* __restrict__ perm,
                                                           uint8_t* __restrict__ ok8) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t wave = g >> 6;
  const uint32_t lane = (uint32_t)(g & 63);
  if (wave * 64ull * M >= n) return;  // whole wave past the end (wave-uniform)
  DevEncode a{pt, pre, sig64, flags, accept_words, stride, n, wave * 64ull * M + lane, wave * M, lane, perm, ok8};
  encode_batch<M>(a);
}

// Accept words from per-request verdict bytes (the key-sorted path): one lane per request.
__global__ __launch_bounds__(kBlock) void edv_ok_pack_kernel(const uint8_t* __restrict__ ok8, uint64_t n,
                                                            unsigned long long* __restrict__ words) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((i & ~63ull) >= n) return;  // whole wave past the end (wave-uniform)
  const unsigned long long bits = __ballot(i < n && ok8[i] != 0);
  if ((i & 63) == 0) words[i >> 6] = bits;
}

// edv_verify_staged_subset: item idx[j] of the last staged batch (its decoded signature and its
// message span, starts [n] then ends [n]) into position j of the subset's contiguous inputs.
__global__ __launch_bounds__(kBlock) void edv_subset_gather_kernel(const uint32_t* __restrict__ idx, uint64_t m,
                                                                  uint64_t n, const uint8_t* __restrict__ sig,
                                                                  const uint64_t* __restrict__ spans,
                                                                  uint8_t* __restrict__ sig_out,
                                                                  uint64_t* __restrict__ spans_out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint64_t i = idx[j] < n ? idx[j] : 0;  // (checked on the host)
  const uint4* s = (const uint4*)(sig + 64 * i);
  uint4* o = (uint4*)(sig_out + 64 * j);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = s[k];
  spans_out[j] = spans[i];
  spans_out[m + j] = spans[n + i];
}

// ---- key order of the comb (edv_options.key_sort) ------------------------------
// A counting sort of a sub-batch's key ids: requests of one key become
// neighbours, so a wave's 64 comb lanes gather from one key's rows (a few
// pages) instead of 64 keys' rows spread over the key store -- what lets the
// wide key window (16: 4 MiB rows, 64 MiB per key) run at its row count when
// the batch arrives in any key order.  Bins = ids, the last bin for
// out-of-range ids.  (1) each block histograms a contiguous range of the
// requests in LDS and adds its bins into the global totals; (2) an exclusive
// scan of the totals gives each bin's base, copied into the cursors; (3) each
// block histograms its range again, reserves a stretch of every bin it uses
// with one global atomic on the bin's cursor, and places its requests there
// with LDS cursors.  Order within a key is arbitrary (verdicts are per
// request).
constexpr uint32_t kSortBlocks = 256, kSortThreads = 1024;
constexpr uint64_t kCompactBytes = 256 << 10;  // host_submit: small chunks in one pinned block, one copy
constexpr size_t kMaxPending = 64;  // uncollected edv_verify_submit tickets per context
constexpr uint32_t kSortMaxBins = 16384;  // 64 KiB of LDS per block
__device__ __forceinline__ void sort_range(uint64_t n, uint64_t& lo, uint64_t& hi) {
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  lo = blockIdx.x * per;
  hi = lo + per < n ? lo + per : n;
}
__device__ __forceinline__ void block_hist(const uint32_t* __restrict__ kidx, uint64_t lo, uint64_t hi, uint32_t nb,
                                           uint32_t* h) {
  for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) h[k] = 0;
  __syncthreads();
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t k = kidx[i];
    atomicAdd(&h[k < nb - 1 ? k : nb - 1], 1u);
  }
  __syncthreads();
}
__global__ __launch_bounds__(kSortThreads) void edv_key_hist_kernel(const uint32_t* __restrict__ kidx, uint64_t n,
                                                                   uint32_t nb, uint32_t* __restrict__ total) {
  extern __shared__ uint32_t h[];
  uint64_t lo, hi;
  sort_range(n, lo, hi);
  block_hist(kidx, lo, hi, nb, h);
  for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x)
    if (h[k]) atomicAdd(&total[k], h[k]);
}
__global__ __launch_bounds__(kSortThreads) void edv_key_scatter_kernel(const uint32_t* __restrict__ kidx, uint64_t n,
                                                                      uint32_t nb, uint32_t* __restrict__ cursor,
                                                                      uint32_t* __restrict__ perm) {
  extern __shared__ uint32_t h[];
  uint64_t lo, hi;
  sort_range(n, lo, hi);
  block_hist(kidx, lo, hi, nb, h);
  for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x)
    if (h[k]) h[k] = atomicAdd(&cursor[k], h[k]);  // this block's stretch of bin k
  __syncthreads();
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t k = kidx[i];
    perm[atomicAdd(&h[k < nb - 1 ? k : nb - 1], 1u)] = (uint32_t)i;
  }
}

// ---- key-table path (comb.h) ---------------------------------------------
// Registered keys: comb tables of -A at the context's key window (EDV_KEY_WINDOWS).
// Base point: W = 8 comb table (512 KiB) built once per context by the same
// kernels.
#ifndef EDV_COMB_MIN_WAVES
#define EDV_COMB_MIN_WAVES 4  // 128 VGPRs: 1M lanes = 3.8 rounds of 262k (3 waves: 5.1 rounds -> 15% tail); -11% vs 3 (tools/ab_keyed.py)
#endif
constexpr uint64_t kBaseTabWords = Window<kBaseW>::kTableWords;  // 2.95G words at W = 24
constexpr int kRowWords = 40;

// One lane per key: decode -A, libsodium's key checks, the row bases.
template <int W>
// ids (edv_keys_set_many_async): key k of the launch is store slot ids[k]; its encoding is
// pk32[k] and is also copied to store_pk[ids[k]] (valid and store_pk indexed by slot); null ids:
// slots are consecutive and pk32 / valid already point at the first
__global__ __launch_bounds__(kBlock) void edv_key_rows_kernel(const uint8_t* __restrict__ pk32, uint64_t nkeys,
                                                             uint32_t* __restrict__ rows,
                                                             uint8_t* __restrict__ valid,
                                                             const uint32_t* __restrict__ ids = nullptr,
                                                             uint8_t* __restrict__ store_pk = nullptr) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  uint32_t pk[8];
  load_words(pk, pk32 + 32 * k, 8);
  const uint64_t slot = ids ? ids[k] : k;
  if (ids) {
#pragma unroll
    for (int j = 0; j < 8; ++j) ((uint32_t*)(store_pk + 32 * slot))[j] = pk[j];
  }
  ge_p3 P;
  const bool dec = ge_frombytes(P, pk, true);
  valid[slot] = (dec && is_canonical_point(pk) && !has_small_order(pk)) ? 1 : 0;
  comb_rows<W>(rows + k * Window<W>::kRows * kRowWords, P);
}

// One lane per (row, c), c < NCH, filling entries c, c + NCH, c + 2 NCH, ...
// of its row (CH = kEntries / NCH of them, one inversion per lane).
template <int W>
struct FillShape {
  static constexpr int E = Window<W>::kEntries;
  static constexpr int CH = E < 32 ? E : 32;
  static constexpr int NCH = E / CH;
};
// Row r of the launch is row r % kRows of table key0 + r / kRows; the store is
// row-major over tables: row `row` of table k at (row * cap + k) * kEntries
// entries (the base table: key0 = 0, cap = 1).
template <int W>
__global__ __launch_bounds__(kBlock) void edv_comb_fill_kernel(const uint32_t* __restrict__ rows, uint64_t nrows,
                                                              uint32_t* __restrict__ tab, uint32_t* __restrict__ pre,
                                                              uint64_t key0, uint64_t cap,
                                                              const uint32_t* __restrict__ ids = nullptr) {
  using F = FillShape<W>;
  const uint64_t nl = nrows * F::NCH;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nl) return;
  const uint64_t r = g / F::NCH;
  const int c = (int)(g % F::NCH);
  const uint64_t row = r % Window<W>::kRows,
                 k = ids ? (uint64_t)ids[key0 + r / Window<W>::kRows] : key0 + r / Window<W>::kRows;
  comb_fill_strided(tab + (row * cap + k) * F::E * kEntryWords, pre + g * 10, nl * 10, rows + r * kRowWords, c,
                    F::NCH, F::CH);
}

// Base-point table: one lane decodes B and writes its 32 row bases ...
__global__ void edv_base_rows_kernel(uint32_t* __restrict__ rows) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint32_t b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) b[k] = 0x66666666u;
  b[0] = 0x66666658u;  // B = (x, 4/5), x even
  ge_p3 P;
  ge_frombytes(P, b, false);
  comb_rows<kBaseW>(rows, P);
}
template <bool kUnits>
__global__ __launch_bounds__(kBlock, EDV_HASH_MIN_WAVES) void edv_hash_keyed_kernel(const uint8_t* __restrict__ sig64,
                                                               const uint32_t* __restrict__ key_idx,
                                                               uint32_t key_count,
                                                               const uint8_t* __restrict__ key_pk,
                                                               const uint8_t* __restrict__ key_valid,
                                                               const uint8_t* __restrict__ msgs,
                                                               const uint64_t* __restrict__ ms,
                                                               const uint64_t* __restrict__ me, uint64_t n,
                                                               uint32_t* __restrict__ h_soa,
                                                               uint8_t* __restrict__ flags, uint64_t stride,
                                                               const uint32_t* __restrict__ perm, UnitArena ua) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = hash_lane_request(t, perm);
  uint32_t sig[16], pk[8], h[8];
  load_words(sig, sig64 + 64 * i, 16);
  const uint32_t key = key_idx[i];
  const bool in_range = key < key_count;  // out-of-range ids reject, never read out of bounds
  const uint64_t k = in_range ? key : 0;
  load_words(pk, key_pk + 32 * k, 8);
  const uint64_t o0 = ms[i], o1 = me[i];
  const Chunk16* units = kUnits ? ua.lane(t) : nullptr;
  const bool hashed = units ? verify_phase_hash_units(h, sig, pk, units, 64, o1 - o0)
                            : verify_phase_hash(h, sig, pk, msgs + o0, o1 - o0);
  const bool ok = hashed && in_range && key_valid[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) h_soa[k * stride + i] = h[k];
  flags[i] = ok ? 1 : 0;
}

#ifndef EDV_COMB_SET
#define EDV_COMB_SET 1  // 1: the key comb's row 0 by comb_set (1 multiplication, not a 7-multiplication addition)
#endif
#ifndef EDV_COMB_LDS
#define EDV_COMB_LDS 0  // 1: entries gathered one row ahead by LDS-DMA (comb_dual_lds): -3% c1, -10% c2 (r02b A/B)
#endif

// LDS-DMA gather of one 128-B table entry per lane: 8 global_load_lds_dwordx4,
// piece k of every lane at lds + k * 1 KiB + lane * 16 B (the DMA's lane-linear
// destination).  No VGPR holds the entry while it is in flight, so the next
// row's gather runs under the current row's mixed addition without the
// register cost of a register prefetch (which spilled at 4 waves / SIMD).
constexpr int kLdsWaveWords = 8 * 64 * 4;  // 8 KiB per wave
__device__ __forceinline__ void dma_entry(const uint32_t* src, uint32_t* lds) {
#pragma unroll
  for (int k = 0; k < 8; ++k)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 4 * k),
                                     (__attribute__((address_space(3))) void*)(lds + k * 256), 16, 0, 0);
}
__device__ __forceinline__ void lds_entry(ge_niels& nb, const uint32_t* lds, uint32_t lane) {
  uint32_t w[32];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 v = *(const uint4*)(lds + k * 256 + lane * 4);
    w[4 * k] = v.x;
    w[4 * k + 1] = v.y;
    w[4 * k + 2] = v.z;
    w[4 * k + 3] = v.w;
  }
#pragma unroll
  for (int l = 0; l < 10; ++l) {
    nb.ypx.v[l] = w[l];
    nb.ymx.v[l] = w[10 + l];
    nb.xy2d.v[l] = w[20 + l];
  }
}

// [h](-A) + [S]B over the key comb (W) and the base comb (kBaseW) as one
// stream of kRows(W) + kRows(kBaseW) entries: entry s + 1 is DMA'd into the
// wave's LDS slot right after entry s has been read out of it, so each gather
// has a whole mixed addition (x 4 waves per SIMD) to land.
template <int W>
__device__ void comb_dual_lds(ge_p3& Q, const uint32_t h[8], const uint32_t S[8], const DevComb<W>& ta,
                              const DevComb<kBaseW>& tb, uint32_t* lds, uint32_t lane) {
  constexpr int RK = Window<W>::kRows, RB = Window<kBaseW>::kRows;
  CombDigits<W> dh(h);
  int e = dh.next();
  dma_entry(ta.entry(0, (e < 0 ? -e : e) - 1), lds);
  ge_niels nb;
  lds_entry(nb, lds, lane);
  int e_next = dh.next();
  dma_entry(ta.entry(1, (e_next < 0 ? -e_next : e_next) - 1), lds);
  comb_set_entry(Q, nb, e);
#pragma unroll 1
  for (int r = 1; r < RK; ++r) {
    e = e_next;
    lds_entry(nb, lds, lane);
    if (r + 1 < RK) {
      e_next = dh.next();
      dma_entry(ta.entry(r + 1, (e_next < 0 ? -e_next : e_next) - 1), lds);
    } else {  // the base comb's row 0: digit 0 of S + bias needs only the low word
      e_next = (int)((S[0] + Window<kBaseW>::bias_word(0)) & ((1u << kBaseW) - 1)) - (1 << (kBaseW - 1));
      dma_entry(tb.entry(0, (e_next < 0 ? -e_next : e_next) - 1), lds);
    }
    comb_apply(Q, nb, e);
  }
  CombDigits<kBaseW> ds(S);
  e_next = ds.next();
#pragma unroll 1
  for (int r = 0; r < RB; ++r) {
    e = e_next;
    lds_entry(nb, lds, lane);
    if (r + 1 < RB) {
      e_next = ds.next();
      dma_entry(tb.entry(r + 1, (e_next < 0 ? -e_next : e_next) - 1), lds);
    }
    comb_apply(Q, nb, e);
  }
}
// [h](-A) + [S]B over the key's comb (W) and the base comb (kBaseW): no doublings.
template <int W>
__global__ __launch_bounds__(kBlock, EDV_COMB_MIN_WAVES) void edv_comb_kernel(const uint8_t* __restrict__ sig64,
                                                         const uint32_t* __restrict__ key_idx, uint32_t key_count,
                                                         uint64_t n, const uint32_t* __restrict__ h_soa,
                                                         const uint32_t* __restrict__ key_tab, uint64_t key_cap,
                                                         const uint32_t* __restrict__ btab,
                                                         const uint32_t* __restrict__ ident,
                                                         uint32_t* __restrict__ pt, uint64_t stride,
                                                         const uint32_t* __restrict__ kperm) {
  // lane t runs request i = kperm[t] (key-sorted order, edv_options.key_sort) and
  // leaves R' in slot t for the encode, which reads kperm back
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = kperm ? kperm[t] : t;
  uint32_t S[8], h[8];
  load_words(S, sig64 + 64 * i + 32, 8);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = h_soa[k * stride + i];
  const uint32_t key0 = key_idx[i];
  const uint32_t key = key0 < key_count ? key0 : 0;  // flags[i] is 0 for an out-of-range id
  constexpr uint64_t kRowWordsW = (uint64_t)Window<W>::kEntries * kEntryWords;
  const DevComb<W> ta{key_tab + (uint64_t)key * kRowWordsW, ident, key_cap * kRowWordsW};  // row-major store
  const DevComb<kBaseW> tb{btab, ident};
  ge_p3 Q;
#if EDV_COMB_LDS
  __shared__ uint32_t lds_slots[kBlock / 64][kLdsWaveWords];
  comb_dual_lds<W>(Q, h, S, ta, tb, lds_slots[threadIdx.x >> 6], threadIdx.x & 63);
  uint32_t sink = 0;
#elif EDV_COMB_SET
  comb_mul_set<W>(Q, h, ta);  // Q = [h](-A): row 0 set, not added to the identity
  uint32_t sink = comb_mul_add<kBaseW>(Q, S, tb);
#else
  ge_p3_0(Q);
  uint32_t sink = comb_mul_add<W>(Q, h, ta);
  sink ^= comb_mul_add<kBaseW>(Q, S, tb);
#endif
  store_point_soa(pt, stride, t, Q);
  if (sink == 0x9e3779b9u && key0 == 0xffffffffu && key_count == 0) pt[t] = sink;  // keeps the prefetches live
}

// ---- low-latency keyed verify for small batches (edv_options.small_batch) -------
// A batch of a few requests (authenticate() of a message the verify-ahead did
// not cover) is latency-bound: the three-kernel path runs each request's 29
// mixed additions and its own ~265-product inversion as serial chains on one
// lane (hash 35 + comb 90 + encode 85 us).  Here each request gets a workgroup
// of three waves:
//   wave 0: prechecks + h = SHA-512(R || A || M) mod L (lane 0), then the key
//           comb's rows on lanes 0..RK-1 -- each lane fetches its row's signed
//           entry and sets it as a point (one product) -- summed as a tree of
//           full additions across lanes (log2 levels, points moved by
//           shuffles), then the base sum added and the result compared;
//   wave 1: the base comb's rows the same way ([S]B needs only S);
//   wave 2: R decoded (libsodium's frombytes: the x of R's sign from y, one
//           exponentiation), so no inversion of R' is needed:
//             encode(R') == R  <=>  y_R < p, (x_R, y_R) on the curve, and
//             X' == x_R Z', Y' == y_R Z'  (x_R = 0 with the sign bit set never
//             matches: libsodium encodes x = 0 with sign 0).
// The exponentiation runs beside the hash instead of after the comb.  Same
// verdicts as the batch path (tests/test_gpu_parity.py: small batches == the
// large path on golden, edge and random items).
__device__ __forceinline__ void shfl_fe(fe& out, const fe& in, int delta) {
#pragma unroll
  for (int l = 0; l < 10; ++l) out.v[l] = (uint32_t)__shfl_down((int)in.v[l], delta, 64);
}
// Sum of the p3 points of lanes 0..width-1 of this wave (width a power of two
// <= 64; lanes >= rows hold the identity) into lane 0: log2(width) levels of
// p + q (q as cached).
#ifndef EDV_SMALL_ORDER
// fe_mul_o order of the small kernel's products.  One wave's serial carry-started chains
// (2) beat ten independent accumulators (1) here too: R's decode 99.6 vs 118.2 us, the kernel
// 103.8 vs 123.4 us (tools/small_probe.py, profiles/r05m); and two half-chains joined by a
// carry ripple (3): decode 107.7 vs 99.0 us (profiles/r05o).
#define EDV_SMALL_ORDER 2
#endif
constexpr int kSO = EDV_SMALL_ORDER;
__device__ void lane_tree_sum(ge_p3& P, int lane, int width) {
#pragma unroll 1
  for (int step = 1; step < width; step <<= 1) {
    ge_p3 Q;
    shfl_fe(Q.X, P.X, step);
    shfl_fe(Q.Y, P.Y, step);
    shfl_fe(Q.Z, P.Z, step);
    shfl_fe(Q.T, P.T, step);
    if ((lane & (2 * step - 1)) == 0 && lane < width) {
      ge_cached c;
      ge_p1p1 t;
      ge_p3_to_cached<kSO>(c, Q);
      ge_add<kSO>(t, P, c);
      ge_p1p1_to_p3_addlike<kSO>(P, t);
    }
  }
}
// The point of row `row` of a comb for the signed digit of y (comb_recode'd scalar).
template <int W, class T>
__device__ void comb_row_point(ge_p3& P, const uint32_t y[9], int row, const T& tab) {
  const int e = comb_digit<W>(y, row);
  ge_niels nb;
  tab.load(row, (e < 0 ? -e : e) - 1, nb);
  comb_set_entry<kSO>(P, nb, e);
}

// libsodium's frombytes of R (ge_frombytes, negate = false) cut in two at a
// point of its exponentiation, so the first ~145 products run beside the hash
// and the rest beside the key comb's tree: part 1 leaves u = y^2 - 1,
// v = d y^2 + 1, v3 = v^3, t0, t1 and t2 = t1^(2^30) of fe_pow22523(u v^7).
struct RDecode {
  fe y, u, v, v3, t0, t1, t2;
};
__device__ void r_decode_part1(RDecode& d, const uint32_t s[8]) {
  fe one, x, z;
  fe_1(one);
  fe_frombytes(d.y, s);
  fe_sq_o<kSO>(d.u, d.y);
  fe_mul_o<kSO>(d.v, d.u, fe_const_d());
  fe_sub(d.u, d.u, one);
  fe_carry(d.u);
  fe_add(d.v, d.v, one);
  fe_sq_o<kSO>(d.v3, d.v);
  fe_mul_o<kSO>(d.v3, d.v3, d.v);
  fe_sq_o<kSO>(x, d.v3);
  fe_mul_o<kSO>(x, x, d.v);
  fe_mul_o<kSO>(z, x, d.u);  // u v^7: fe_pow22523's input, its chain up to t1 = z^(2^100 - 1) then 30 squarings
  fe_sq_o<kSO>(d.t0, z);
  fe_sqn<kSO>(d.t1, d.t0, 2);
  fe_mul_o<kSO>(d.t1, z, d.t1);
  fe_mul_o<kSO>(d.t0, d.t0, d.t1);
  fe_sq_o<kSO>(d.t0, d.t0);
  fe_mul_o<kSO>(d.t0, d.t1, d.t0);
  fe_sqn<kSO>(d.t1, d.t0, 5);
  fe_mul_o<kSO>(d.t0, d.t1, d.t0);
  fe_sqn<kSO>(d.t1, d.t0, 10);
  fe_mul_o<kSO>(d.t1, d.t1, d.t0);
  fe_sqn<kSO>(d.t2, d.t1, 20);
  fe_mul_o<kSO>(d.t1, d.t2, d.t1);
  fe_sqn<kSO>(d.t1, d.t1, 10);
  fe_mul_o<kSO>(d.t0, d.t1, d.t0);
  fe_sqn<kSO>(d.t1, d.t0, 50);
  fe_mul_o<kSO>(d.t1, d.t1, d.t0);
  fe_sqn<kSO>(d.t2, d.t1, 30);
}
// The rest: x of R with R's sign (false: no square root).  Same value as ge_frombytes.
__device__ bool r_decode_part2(fe& x, RDecode& d, const uint32_t s[8]) {
  fe_sqn<kSO>(d.t2, d.t2, 70);
  fe_mul_o<kSO>(d.t1, d.t2, d.t1);
  fe_sqn<kSO>(d.t1, d.t1, 50);
  fe_mul_o<kSO>(d.t0, d.t1, d.t0);
  fe_sqn<kSO>(d.t0, d.t0, 2);
  fe z;
  fe_sq_o<kSO>(x, d.v3);
  fe_mul_o<kSO>(x, x, d.v);
  fe_mul_o<kSO>(z, x, d.u);
  fe_mul_o<kSO>(x, d.t0, z);  // (u v^7)^((p-5)/8)
  fe_mul_o<kSO>(x, x, d.v3);
  fe_mul_o<kSO>(x, x, d.u);   // u v^3 (u v^7)^((p-5)/8)
  fe vxx, chk;
  fe_sq_o<kSO>(vxx, x);
  fe_mul_o<kSO>(vxx, vxx, d.v);
  fe_sub(chk, vxx, d.u);
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, d.u);
    if (!fe_iszero(chk)) return false;
    fe_mul_o<kSO>(x, x, fe_const_sqrtm1());
  }
  if (fe_isnegative(x) != (s[7] >> 31)) {
    fe_neg(x, x);
    fe_carry(x);
  }
  return true;
}

// The same decode with fe_pow22523's chain spread over wave 2's lanes (fe_lanes.h): lane 0 runs
// the few products before and after it, every lane of the wave the chain.  EDV_SMALL_LANES=0: the
// one-lane chain above (A/B).
#ifndef EDV_SMALL_LANES
#define EDV_SMALL_LANES 1
#endif
// EDV_SMALL_DIST_EDGES 1 (default): the products before the chain (u, v, v^3, u v^7) and after it
// (x, v x^2) distributed too -- ~0.17 us each on the wave against ~0.37 us on lane 0 -- with u - 1
// formed as u + 2p - 1 and carried back into the dist_* input bounds; 0: on lane 0 (A/B).
#ifndef EDV_SMALL_DIST_EDGES
#define EDV_SMALL_DIST_EDGES 1
#endif
struct RDecodeL {
  fe y, u, v, v3, uv7;      // lane 0 (EDV_SMALL_DIST_EDGES 0); y in every lane
  uint32_t t0, t1, t2;      // distributed (limb k in lane k)
  uint32_t du, dv, dv3, duv7;  // distributed (EDV_SMALL_DIST_EDGES 1)
};
// limb k of a lane-uniform fe in lane k (every lane holds f; no cross-lane moves)
__device__ __forceinline__ uint32_t dist_pick(const fe& f, uint32_t k) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) r = k == (uint32_t)i ? f.v[i] : r;
  return r;
}
__device__ void r_decode_part1_lanes(RDecodeL& d, const uint32_t s[8], uint32_t lane) {
  fe z;
  fe_0(z);
#if EDV_SMALL_DIST_EDGES
  const uint32_t k = lane & 15;
  const LaneTerms sq = c_lane_sq.t[lane], mu = c_lane_mul.t[lane];
  fe_frombytes(d.y, s);  // (every lane: the same words)
  const bool row0 = lane < 10;
  const uint32_t yd = dist_form(k < 10 ? dist_pick(d.y, k) : 0u, lane);
  const uint32_t y2 = dist_sq(yd, sq, lane);
  // v = d y^2 + 1 (limb 0 of a dist_* output < 2^26: the + 1 stays in bounds)
  const uint32_t dd = dist_form(k < 10 ? dist_pick(fe_const_d(), k) : 0u, lane);
  d.dv = dist_mul(y2, dd, mu, lane) + dist_form(k == 0 ? 1u : 0u, lane);
  // u = y^2 - 1 = y^2 + 2p - 1, carried: limbs of 2p are 2^27 - 38, then 2^26 - 2 / 2^27 - 2
  const uint32_t two_p = k == 0 ? (1u << 27) - 38 : (k & 1) ? (1u << 26) - 2 : (1u << 27) - 2;
  d.du = lane_cols_carry(row0 ? (uint64_t)y2 + two_p - (lane == 0 ? 1u : 0u) : 0ull, lane);
  d.dv3 = dist_mul(dist_sq(d.dv, sq, lane), d.dv, mu, lane);
  d.duv7 = dist_mul(dist_mul(dist_sq(d.dv3, sq, lane), d.dv, mu, lane), d.du, mu, lane);  // u v^7
  const uint32_t zd = d.duv7;
#else
  if (lane == 0) {
    fe one, x;
    fe_1(one);
    fe_frombytes(d.y, s);
    fe_sq_o<kSO>(d.u, d.y);
    fe_mul_o<kSO>(d.v, d.u, fe_const_d());
    fe_sub(d.u, d.u, one);
    fe_carry(d.u);
    fe_add(d.v, d.v, one);
    fe_sq_o<kSO>(d.v3, d.v);
    fe_mul_o<kSO>(d.v3, d.v3, d.v);
    fe_sq_o<kSO>(x, d.v3);
    fe_mul_o<kSO>(x, x, d.v);
    fe_mul_o<kSO>(z, x, d.u);  // u v^7
    d.uv7 = z;                 // (part 2 needs it again)
  }
  const uint32_t k = lane & 15;
  const LaneTerms sq = c_lane_sq.t[lane], mu = c_lane_mul.t[lane];
  const uint32_t zd = dist_from_lane0(z, lane);
#endif
  uint32_t t0 = dist_sq(zd, sq, lane);
  uint32_t t1 = dist_sqn(t0, 2, sq, lane);
  t1 = dist_mul(zd, t1, mu, lane);
  t0 = dist_mul(t0, t1, mu, lane);
  t0 = dist_sq(t0, sq, lane);
  t0 = dist_mul(t1, t0, mu, lane);
  t1 = dist_sqn(t0, 5, sq, lane);
  t0 = dist_mul(t1, t0, mu, lane);
  t1 = dist_sqn(t0, 10, sq, lane);
  t1 = dist_mul(t1, t0, mu, lane);
  uint32_t t2 = dist_sqn(t1, 20, sq, lane);
  t1 = dist_mul(t2, t1, mu, lane);
  t1 = dist_sqn(t1, 10, sq, lane);
  t0 = dist_mul(t1, t0, mu, lane);
  t1 = dist_sqn(t0, 50, sq, lane);
  t1 = dist_mul(t1, t0, mu, lane);
  d.t2 = dist_sqn(t1, 30, sq, lane);
  d.t0 = t0;
  d.t1 = t1;
}
// every lane of the wave calls; lane 0's x and result are r_decode_part2's
__device__ bool r_decode_part2_lanes(fe& x, RDecodeL& d, const uint32_t s[8], uint32_t lane) {
  const LaneTerms sq = c_lane_sq.t[lane], mu = c_lane_mul.t[lane];
  uint32_t t2 = dist_sqn(d.t2, 70, sq, lane);
  uint32_t t1 = dist_mul(t2, d.t1, mu, lane);
  t1 = dist_sqn(t1, 50, sq, lane);
  uint32_t t0 = dist_mul(t1, d.t0, mu, lane);
  t0 = dist_sqn(t0, 2, sq, lane);
  fe vxx, chk;
#if EDV_SMALL_DIST_EDGES
  // x = u v^3 (u v^7)^((p-5)/8), then v x^2, on the wave; lane 0 takes x, v x^2 and u
  uint32_t xd = dist_mul(dist_mul(dist_mul(t0, d.duv7, mu, lane), d.dv3, mu, lane), d.du, mu, lane);
  const uint32_t vxxd = dist_mul(dist_sq(xd, sq, lane), d.dv, mu, lane);
  fe u;
  dist_to_fe(x, xd);  // class C, in every lane
  dist_to_fe(vxx, vxxd);
  dist_to_fe(u, d.du);
  if (lane != 0) return false;
  fe_sub(chk, vxx, u);
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, u);
    if (!fe_iszero(chk)) return false;
    fe_mul_o<kSO>(x, x, fe_const_sqrtm1());
  }
  if (fe_isnegative(x) != (s[7] >> 31)) {
    fe_neg(x, x);
    fe_carry(x);
  }
  return true;
#else
  fe pw;
  dist_to_fe(pw, t0);  // (u v^7)^((p-5)/8), class C, in every lane
  if (lane != 0) return false;
  fe_mul_o<kSO>(x, pw, d.uv7);
  fe_mul_o<kSO>(x, x, d.v3);
  fe_mul_o<kSO>(x, x, d.u);   // u v^3 (u v^7)^((p-5)/8)
  fe_sq_o<kSO>(vxx, x);
  fe_mul_o<kSO>(vxx, vxx, d.v);
  fe_sub(chk, vxx, d.u);
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, d.u);
    if (!fe_iszero(chk)) return false;
    fe_mul_o<kSO>(x, x, fe_const_sqrtm1());
  }
  if (fe_isnegative(x) != (s[7] >> 31)) {
    fe_neg(x, x);
    fe_carry(x);
  }
  return true;
#endif
}

// verify_phase_hash for the single-request kernel: SHA-512(R || A || M) with the blocks' message
// schedules on wave 0's lanes (lane j: block p0 + j of a pass of kHashPass blocks, its 80 words
// into LDS) and only the rounds on lane 0 -- the schedule is ~35 % of a round's instructions, and
// on one lane every instruction is on the critical path.  Every lane of the wave calls; lane 0's
// h and result are verify_phase_hash's.  EDV_SMALL_HASH_LANES=0: verify_phase_hash on lane 0 (A/B).
#ifndef EDV_SMALL_HASH_LANES
#define EDV_SMALL_HASH_LANES 1
#endif
constexpr int kHashPass = 8;
constexpr int kHashRow = 81;  // u64 per block row (odd: the lanes' rows start in different banks)
__device__ __forceinline__ void sha512_schedule_lds(uint64_t* out, uint64_t w[16]) {
#pragma unroll
  for (int t = 0; t < 16; ++t) out[t] = w[t];
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
      w[i] += s0 + w[(i + 9) & 15] + s1;
      out[r + i] = w[i];
    }
  }
}
__device__ __forceinline__ void sha512_rounds_lds(uint64_t st[8], const uint64_t* w) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
      const uint64_t ch = bitop3_64<0xca>(e, f, g);
      const uint64_t t1 = h + S1 + ch + SHA512_K[r + i] + w[r + i];
      const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
      const uint64_t mj = bitop3_64<0xe8>(a, b, c);
      h = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + S0 + mj;
    }
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}
__device__ bool verify_phase_hash_lanes(uint32_t hout[8], const uint32_t sig[16], const uint32_t pk[8],
                                        const uint8_t* msg, uint64_t mlen, uint32_t lane, uint64_t* sw) {
  constexpr int NP = 16;
  uint32_t prefix[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    prefix[k] = sig[k];
    prefix[8 + k] = pk[k];
  }
  const uint64_t total = 4 * NP + mlen, nblocks = (total + 16) / 128 + 1, bitlen = total * 8;
  const uint32_t d16 = (uint32_t)((uintptr_t)msg & 15);
  const Chunk16* c16 = (const Chunk16*)(msg - d16);
  const uint64_t nq = (d16 + mlen + 15) / 16;
  uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
#pragma unroll 1
  for (uint64_t p0 = 0; p0 < nblocks; p0 += kHashPass) {
    const uint64_t b = p0 + lane;
    if (lane < (uint32_t)kHashPass && b < nblocks) {
      uint64_t w[16];
      if (b == 0)
        sha512_block_words<NP, true>(w, 0, prefix, c16, nq, d16, mlen);
      else
        sha512_block_words<NP, false>(w, b, prefix, c16, nq, d16, mlen);
      if (b == nblocks - 1) {
        w[14] = 0;
        w[15] = bitlen;
      }
      sha512_schedule_lds(sw + lane * kHashRow, w);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
      const uint64_t nb = nblocks - p0 < (uint64_t)kHashPass ? nblocks - p0 : (uint64_t)kHashPass;
#pragma unroll 1
      for (uint64_t j = 0; j < nb; ++j) sha512_rounds_lds(st, sw + j * kHashRow);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next pass overwrites sw
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (lane != 0) return false;
  uint32_t digest[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    digest[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    digest[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
  const uint32_t* S = sig + 8;
  const bool ok = sc_is_canonical(S) && !has_small_order(sig) && is_canonical_point(pk) && !has_small_order(pk);
  sc_reduce(hout, digest);
  return ok;
}

constexpr int kSmallThreads = 192;
// EDV_SMALL_PROFILE=1 (probe builds only, tools/small_probe.py): the wall clock (100 MHz) at the
// phase boundaries of request 0, read back with edv_small_profile.
#ifndef EDV_SMALL_PROFILE
#define EDV_SMALL_PROFILE 0
#endif
#if EDV_SMALL_PROFILE
__device__ unsigned long long g_small_prof[10];  // [8], [9]: the shader clock at stamps 0 and 7
#define EDV_SP(k)                                                   \
  do {                                                              \
    if (blockIdx.x == 0 && lane == 0) g_small_prof[k] = wall_clock64(); \
  } while (0)
#else
#define EDV_SP(k) \
  do {            \
  } while (0)
#endif
struct SmallShared {
  uint64_t sw[kHashPass * kHashRow];  // wave 0's message schedules (verify_phase_hash_lanes)
  uint32_t h[8];
  uint32_t xr[10];  // R decoded (wave 2; its y: wave 0 reads the bytes itself)
  uint32_t base[40];        // [S]B (wave 1): X, Y, Z, T
  int ok_hash, ok_r;
};
// One request's verify on a 192-thread workgroup (every thread calls, with the request's signature
// words loaded): wave 0 hashes, then sums the key comb's rows on its lanes; wave 1 sums the base
// comb's rows; wave 2 decodes R; the verdict is returned on thread 0 (false elsewhere).  The body
// of edv_verify_small_kernel (one workgroup per request) and of edv_resident_kernel (one
// workgroup serving request after request).
template <int W>
__device__ __forceinline__ bool small_verify(SmallShared& sh, const uint32_t sig[16], uint32_t key0, uint32_t key_count,
                                             const uint8_t* __restrict__ key_pk, const uint8_t* __restrict__ key_valid,
                                             const uint8_t* msg, uint64_t mlen, const uint32_t* __restrict__ key_tab,
                                             uint64_t key_cap, const uint32_t* __restrict__ btab,
                                             const uint32_t* __restrict__ ident) {
  constexpr int RK = Window<W>::kRows, RB = Window<kBaseW>::kRows;
  static_assert(RK <= 64 && RB <= 64, "one lane per row");
  constexpr int WK = RK <= 16 ? 16 : RK <= 32 ? 32 : 64, WB = RB <= 16 ? 16 : RB <= 32 ? 32 : 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#if EDV_SMALL_LANES
  RDecodeL rd;  // wave 2: R's decode, across the first barrier
#else
  RDecode rd;  // wave 2, lane 0: R's decode, across the first barrier
#endif
  const bool in_range = key0 < key_count;
  const uint64_t key = in_range ? key0 : 0;
  if (wave == 0) EDV_SP(0);
  if (wave == 0) {
#if EDV_SMALL_HASH_LANES
    uint32_t pk[8], h[8];
    load_words(pk, key_pk + 32 * key, 8);
    const bool hok = verify_phase_hash_lanes(h, sig, pk, msg, mlen, (uint32_t)lane, sh.sw);
    if (lane == 0) {
      const bool ok = hok && in_range && key_valid[key];
#else
    if (lane == 0) {
      uint32_t pk[8], h[8];
      load_words(pk, key_pk + 32 * key, 8);
      const bool ok = verify_phase_hash(h, sig, pk, msg, mlen) && in_range && key_valid[key];
#endif
#pragma unroll
      for (int k = 0; k < 8; ++k) sh.h[k] = h[k];
      sh.ok_hash = ok ? 1 : 0;
    }
    EDV_SP(1);
  } else if (wave == 1) {
    uint32_t y[9];
    comb_recode<kBaseW>(y, sig + 8);
    ge_p3 P;
    if (lane < RB) {
      const DevComb<kBaseW> tb{btab, ident};
      comb_row_point<kBaseW>(P, y, lane, tb);
    } else {
      ge_p3_0(P);
    }
    lane_tree_sum(P, lane, WB);
    if (lane == 0) {
      store_fe(sh.base, P.X);
      store_fe(sh.base + 10, P.Y);
      store_fe(sh.base + 20, P.Z);
      store_fe(sh.base + 30, P.T);
    }
    EDV_SP(2);
  } else {
#if EDV_SMALL_LANES
    r_decode_part1_lanes(rd, sig, (uint32_t)lane);
#else
    if (lane == 0) r_decode_part1(rd, sig);
#endif
    EDV_SP(3);
  }
  __syncthreads();
  if (wave == 2) {
    fe x;
#if EDV_SMALL_LANES
    const bool dec = r_decode_part2_lanes(x, rd, sig, (uint32_t)lane);  // false: no root (lane 0)
#endif
    if (lane == 0) {
#if !EDV_SMALL_LANES
      const bool dec = r_decode_part2(x, rd, sig);  // false: y^2 - 1 / (d y^2 + 1) has no root
#endif
      const bool zero_signed = (sig[7] >> 31) && fe_iszero(x);
      store_fe(sh.xr, x);
      sh.ok_r = (dec && is_canonical_point(sig) && !zero_signed) ? 1 : 0;
      EDV_SP(5);
    }
  }
  ge_p3 P;
  if (wave == 0) {  // [h](-A): the key comb's rows on lanes, summed as a tree
    EDV_SP(4);
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = sh.h[k];
    uint32_t y[9];
    comb_recode<W>(y, h);
    if (lane < RK) {
      constexpr uint64_t kRowWordsW = (uint64_t)Window<W>::kEntries * kEntryWords;
      const DevComb<W> ta{key_tab + key * kRowWordsW, ident, key_cap * kRowWordsW};  // row-major store
      comb_row_point<W>(P, y, lane, ta);
    } else {
      ge_p3_0(P);
    }
    lane_tree_sum(P, lane, WK);
    EDV_SP(6);
  }
  ge_p2 Q;
  bool ok_y = false;
  if (wave == 0 && lane == 0) {  // R' while wave 2 still decodes R ([S]B is in LDS since the first barrier)
    ge_p3 B;
    load_fe(B.X, sh.base);
    load_fe(B.Y, sh.base + 10);
    load_fe(B.Z, sh.base + 20);
    load_fe(B.T, sh.base + 30);
    ge_cached c;
    ge_p1p1 t;
    ge_p3_to_cached<kSO>(c, B);
    ge_add<kSO>(t, P, c);
    ge_p1p1_to_p2_addlike<kSO>(Q, t);  // R' = [h](-A) + [S]B, classes C
    // Y' = y_R Z' needs only R's bytes (y_R as r_decode reads it): checked here, while wave 2 still
    // decodes, so one product follows the last barrier, not two
    fe yr, u, d;
    fe_frombytes(yr, sig);
    fe_mul_o<kSO>(u, yr, Q.Z);
    fe_sub(d, Q.Y, u);
    ok_y = fe_iszero(d);
  }
  __syncthreads();  // R's decode (wave 2) done
  if (wave != 0 || lane != 0) return false;
  fe xr, u, d;
  load_fe(xr, sh.xr);
  fe_mul_o<kSO>(u, xr, Q.Z);
  fe_sub(d, Q.X, u);  // X' - x_R Z'  (L)
  const bool ok = ok_y && sh.ok_hash && sh.ok_r && fe_iszero(d);
  EDV_SP(7);
#if EDV_SMALL_PROFILE
  if (blockIdx.x == 0) g_small_prof[9] = __builtin_amdgcn_s_memtime();
#endif
  return ok;
}


template <int W>
__global__ __launch_bounds__(kSmallThreads) void edv_verify_small_kernel(
    const uint8_t* __restrict__ sig64, const uint32_t* __restrict__ key_idx, uint32_t key_count,
    const uint8_t* __restrict__ key_pk, const uint8_t* __restrict__ key_valid, const uint8_t* __restrict__ msgs,
    const uint64_t* __restrict__ ms, const uint64_t* __restrict__ me, uint64_t n,
    const uint32_t* __restrict__ key_tab, uint64_t key_cap, const uint32_t* __restrict__ btab,
    const uint32_t* __restrict__ ident, uint8_t* __restrict__ ok8) {
  __shared__ SmallShared sh;
  const uint64_t i = blockIdx.x;
  if (i >= n) return;  // block-uniform
#if EDV_SMALL_PROFILE
  if (blockIdx.x == 0 && threadIdx.x == 0) g_small_prof[8] = __builtin_amdgcn_s_memtime();
#endif
  uint32_t sig[16];
  load_words(sig, sig64 + 64 * i, 16);
  const bool ok = small_verify<W>(sh, sig, key_idx[i], key_count, key_pk, key_valid, msgs + ms[i], me[i] - ms[i],
                                  key_tab, key_cap, btab, ident);
  if (threadIdx.x == 0) ok8[i] = ok ? 1 : 0;
}

// ---------------------------------------------------------------- resident single-request kernel
// edv_verify_one: one authenticate() that missed the verify-ahead cache.  Launching a kernel, copying
// its inputs and waiting for its completion cost ~16 us around a ~52 us edv_verify_small_kernel; here
// one workgroup stays resident and takes requests from a mailbox in fine-grained pinned host memory:
// the host writes the request and then its number (req_seq); thread 0 polls req_seq with
// system-scope loads, the workgroup copies the request into LDS, runs small_verify, and thread 0
// writes the verdict and then done_seq with system-scope stores the host spins on.  It exits when
// the host sets `stop` (every other library call that queues GPU work does: the stream it runs on may
// share a hardware queue with theirs) or after idle_ticks of the 100 MHz wall clock without a
// request, and clears `running` as it leaves -- so the grid always drains, whatever the host does.
constexpr uint64_t kResMsgMax = 4096;  // longer messages take the launch path
struct ResBox {
  uint64_t req_seq;   // host: the request's number, stored after its fields
  uint64_t stop;      // host: 1 = exit at the next poll
  uint64_t done_seq;  // kernel: the last request verified, stored after its verdict
  uint32_t verdict;   // kernel
  uint32_t running;   // host: 1 at launch; kernel: 0 as it exits
  uint64_t mlen;
  uint32_t key_id, key_count;
  const uint32_t* key_tab;
  const uint8_t* key_pk;
  const uint8_t* key_valid;
  uint64_t key_cap;
  uint64_t service_ticks;  // kernel: 100 MHz wall-clock ticks from seeing the request to its verdict (diagnostic)
  uint64_t pad[5];
  uint8_t sig[64];
  uint8_t msg[kResMsgMax];
};
static_assert(offsetof(ResBox, sig) % 64 == 0, "sig 64-byte aligned");
static_assert(offsetof(ResBox, key_id) == offsetof(ResBox, mlen) + 8 && offsetof(ResBox, key_tab) == offsetof(ResBox, mlen) + 16 &&
                  offsetof(ResBox, key_cap) == offsetof(ResBox, mlen) + 40,
              "the kernel loads mlen .. key_cap as six consecutive words");
struct alignas(16) ResShared {
  uint64_t seq, t_seen;
  uint64_t field[6];  // ResBox's mlen .. key_cap, as loaded
  uint32_t cmd, pad;
  uint32_t sig[16];
  uint64_t msg[kResMsgMax / 8 + 2];
};
__device__ __forceinline__ uint64_t sys_load64_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int W>
__global__ __launch_bounds__(kSmallThreads) void edv_resident_kernel(ResBox* box, const uint32_t* __restrict__ btab,
                                                                     const uint32_t* __restrict__ ident,
                                                                     uint64_t idle_ticks) {
  __shared__ SmallShared sh;
  __shared__ ResShared rs;
  const uint32_t t = threadIdx.x;
  uint64_t last = 0;
  if (t == 0) last = sys_load64_relaxed(&box->done_seq);
  for (;;) {
    if (t == 0) {
      const uint64_t t0 = wall_clock64();
      uint32_t cmd = 0;
      uint64_t seq = last;
      for (;;) {
        // relaxed: an acquire here would invalidate this XCD's L2 on every poll, under whatever
        // kernels share it; the one acquire follows the change
        seq = sys_load64_relaxed(&box->req_seq);
        if (seq != last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the request's fields after its number
          cmd = 1;
          break;
        }
        if (sys_load64_relaxed(&box->stop) || wall_clock64() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(1);
      }
      rs.cmd = cmd;
      rs.seq = seq;
      rs.t_seen = wall_clock64();
    }
    __syncthreads();
    if (!rs.cmd) break;  // workgroup-uniform
    // the request into LDS in one PCIe round trip: its fields (threads 0-5), signature (8-15) and the
    // first kResHead message words (16 ..) are loaded side by side, each an 8-byte system-scope load
    // (serially, thread 0's six field loads alone took ~10 us); a longer message's rest follows
    constexpr uint32_t kResHead = kSmallThreads - 16;
    if (t < 6) {
      const uint64_t* f = (const uint64_t*)&box->mlen;  // mlen, key_id | key_count, key_tab, key_pk, key_valid, key_cap
      rs.field[t] = sys_load64_relaxed(f + t);
    } else if (t >= 8 && t < 16) {
      const uint64_t v = sys_load64_relaxed((const uint64_t*)box->sig + (t - 8));
      rs.sig[2 * (t - 8)] = (uint32_t)v;
      rs.sig[2 * (t - 8) + 1] = (uint32_t)(v >> 32);
    } else if (t >= 16) {
      rs.msg[t - 16] = sys_load64_relaxed((const uint64_t*)box->msg + (t - 16));
    }
    __syncthreads();
    const uint64_t mlen = rs.field[0] < kResMsgMax ? rs.field[0] : kResMsgMax;  // (the host never sends more)
    const uint64_t nw = (mlen + 7) / 8;
    for (uint64_t w = kResHead + t; w < nw; w += kSmallThreads)
      rs.msg[w] = sys_load64_relaxed((const uint64_t*)box->msg + w);
    if (t < 2) rs.msg[nw + t] = 0;  // (the hash's last chunk load reads past the message)
    // key tables rebuilt since the last request (an eviction's build, finished before the host sent
    // this request) must not be read from this CU's or this XCD's stale cache lines
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __syncthreads();
    uint32_t sig[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) sig[k] = rs.sig[k];
    const bool ok = small_verify<W>(sh, sig, (uint32_t)rs.field[1], (uint32_t)(rs.field[1] >> 32),
                                    (const uint8_t*)rs.field[3], (const uint8_t*)rs.field[4], (const uint8_t*)rs.msg,
                                    mlen, (const uint32_t*)rs.field[2], rs.field[5], btab, ident);
    if (t == 0) {
      __hip_atomic_store(&box->service_ticks, wall_clock64() - rs.t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&box->verdict, ok ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&box->done_seq, rs.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      last = rs.seq;
    }
    __syncthreads();  // rs and sh are the next request's
  }
  if (t == 0) __hip_atomic_store(&box->running, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Fixed-base comb: [x]B with x < 2^253, 64 madds over BASE_COMB (global).
__device__ void ge_scalarmult_base(ge_p3& Q, const uint32_t x[8], const uint32_t* __restrict__ comb) {
  uint32_t y[8];
  sc_recode16(y, x);
  ge_p3_0(Q);
  ge_p1p1 t;
  for (int i = 0; i < 64; ++i) {
    const int e = recode_digit(y, i);
    const int m = e < 0 ? -e : e;
    ge_niels nb;
    ge_niels_0(nb);
    if (m != 0) {
      const uint32_t* p = comb + (uint64_t)(i * 8 + m - 1) * 30;
#pragma unroll
      for (int l = 0; l < 10; ++l) {
        nb.ypx.v[l] = p[l];
        nb.ymx.v[l] = p[10 + l];
        nb.xy2d.v[l] = p[20 + l];
      }
    }
    if (e < 0) {
      fe tmp = nb.ypx;
      nb.ypx = nb.ymx;
      nb.ymx = tmp;
      fe_neg(nb.xy2d, nb.xy2d);
    }
    ge_madd(t, Q, nb);
    ge_p1p1_to_p3_addlike(Q, t);
  }
}

__device__ void clamp_reduce(uint32_t a_red[8], uint32_t a_clamped[8], const uint32_t az[16]) {
  uint32_t wide[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) a_clamped[k] = az[k];
  a_clamped[0] &= ~7u;
  a_clamped[7] &= 0x3fffffffu;
  a_clamped[7] |= 0x40000000u;
#pragma unroll
  for (int k = 0; k < 16; ++k) wide[k] = k < 8 ? a_clamped[k] : 0u;
  sc_reduce(a_red, wide);
}

__global__ __launch_bounds__(kBlock) void edv_keypair_kernel(const uint8_t* __restrict__ seeds, uint64_t n,
                                                            const uint32_t* __restrict__ comb,
                                                            uint8_t* __restrict__ pk_out, uint8_t* __restrict__ sk_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8], az[16], a_red[8], a_cl[8], pk[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) seed[k] = ((const uint32_t*)(seeds + 32 * i))[k];
  sha512_prefixed<8>(az, seed, nullptr, 0);
  clamp_reduce(a_red, a_cl, az);
  ge_p3 A;
  ge_scalarmult_base(A, a_red, comb);
  ge_p2 a2;
  ge_p3_to_p2(a2, A);
  ge_tobytes(pk, a2);
  uint32_t* po = (uint32_t*)(pk_out + 32 * i);
  uint32_t* so = (uint32_t*)(sk_out + 64 * i);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    po[k] = pk[k];
    so[k] = seed[k];
    so[8 + k] = pk[k];
  }
}

__global__ __launch_bounds__(kBlock) void edv_sign_kernel(const uint8_t* __restrict__ sk64,
                                                         const uint32_t* __restrict__ key_idx,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ ms,
                                                         const uint64_t* __restrict__ me, uint64_t n,
                                                         const uint32_t* __restrict__ comb,
                                                         uint8_t* __restrict__ sig_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* sk = (const uint32_t*)(sk64 + 64 * (uint64_t)key_idx[i]);
  uint32_t seed[8], pk[8], az[16], a_red[8], a_cl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    seed[k] = sk[k];
    pk[k] = sk[8 + k];
  }
  const uint8_t* m = msgs + ms[i];
  const uint64_t mlen = me[i] - ms[i];
  sha512_prefixed<8>(az, seed, nullptr, 0);
  clamp_reduce(a_red, a_cl, az);
  uint32_t nonce_full[16], nonce[8];
  sha512_prefixed<8>(nonce_full, az + 8, m, mlen);
  sc_reduce(nonce, nonce_full);
  ge_p3 R;
  ge_scalarmult_base(R, nonce, comb);
  ge_p2 r2;
  ge_p3_to_p2(r2, R);
  uint32_t rb[8];
  ge_tobytes(rb, r2);
  uint32_t prefix[16], hram_full[16], hram[8], s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    prefix[k] = rb[k];
    prefix[8 + k] = pk[k];
  }
  sha512_prefixed<16>(hram_full, prefix, m, mlen);
  sc_reduce(hram, hram_full);
  sc_muladd(s, hram, a_cl, nonce);
  uint32_t* so = (uint32_t*)(sig_out + 64 * i);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    so[k] = rb[k];
    so[8 + k] = s[k];
  }
}

// Request digests (request.py:51-52): SHA-256 of each message span.
__global__ __launch_bounds__(kBlock) void edv_sha256_kernel(const uint8_t* __restrict__ msgs,
                                                           const uint64_t* __restrict__ ms,
                                                           const uint64_t* __restrict__ me, uint64_t n,
                                                           uint8_t* __restrict__ out32) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t d[8];
  sha256_msg(d, msgs + ms[i], me[i] - ms[i]);
  uint4* o = (uint4*)(out32 + 32 * i);
  o[0] = make_uint4(d[0], d[1], d[2], d[3]);
  o[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// Replica.validatePrepare (plenum/server/replica.py:1289-1291): a PREPARE from
// the primary of its key's view is rejected (SuspiciousNode) before it reaches
// Prepares.addVote, so it never counts.  primary[k] = that voter (0xff: none).
__global__ void edv_tally_scatter_kernel(const uint32_t* __restrict__ key, const uint8_t* __restrict__ voter,
                                         const uint8_t* __restrict__ phase, const uint8_t* __restrict__ valid,
                                         const uint8_t* __restrict__ primary, uint64_t n_votes, uint32_t n_keys,
                                         uint32_t n_validators, uint8_t* __restrict__ ballot) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_votes) return;
  const uint32_t k = key[i], v = voter[i], ph = phase[i];
  if (!valid[i] || k >= n_keys || v >= n_validators || ph >= 2) return;
  if (ph == 0 && primary && primary[k] == v) return;
  ballot[((uint64_t)k * 2 + ph) * n_validators + v] = 1;
}

__global__ void edv_tally_count_kernel(const uint8_t* __restrict__ ballot, uint32_t n_keys, uint32_t n_validators,
                                       uint32_t q_prepare, uint32_t q_commit, uint32_t* __restrict__ counts,
                                       uint8_t* __restrict__ quorum) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_keys) return;
  uint32_t c[2] = {0, 0};
  for (int ph = 0; ph < 2; ++ph) {
    const uint8_t* b = ballot + (k * 2 + ph) * n_validators;
    for (uint32_t v = 0; v < n_validators; ++v) c[ph] += b[v] != 0;
  }
  counts[2 * k] = c[0];
  counts[2 * k + 1] = c[1];
  quorum[k] = (uint8_t)((c[0] >= q_prepare ? 1 : 0) | (c[1] >= q_commit ? 2 : 0));
}

uint64_t div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// Auto length buckets (edv_options.length_buckets = 2) for calls whose offsets
// are on the host: sort the hash lanes when unsorted waves would run more than
// 1.25x the batch's SHA-512 blocks (each wave runs its longest message's
// block count on all 64 lanes).  Uniform batches (configs[1]: 147-149 B, all
// 2 blocks) skip the sort's launches.
bool lengths_mixed(const uint64_t* off, uint64_t n) {
  uint64_t sum = 0, padded = 0;
  for (uint64_t g = 0; g < n; g += 64) {
    const uint64_t e = g + 64 < n ? g + 64 : n;
    uint64_t mx = 0;
    for (uint64_t i = g; i < e; ++i) {
      const uint64_t b = (off[i + 1] - off[i] + 64 + 17 + 127) / 128;
      sum += b;
      mx = b > mx ? b : mx;
    }
    padded += mx * (e - g);
  }
  return 4 * padded > 5 * sum;
}

}  // namespace

// ------------------------------------------------------------------ context

struct edv_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t* d_btab_comb = nullptr;    // W = 4 base comb (signer / keypair)
  uint32_t* d_scratch = nullptr;  // per-lane A tables, kMaxLanes / kBlock regions
  uint32_t* d_hsoa = nullptr;     // h words, SoA [8][kMaxLanes]
  uint8_t* d_flags = nullptr;     // precheck / decode verdicts [kMaxLanes]
  uint32_t* d_pt = nullptr;       // R' = (X:Y:Z), SoA [30][kMaxLanes]
  uint32_t* d_pre = nullptr;      // batch-encode prefix products, SoA [10][kMaxLanes]
  uint32_t* d_perm = nullptr;     // length-bucket order of the hash lanes [kMaxLanes]
  uint8_t* d_lenkey = nullptr;    // block-count keys, in | sorted [2][kMaxLanes]
  // general-path key dedupe (per sub-batch at its lane offset): hash slots
  // [2][kMaxLanes] (2 per lane), slot -> key index [2][kMaxLanes], request ->
  // slot, key index -> representative request [kMaxLanes] each; key_ok
  // [kMaxLanes]; distinct-key counts [kSub]
  uint32_t* d_dedup = nullptr;
  uint8_t* d_key_ok = nullptr;
  uint32_t* d_ucount = nullptr;
  void* d_sort_tmp = nullptr;     // radix-sort temporary storage, one slot per sub-batch
  size_t sort_tmp_bytes = 0;      // per slot (sized for kMaxLanes)
  int bucket_mode = 2;            // edv_options.length_buckets: 0 off, 1 on, 2 auto, 3 on + packed units
  bool bucket_now = false;        // this launch sorts its hash lanes
  bool pack_now = false;          // ... and packs the messages into the unit arena (mode 3)
  // packed message layout (mode 3): per-group units and offsets
  // [kMaxLanes / 64 + 1] each, the scan's temporary storage, the arena
  uint64_t* d_gunits = nullptr;
  uint64_t* d_goff = nullptr;
  void* d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  Chunk16* d_arena = nullptr;
  uint64_t arena_units = 0;                  // allocated
  uint64_t arena_want = kMaxLanes * 80ull;   // edv_options.unit_arena_bytes (1.25 GiB: 1,280 B per lane)
  uint64_t scratch_lanes = 0;
  // Pipelined launches: each chunk of up to kMaxLanes requests is cut into
  // kSub sub-batches whose kernels alternate between `stream` (or the
  // caller's) and `stream2`, so one sub-batch's encode (a latency-bound
  // kernel of ~1 wave per SIMD) and the kernels' tail rounds overlap the next
  // sub-batch's work.  ev_sub[s][0..4] bracket hash | table | dsm-or-comb |
  // encode of sub-batch s.
  static constexpr int kSub = 4;
  static constexpr int kEv = 5;
  hipStream_t stream2 = nullptr;
  // general path: a sub-batch's key dedupe + tables run on stream_key while
  // its hash kernel runs (both read only the keys); the ladder waits for both
  hipStream_t stream_key = nullptr;
  hipEvent_t ev_kfork[kSub] = {}, ev_kjoin[kSub] = {};
  hipEvent_t ev_sub[kSub][kEv] = {};
  hipEvent_t ev_join[2] = {};
  int last_nsub = 0;
  uint64_t last_chunk_n = 0;  // requests in the last chunk (what edv_stats.phase_ms covers)
  int max_sub = 1;  // edv_options.pipeline (1, 2 and 4 sub-batches measure within 1% at 1M: profiles/r02b)
  // key-sorted comb order (edv_options.key_sort): the permutation and the verdict bytes [kMaxLanes];
  // per sub-batch: block offsets [kSortBlocks][bins], bin totals / bases [bins] x 2, scan scratch
  int key_sort = 2;
  uint64_t bls_pair_max = 32768;  // edv_options.bls_pair_lanes
  uint64_t bls_wave_max = 8192;   // edv_options.bls_wave_checks (8,192 checks 21.8 ms; the two-lane form 27.3)
  // the small keyed path reads its packed inputs straight from pinned host memory (no H2D copy
  // before the kernel); A/B switch EDV_SMALL_ZC=1
  bool small_zero_copy = getenv("EDV_SMALL_ZC") != nullptr;
  // phase events around a single request's small kernel (edv_stats.phase_ms): off unless
  // EDV_SMALL_EVENTS=1 -- the two timestamps cost ~8 us of the round trip (119-126 against
  // 128-134 us per engine call, profiles/r05y)
  bool small_events = getenv("EDV_SMALL_EVENTS") != nullptr;
  // edv_verify_one's resident kernel (edv_resident_kernel): its mailbox, stream, request counter,
  // whether one was launched (it may have left since: box->running), the key window it serves, and
  // whether the path is on (EDV_RESIDENT=0: every single request launches edv_verify_small_kernel)
  ResBox* res_box = nullptr;
  hipStream_t stream_res = nullptr;
  uint64_t res_seq = 0;
  bool res_launched = false, res_stopping = false;
  int res_w = 0;
  bool res_on = !(getenv("EDV_RESIDENT") && getenv("EDV_RESIDENT")[0] == '0');
  uint64_t res_launches = 0, res_served = 0;
  uint64_t small_max = 256;  // edv_options.small_batch: keyed host-pointer chunks of at most this many requests take
                             // edv_verify_small_kernel (0 = never)
  uint32_t* d_kperm = nullptr;
  uint8_t* d_ok8 = nullptr;
  uint32_t* d_kbin = nullptr;
  uint64_t kbin_cap = 0;  // bins allocated per sub-batch
  void* d_kscan_tmp = nullptr;
  size_t kscan_tmp_bytes = 0;  // per sub-batch
  bool timed = false;
  bool small_timed = false;  // the last timed launch was launch_small: ev_sub[0][0] -> [3] only
  // key-table store (registered public keys)
  uint32_t* d_btab_comb32 = nullptr;  // base-point comb table (kBaseW; 11 GiB at W = 24)
  uint32_t* d_ident = nullptr;        // identity niels entry (comb accessors' j = -1)
  uint8_t* d_key_pk = nullptr;
  uint8_t* d_key_valid = nullptr;
  uint32_t* d_key_tab = nullptr;
  uint64_t key_count = 0, key_cap = 0;
  int key_w = 10;                     // comb window of the key tables (EDV_KEY_WINDOWS)
  // staging buffers for host-pointer calls
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    bool pinned = false;  // hipHostMalloc'd host memory
  } b_sig, b_pk, b_msg, b_off, b_bits, b_aux;
  // Host-pointer verifies (host_verify): chunks of kHostChunk requests go
  // through two slots of pinned host + device buffers; the CPU copy of chunk
  // c + 1 into pinned memory and its H2D copy (on stream_copy) overlap the
  // kernels of chunk c (on stream).
  static constexpr int kSlots = 2;
  hipStream_t stream_copy = nullptr;
  hipEvent_t ev_h2d[kSlots] = {}, ev_done[kSlots] = {};
  Buf h_sig[kSlots], h_key[kSlots], h_msg[kSlots], h_off[kSlots], h_bits[kSlots];
  Buf d_sig[kSlots], d_key[kSlots], d_msg[kSlots], d_off[kSlots], d_bits[kSlots];
  Buf d_slot[kSlots];  // EDV_SIG_SLOT96 input of edv_b58_sig_kernel
  // Asynchronous host-pointer verifies (edv_verify_submit / edv_verify_collect): which
  // submission's chunk each slot holds, and per submission its accept bits so far.
  struct SlotUse {
    uint64_t ticket = 0;  // 0 = free
    uint64_t c0 = 0, cn = 0;
    bool bytes = false;  // h_bits holds one verdict byte per request (the small kernel's output)
  } slot_use[kSlots];
  struct Pending {
    uint64_t ticket = 0, n = 0;
    std::vector<uint8_t> bits;
  };
  std::vector<Pending> pending;
  uint64_t next_ticket = 1;
  uint64_t next_slot = 0;  // round robin over the slots, across submissions
  // what the last host-pointer verify did (edv_last_host_stats)
  double last_stage_ms = 0.0;   // CPU copies into the pinned staging (0 when every source was pinned)
  double last_call_ms = 0.0;    // the whole call
  uint64_t last_h2d_bytes = 0;  // bytes copied host -> device
  int last_direct = 0;          // bit 0 sig, 1 keys, 2 msgs, 3 offsets: DMA straight from the caller's pinned memory
  // Asynchronous key-table builds (edv_keys_add_async / edv_keys_set_async): serialized on
  // stream_build with scratch of their own; build k records builds[k].ev; tickets complete in order
  hipStream_t stream_build = nullptr;
  Buf b_build;
  // edv_keys_set_many_async: ids + encodings through pinned staging (a ring of kManyRing, each reused
  // after its copy's event) into device buffers the builds read (one per ring entry)
  static constexpr int kManyRing = 4;
  Buf h_many[kManyRing], d_many[kManyRing];
  hipEvent_t ev_many[kManyRing] = {};
  int many_next = 0;
  struct BuildEv {
    uint64_t ticket;
    hipEvent_t ev;
  };
  std::deque<BuildEv> builds;
  uint64_t build_ticket = 0, build_done = 0;
  hipEvent_t ev_fence[4] = {};  // in-flight work of the context's streams, awaited by a slot rebuild
  // Staged inputs (edv_stage_reserve / edv_stage_put / edv_verify_staged): a device buffer the
  // caller fills piece by piece from pinned memory while it still produces the rest; the puts
  // queue on stream_copy (any thread, under stage_mu) and edv_verify_staged orders after them
  // Two staging sets (edv_stage_select): batch k + 1 is staged into one set while batch k's
  // kernels still read the other (edv_verify_staged_submit / _collect); each set has its
  // own staging buffer, inputs, verdict buffers and completion event.
  static constexpr int kSets = 2;
  int cur_set = 0;
  Buf d_stage_set[kSets];
  std::mutex stage_mu;
  int stage_err = 0;  // first failed put since the last reserve (reported by edv_verify_staged)
  Buf d_spans[kSets];  // message starts and ends of a staged verify [2][n]
  Buf s_sig[kSets], s_key[kSets], s_bits[kSets];  // device: decoded signatures, key ids, accept words
  Buf sh_key[kSets], sh_off[kSets], sh_bits[kSets];  // pinned: staging of non-pinned inputs, verdicts
  hipEvent_t ev_sh2d[kSets] = {}, ev_sdone[kSets] = {};
  uint64_t set_ticket[kSets] = {}, set_n[kSets] = {};  // the uncollected submission holding each set
  // parts of a staged batch launched while it is still being scanned (edv_verify_staged_begin /
  // _part / _end): the set the batch holds, its keying, the first part error, parts launched
  int part_set = -1;
  bool part_keyed = true;
  int part_err = 0;
  std::string part_msg;  // the first failed part's message (the part ran on the scan's copier thread)
  uint64_t part_launched = 0;
  // edv_verify_staged_subset: each set's last submitted staged batch (its item count and message
  // base, kept after the collect while its decoded signatures, spans and messages stay in HBM;
  // cleared by the next reserve or begin of the set) and the subset's own buffers
  uint64_t last_n[kSets] = {}, last_msg_base[kSets] = {};
  bool last_ok[kSets] = {};
  Buf sub_h, sub_d_in, sub_d_sig, sub_d_spans, sub_d_words, sub_h_bits;
  Buf& d_stage() { return d_stage_set[cur_set]; }
};

namespace {

int ensure(edv_ctx::Buf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return 0;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t want = bytes + bytes / 4 + 64;
  hipError_t e = hipMalloc(&b.p, want);
  if (e != hipSuccess) return set_err(EDV_ENOMEM, "hipMalloc(%zu): %s", want, hipGetErrorString(e));
  b.cap = want;
  return 0;
}

int ensure_pinned(edv_ctx::Buf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return 0;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t want = bytes + bytes / 4 + 64;
  hipError_t e = hipHostMalloc(&b.p, want, hipHostMallocDefault);
  if (e != hipSuccess) return set_err(EDV_ENOMEM, "hipHostMalloc(%zu): %s", want, hipGetErrorString(e));
  b.cap = want;
  b.pinned = true;
  return 0;
}

void free_buf(edv_ctx::Buf& b) {
  if (!b.p) return;
  if (b.pinned)
    (void)hipHostFree(b.p);
  else
    (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

// The resident kernel leaves at its next poll: any call that queues GPU work asks it to, since its
// stream may share a hardware queue with the call's streams (GPU_MAX_HW_QUEUES), where it would
// hold the call's kernels back until its idle timeout.
void resident_yield(edv_ctx* ctx) {
  if (ctx->res_launched && !ctx->res_stopping) {
    __atomic_store_n(&ctx->res_box->stop, (uint64_t)1, __ATOMIC_RELEASE);
    ctx->res_stopping = true;
  }
}

int set_device(edv_ctx* ctx) {
  if (!ctx) return set_err(EDV_EINVAL, "null context");
  resident_yield(ctx);
  HIP_TRY(hipSetDevice(ctx->device));
  return 0;
}

hipStream_t pick_stream(edv_ctx* ctx, void* stream) { return stream ? (hipStream_t)stream : ctx->stream; }

// Key windows a context accepts (edv_keys_set_window); every one instantiates
// its own comb / fill kernels.
#ifndef EDV_KEY_WINDOWS
#define EDV_KEY_WINDOWS(X) X(4) X(6) X(8) X(10) X(12) X(13) X(14) X(16)
#endif
bool key_window_ok(int w) {
#define EDV_KW_OK(W) || w == W
  return false EDV_KEY_WINDOWS(EDV_KW_OK);
#undef EDV_KW_OK
}
uint32_t key_rows(int w) {
#define EDV_KW_ROWS(W) \
  if (w == W) return Window<W>::kRows;
  EDV_KEY_WINDOWS(EDV_KW_ROWS)
#undef EDV_KW_ROWS
  return Window<8>::kRows;
}
uint32_t key_tab_words(int w) {
#define EDV_KW_WORDS(W) \
  if (w == W) return Window<W>::kTableWords;
  EDV_KEY_WINDOWS(EDV_KW_WORDS)
#undef EDV_KW_WORDS
  return Window<8>::kTableWords;
}

int launch_encode(edv_ctx* ctx, const uint8_t* sig, uint64_t cn, unsigned long long* words, uint64_t off,
                  uint64_t chunk, hipStream_t st, const uint32_t* perm = nullptr) {
  const uint64_t waves = div_up(cn, 64ull * kEncodeM);
  const uint32_t grid = (uint32_t)div_up(waves * 64, kBlock);
  uint8_t* ok8 = perm ? ctx->d_ok8 + off : nullptr;
  hipLaunchKernelGGL(edv_encode_kernel<kEncodeM>, dim3(grid), dim3(kBlock), 0, st, sig, cn, ctx->d_pt + off,
                     ctx->d_pre + off, ctx->d_flags + off, words, chunk, perm, ok8);
  HIP_TRY(hipGetLastError());
  if (perm) {
    hipLaunchKernelGGL(edv_ok_pack_kernel, dim3((uint32_t)div_up(cn, kBlock)), dim3(kBlock), 0, st, ok8, cn, words);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// The key-sort scratch for `bins` bins (grown when the key count passes it; in-flight launches
// may read the old one, so a regrowth waits for the device).
int ensure_key_sort(edv_ctx* ctx, uint64_t bins) {
  if (bins <= ctx->kbin_cap) return 0;
  uint64_t cap = ctx->kbin_cap ? ctx->kbin_cap : 1024;
  while (cap < bins) cap *= 2;
  if (cap > kSortMaxBins) cap = kSortMaxBins;
  if (ctx->d_kbin) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(ctx->d_kbin));
    ctx->d_kbin = nullptr;
  }
  if (ctx->d_kscan_tmp) {
    HIP_TRY(hipFree(ctx->d_kscan_tmp));
    ctx->d_kscan_tmp = nullptr;
  }
  ctx->kbin_cap = 0;
  const uint64_t per_sub = 2 * cap;
  hipError_t e = hipMalloc(&ctx->d_kbin, edv_ctx::kSub * per_sub * sizeof(uint32_t));
  if (e != hipSuccess) return set_err(EDV_ENOMEM, "key-sort scratch: %s", hipGetErrorString(e));
  size_t bytes = 0;
  HIP_TRY(rocprim::exclusive_scan(nullptr, bytes, ctx->d_kbin, ctx->d_kbin, 0u, (size_t)cap, rocprim::plus<uint32_t>(),
                                  ctx->stream));
  ctx->kscan_tmp_bytes = (bytes + 255) & ~(size_t)255;
  e = hipMalloc(&ctx->d_kscan_tmp, edv_ctx::kSub * (ctx->kscan_tmp_bytes ? ctx->kscan_tmp_bytes : 256));
  if (e != hipSuccess) return set_err(EDV_ENOMEM, "key-sort scan scratch: %s", hipGetErrorString(e));
  ctx->kbin_cap = cap;
  return 0;
}

// kperm of a keyed sub-batch: its requests in key-id order (edv_key_*_kernel).
int launch_key_sort(edv_ctx* ctx, const uint32_t* kidx, uint64_t cn, uint32_t bins, uint32_t* kperm, int sub,
                    hipStream_t q) {
  uint32_t* total = ctx->d_kbin + sub * 2 * ctx->kbin_cap;
  uint32_t* cursor = total + ctx->kbin_cap;
  const size_t lds = (size_t)bins * sizeof(uint32_t);
  // blocks of at least 2,048 requests (a block's LDS histogram costs its bins)
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(kSortBlocks, div_up(cn, 2048));
  HIP_TRY(hipMemsetAsync(total, 0, (size_t)bins * sizeof(uint32_t), q));
  hipLaunchKernelGGL(edv_key_hist_kernel, dim3(blocks), dim3(kSortThreads), lds, q, kidx, cn, bins, total);
  HIP_TRY(hipGetLastError());
  size_t tmp = ctx->kscan_tmp_bytes;
  HIP_TRY(rocprim::exclusive_scan((char*)ctx->d_kscan_tmp + (size_t)sub * tmp, tmp, total, cursor, 0u, (size_t)bins,
                                  rocprim::plus<uint32_t>(), q));
  hipLaunchKernelGGL(edv_key_scatter_kernel, dim3(blocks), dim3(kSortThreads), lds, q, kidx, cn, bins, cursor, kperm);
  HIP_TRY(hipGetLastError());
  return 0;
}

// Length-bucket flags of the next launch: mode 1 / 3 always sort (3 also
// packs), mode 2 sorts when the caller saw mixed lengths (host offsets).
void set_bucketing(edv_ctx* ctx, bool mixed) {
  ctx->bucket_now = ctx->bucket_mode == 1 || ctx->bucket_mode == 3 || (ctx->bucket_mode == 2 && mixed);
  ctx->pack_now = ctx->bucket_mode == 3;
}

int ensure_arena(edv_ctx* ctx) {
  const uint64_t groups = kMaxLanes / 64;
  if (!ctx->d_gunits) {
    HIP_TRY(hipMalloc(&ctx->d_gunits, (groups + 1) * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&ctx->d_goff, (groups + 1) * sizeof(uint64_t)));
    size_t bytes = 0;
    HIP_TRY(rocprim::exclusive_scan(nullptr, bytes, ctx->d_gunits, ctx->d_goff, (uint64_t)0, (size_t)groups,
                                    rocprim::plus<uint64_t>(), ctx->stream));
    ctx->scan_tmp_bytes = bytes;
    HIP_TRY(hipMalloc(&ctx->d_scan_tmp, bytes ? bytes : 16));
  }
  if (ctx->arena_units != ctx->arena_want) {
    if (ctx->d_arena) {
      HIP_TRY(hipDeviceSynchronize());  // earlier launches may still read the old arena
      HIP_TRY(hipFree(ctx->d_arena));
    }
    ctx->d_arena = nullptr;
    ctx->arena_units = 0;
    if (ctx->arena_want) {
      hipError_t e = hipMalloc(&ctx->d_arena, ctx->arena_want * sizeof(Chunk16));
      if (e != hipSuccess)
        return set_err(EDV_ENOMEM, "unit arena (%llu units): %s", (unsigned long long)ctx->arena_want,
                       hipGetErrorString(e));
    }
    ctx->arena_units = ctx->arena_want;
  }
  return 0;
}

// The kernels of one sub-batch [off, off + cn) of a chunk (scratch index
// off.. with the chunk's stride), on stream q, bracketed by ev[0..4].
struct SubBatch {
  const uint8_t* sig;  // first request of the sub-batch
  const uint8_t* pk;   // general path: its keys
  const uint32_t* kidx;  // keyed path: its key ids
  const uint64_t* ms;    // its message starts
  const uint64_t* me;    // its message ends
  unsigned long long* words;
  uint64_t cn, soff;
};

// Packed message layout of a sorted sub-batch (the UnitArena comment):
// group sizes, their exclusive scan, the pack; *ua describes the result.
int launch_pack(edv_ctx* ctx, const SubBatch& b, const uint8_t* msgs, const uint32_t* perm, hipStream_t q,
                UnitArena* ua) {
  int r = ensure_arena(ctx);
  if (r) return r;
  if (!ctx->d_arena) return 0;  // arena size 0: every group reads in place
  const uint32_t grid = (uint32_t)div_up(b.cn, kBlock);
  const uint64_t groups = div_up(b.cn, 64);
  hipLaunchKernelGGL(edv_group_units_kernel, dim3(grid), dim3(kBlock), 0, q, b.ms, b.me, b.cn, perm, ctx->d_gunits);
  HIP_TRY(hipGetLastError());
  size_t tmp = ctx->scan_tmp_bytes;
  HIP_TRY(rocprim::exclusive_scan(ctx->d_scan_tmp, tmp, ctx->d_gunits, ctx->d_goff, (uint64_t)0, (size_t)groups,
                                  rocprim::plus<uint64_t>(), q));
  *ua = {ctx->d_arena, ctx->d_gunits, ctx->d_goff, ctx->arena_units};
  hipLaunchKernelGGL(edv_pack_units_kernel, dim3(grid), dim3(kBlock), 0, q, msgs, b.ms, b.me, b.cn, perm, *ua);
  HIP_TRY(hipGetLastError());
  return 0;
}

int launch_sub(edv_ctx* ctx, bool keyed, const SubBatch& b, const uint8_t* msgs, uint64_t chunk, hipStream_t q,
               hipEvent_t* ev, int sub) {
  const uint32_t grid = (uint32_t)div_up(b.cn, kBlock);
  uint32_t* hs = ctx->d_hsoa + b.soff;
  uint8_t* fl = ctx->d_flags + b.soff;
  uint32_t* pt = ctx->d_pt + b.soff;
  uint32_t* perm = nullptr;
  uint32_t* kperm = nullptr;  // keyed path: the comb's key-sorted lane order (nullptr = request order)
  UnitArena ua = {nullptr, nullptr, nullptr, 0};
  HIP_TRY(hipEventRecord(ev[0], q));
  if (ctx->bucket_now && (b.cn > 64 || ctx->pack_now)) {
    // hash lanes in SHA-512 block-count order, longest first (stable)
    perm = ctx->d_perm + b.soff;
    uint8_t* key = ctx->d_lenkey + b.soff;
    hipLaunchKernelGGL(edv_len_key_kernel, dim3(grid), dim3(kBlock), 0, q, b.ms, b.me, b.cn, key);
    HIP_TRY(hipGetLastError());
    size_t tmp = ctx->sort_tmp_bytes;
    HIP_TRY(rocprim::radix_sort_pairs_desc((char*)ctx->d_sort_tmp + (size_t)sub * tmp, tmp, key, key + kMaxLanes,
                                           rocprim::counting_iterator<uint32_t>(0), perm, (uint32_t)b.cn, 0,
                                           kLenKeyBits, q));
  }
  if (ctx->pack_now && perm) {
    int r = launch_pack(ctx, b, msgs, perm, q, &ua);
    if (r) return r;
  }
  if (keyed) {
    const uint32_t kc = (uint32_t)ctx->key_count;
    if (ua.base)
      hipLaunchKernelGGL(edv_hash_keyed_kernel<true>, dim3(grid), dim3(kBlock), 0, q, b.sig, b.kidx, kc,
                         ctx->d_key_pk, ctx->d_key_valid, msgs, b.ms, b.me, b.cn, hs, fl, chunk, perm, ua);
    else
      hipLaunchKernelGGL(edv_hash_keyed_kernel<false>, dim3(grid), dim3(kBlock), 0, q, b.sig, b.kidx, kc,
                         ctx->d_key_pk, ctx->d_key_valid, msgs, b.ms, b.me, b.cn, hs, fl, chunk, perm, ua);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], q));
    // key order of the comb lanes (the keyed path's "table" phase): auto sorts sub-batches of
    // 4,096 requests or more at key windows of 15 and up (rows of 2 MiB and more) whose ids fit
    // the LDS cursors (kSortMaxBins)
    const uint64_t bins = (uint64_t)kc + 1;
    if ((ctx->key_sort == 1 || (ctx->key_sort == 2 && b.cn >= 4096 && ctx->key_w >= 15)) && bins <= kSortMaxBins) {
      int r = ensure_key_sort(ctx, bins);
      if (r) return r;
      kperm = ctx->d_kperm + b.soff;
      if ((r = launch_key_sort(ctx, b.kidx, b.cn, (uint32_t)bins, kperm, sub, q))) return r;
    }
    HIP_TRY(hipEventRecord(ev[2], q));
#define EDV_COMB_LAUNCH(W)                                                                                   \
  hipLaunchKernelGGL(edv_comb_kernel<W>, dim3(grid), dim3(kBlock), 0, q, b.sig, b.kidx, kc, b.cn, hs,        \
                     ctx->d_key_tab, ctx->key_cap, ctx->d_btab_comb32, ctx->d_ident, pt, chunk, kperm)
#define EDV_COMB_CASE(W) \
  case W:                \
    EDV_COMB_LAUNCH(W);  \
    break;
    switch (ctx->key_w) {
      EDV_KEY_WINDOWS(EDV_COMB_CASE)
      default:
        return set_err(EDV_EINVAL, "key window %d", ctx->key_w);
    }
#undef EDV_COMB_CASE
#undef EDV_COMB_LAUNCH
    HIP_TRY(hipGetLastError());
  } else {
    // the per-lane A tables are per 256-lane block of the chunk: sub-batch
    // offsets are multiples of the block size, so each sub-batch has its own
    uint32_t* tab = (uint32_t*)((char*)ctx->d_scratch + (b.soff / kBlock) * (uint64_t)kRegionBytes);
    const uint64_t L = kMaxLanes;
    uint32_t* slots = ctx->d_dedup + 2 * b.soff;
    uint32_t* slot_u = ctx->d_dedup + 2 * L + 2 * b.soff;
    uint32_t* req_slot = ctx->d_dedup + 4 * L + b.soff;
    uint32_t* reps = ctx->d_dedup + 5 * L + b.soff;
    uint8_t* key_ok = ctx->d_key_ok + b.soff;
    uint32_t* count = ctx->d_ucount + sub;
    const uint32_t nslots = (uint32_t)(2 * b.cn);
    hipStream_t qk = ctx->stream_key;
    HIP_TRY(hipEventRecord(ctx->ev_kfork[sub], q));
    HIP_TRY(hipStreamWaitEvent(qk, ctx->ev_kfork[sub], 0));
    HIP_TRY(hipMemsetAsync(slots, 0xff, nslots * sizeof(uint32_t), qk));
    HIP_TRY(hipMemsetAsync(count, 0, sizeof(uint32_t), qk));
    hipLaunchKernelGGL(edv_dedup_insert_kernel, dim3(grid), dim3(kBlock), 0, qk, b.pk, b.cn, slots, nslots, req_slot);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(edv_dedup_assign_kernel, dim3(grid), dim3(kBlock), 0, qk, b.cn, slots, req_slot, slot_u, reps,
                       count);
    HIP_TRY(hipGetLastError());
    // one lane per distinct key; the grid covers the worst case (all distinct)
    hipLaunchKernelGGL(edv_table_kernel, dim3(grid), dim3(kBlock), 0, qk, b.pk, b.cn, reps, count, tab, key_ok);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ctx->ev_kjoin[sub], qk));
    if (ua.base)
      hipLaunchKernelGGL(edv_hash_kernel<true>, dim3(grid), dim3(kBlock), 0, q, b.sig, b.pk, msgs, b.ms, b.me, b.cn,
                         hs, fl, chunk, perm, ua);
    else
      hipLaunchKernelGGL(edv_hash_kernel<false>, dim3(grid), dim3(kBlock), 0, q, b.sig, b.pk, msgs, b.ms, b.me, b.cn,
                         hs, fl, chunk, perm, ua);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], q));
    HIP_TRY(hipStreamWaitEvent(q, ctx->ev_kjoin[sub], 0));
    HIP_TRY(hipEventRecord(ev[2], q));  // hash | key tables not hidden behind it | ladder
    hipLaunchKernelGGL(edv_dsm_kernel, dim3(grid), dim3(kBlock), 0, q, b.sig, b.cn, hs, tab, chunk, ctx->d_btab_comb32,
                       ctx->d_ident, pt, req_slot, slot_u, count, key_ok, fl);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(ev[3], q));
  int r = launch_encode(ctx, b.sig, b.cn, b.words, b.soff, chunk, q, kperm);
  if (r) return r;
  HIP_TRY(hipEventRecord(ev[4], q));
  return 0;
}

// Sub-batch boundaries: multiples of 64 * kEncodeM (whole encode groups and
// bitmask words) and of kBlock (whole A-table regions).
constexpr uint64_t kSubAlign = 64ull * kEncodeM > (uint64_t)kBlock ? 64ull * kEncodeM : (uint64_t)kBlock;

int launch_pipeline(edv_ctx* ctx, bool keyed, const void* d_sig, const void* d_keys, const void* d_msgs,
                    const uint64_t* ms, const uint64_t* me, uint64_t n, void* d_words, hipStream_t st) {
  if (n == 0) return 0;
  const uint8_t* sig = (const uint8_t*)d_sig;
  unsigned long long* words = (unsigned long long*)d_words;
  const uint64_t chunk = ctx->scratch_lanes;  // multiple of kSubAlign
  // stream2 starts after everything already queued on st (the inputs)
  HIP_TRY(hipEventRecord(ctx->ev_join[0], st));
  HIP_TRY(hipStreamWaitEvent(ctx->stream2, ctx->ev_join[0], 0));
  for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
    const uint64_t cn = (n - c0) < chunk ? (n - c0) : chunk;
    // sub-batches of the chunk; the next chunk reuses the scratch, so it
    // starts only after both streams are done with this one
    // (sorted hash lanes: at most 2 -- measured on configs[3], 3 or 4
    // sub-batches are 10% slower than 1 or 2)
    // (packed units: 1 -- the sub-batch owns the whole unit arena)
    const uint64_t nsub = ctx->pack_now ? 1 : ctx->bucket_now && ctx->max_sub > 2 ? 2 : (uint64_t)ctx->max_sub;
    const uint64_t per = div_up(div_up(cn, nsub), kSubAlign) * kSubAlign;
    int ns = 0;
    for (uint64_t s0 = 0; s0 < cn; s0 += per, ++ns) {
      SubBatch b;
      b.cn = (cn - s0) < per ? (cn - s0) : per;
      b.soff = s0;
      b.sig = sig + 64 * (c0 + s0);
      b.pk = keyed ? nullptr : (const uint8_t*)d_keys + 32 * (c0 + s0);
      b.kidx = keyed ? (const uint32_t*)d_keys + (c0 + s0) : nullptr;
      b.ms = ms + c0 + s0;
      b.me = me + c0 + s0;
      b.words = words + (c0 + s0) / 64;
      hipStream_t q = (ns & 1) ? ctx->stream2 : st;
      int r = launch_sub(ctx, keyed, b, (const uint8_t*)d_msgs, chunk, q, ctx->ev_sub[ns], ns);
      if (r) return r;
    }
    ctx->last_nsub = ns;
    ctx->last_chunk_n = cn;
    if (c0 + cn < n) {  // join before the scratch is reused
      HIP_TRY(hipEventRecord(ctx->ev_join[1], ctx->stream2));
      HIP_TRY(hipStreamWaitEvent(st, ctx->ev_join[1], 0));
      HIP_TRY(hipEventRecord(ctx->ev_join[0], st));
      HIP_TRY(hipStreamWaitEvent(ctx->stream2, ctx->ev_join[0], 0));
    }
  }
  // the caller's stream completes when both have
  HIP_TRY(hipEventRecord(ctx->ev_join[1], ctx->stream2));
  HIP_TRY(hipStreamWaitEvent(st, ctx->ev_join[1], 0));
  ctx->timed = true;
  ctx->small_timed = false;
  return 0;
}

// A small keyed batch through edv_verify_small_kernel (one workgroup per request) and the
// verdict-byte pack; its duration lands in the comb phase of edv_stats.phase_ms.
// host_ok8 (pinned host memory, n bytes): the kernel stores the verdict bytes there itself and
// no pack kernel or D2H copy follows (d_words unused) -- two fewer GPU commands on the latency
// path of one authenticate().
int launch_small(edv_ctx* ctx, const void* d_sig, const void* d_kidx, const void* d_msgs, const uint64_t* ms,
                 const uint64_t* me, uint64_t n, void* d_words, hipStream_t st, uint8_t* host_ok8 = nullptr) {
  if (n == 0) return 0;
  if (ctx->key_count == 0) return set_err(EDV_EINVAL, "no registered keys");
  hipEvent_t* ev = ctx->ev_sub[0];
  const bool timed = ctx->small_events || !host_ok8;
  if (timed) HIP_TRY(hipEventRecord(ev[0], st));
  uint8_t* ok8 = host_ok8 ? host_ok8 : ctx->d_ok8;
  const uint32_t kc = (uint32_t)ctx->key_count;
#define EDV_SMALL_CASE(W)                                                                                        \
  case W:                                                                                                        \
    hipLaunchKernelGGL(edv_verify_small_kernel<W>, dim3((uint32_t)n), dim3(kSmallThreads), 0, st,                \
                       (const uint8_t*)d_sig, (const uint32_t*)d_kidx, kc, ctx->d_key_pk, ctx->d_key_valid,      \
                       (const uint8_t*)d_msgs, ms, me, n, ctx->d_key_tab, ctx->key_cap, ctx->d_btab_comb32,     \
                       ctx->d_ident, ok8);                                                                       \
    break;
  switch (ctx->key_w) {
    EDV_KEY_WINDOWS(EDV_SMALL_CASE)
    default:
      return set_err(EDV_EINVAL, "key window %d", ctx->key_w);
  }
#undef EDV_SMALL_CASE
  HIP_TRY(hipGetLastError());
  if (timed) HIP_TRY(hipEventRecord(ev[3], st));
  if (!host_ok8) {
    hipLaunchKernelGGL(edv_ok_pack_kernel, dim3((uint32_t)div_up(n, kBlock)), dim3(kBlock), 0, st, ctx->d_ok8, n,
                       (unsigned long long*)d_words);
    HIP_TRY(hipGetLastError());
  }
  if (timed) {  // (an untimed launch leaves the previous launch's phases readable)
    ctx->last_nsub = 1;
    ctx->last_chunk_n = n;
    ctx->timed = true;
    ctx->small_timed = true;
  }
  return 0;
}

int launch_verify(edv_ctx* ctx, const void* d_sig, const void* d_pk, const void* d_msgs, const void* d_off, uint64_t n,
                  void* d_words, hipStream_t st) {
  const uint64_t* off = (const uint64_t*)d_off;
  return launch_pipeline(ctx, false, d_sig, d_pk, d_msgs, off, off + 1, n, d_words, st);
}

}  // namespace


// ------------------------------------------------------------- key tables

static int keys_reserve(edv_ctx* ctx, uint64_t need) {
  if (need <= ctx->key_cap) return 0;
  uint64_t cap = ctx->key_cap ? ctx->key_cap : 64;  // W = 16: 64 MiB per key
  while (cap < need) cap *= 2;
  uint8_t *pk = nullptr, *valid = nullptr;
  uint32_t* tab = nullptr;
  hipError_t e;
  if ((e = hipMalloc(&pk, cap * 32)) || (e = hipMalloc(&valid, cap)) ||
      (e = hipMalloc(&tab, cap * (uint64_t)key_tab_words(ctx->key_w) * 4))) {
    if (pk) (void)hipFree(pk);
    if (valid) (void)hipFree(valid);
    if (tab) (void)hipFree(tab);
    return set_err(EDV_ENOMEM, "key store of %llu keys: %s", (unsigned long long)cap, hipGetErrorString(e));
  }
  if (ctx->key_count) {
    // table builds of edv_keys_add_device may still run on a caller's stream:
    // the copies below must see them complete
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyAsync(pk, ctx->d_key_pk, ctx->key_count * 32, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(valid, ctx->d_key_valid, ctx->key_count, hipMemcpyDeviceToDevice, ctx->stream));
    // row-major over keys: row r of every table is one slab of key_cap tables
    const uint64_t rows = key_rows(ctx->key_w), row_bytes = key_tab_words(ctx->key_w) / rows * 4;
    for (uint64_t r = 0; r < rows; ++r)
      HIP_TRY(hipMemcpyAsync((char*)tab + r * cap * row_bytes, (const char*)ctx->d_key_tab + r * ctx->key_cap * row_bytes,
                             ctx->key_count * row_bytes, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  if (ctx->d_key_pk) (void)hipFree(ctx->d_key_pk);
  if (ctx->d_key_valid) (void)hipFree(ctx->d_key_valid);
  if (ctx->d_key_tab) (void)hipFree(ctx->d_key_tab);
  ctx->d_key_pk = pk;
  ctx->d_key_valid = valid;
  ctx->d_key_tab = tab;
  ctx->key_cap = cap;
  return 0;
}

// Build tables for keys [first, first + nkeys) whose 32-byte encodings are
// already in d_key_pk, in slices of kKeyBuildSlice keys (bounded scratch).
constexpr uint64_t kKeyBuildScratch = 1ull << 30;  // bytes of row bases + prefix products per slice (the row
                                                   // kernel is one lane per key: fewer, larger slices)
template <int W>
static int keys_build_w(edv_ctx* ctx, uint64_t first, uint64_t nkeys, hipStream_t st, edv_ctx::Buf& aux) {
  constexpr int R = Window<W>::kRows, E = Window<W>::kEntries;
  constexpr uint64_t per_key = (uint64_t)R * kRowWords * 4 + (uint64_t)R * E * 10 * 4;
  const uint64_t max_slice = kKeyBuildScratch / per_key > 0 ? kKeyBuildScratch / per_key : 1;
  const uint64_t slice = nkeys < max_slice ? nkeys : max_slice;
  int r;
  // rows: R p3 bases per key; pre: E prefix products per row
  const size_t need = slice * R * kRowWords * 4 + slice * R * E * 10 * 4;
  // an earlier build on this stream may still read the scratch: it finishes before a regrowth frees it
  if (aux.cap < need) HIP_TRY(hipStreamSynchronize(st));
  if ((r = ensure(aux, need))) return r;
  uint32_t* rows = (uint32_t*)aux.p;
  uint32_t* pre = rows + slice * R * kRowWords;
  for (uint64_t k0 = 0; k0 < nkeys; k0 += slice) {
    const uint64_t kn = nkeys - k0 < slice ? nkeys - k0 : slice;
    const uint64_t k = first + k0;
    hipLaunchKernelGGL(edv_key_rows_kernel<W>, dim3((uint32_t)div_up(kn, kBlock)), dim3(kBlock), 0, st,
                       ctx->d_key_pk + 32 * k, kn, rows, ctx->d_key_valid + k);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(edv_comb_fill_kernel<W>, dim3((uint32_t)div_up(kn * R * FillShape<W>::NCH, kBlock)),
                       dim3(kBlock), 0, st, rows, kn * R, ctx->d_key_tab, pre, k, ctx->key_cap);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// Tables for keys d_pk[0 .. nkeys) (device) into store slots d_ids[0 .. nkeys) (device, distinct), their
// encodings copied into the store too: edv_keys_set_many_async.
template <int W>
static int keys_build_ids_w(edv_ctx* ctx, const uint8_t* d_pk, const uint32_t* d_ids, uint64_t nkeys, hipStream_t st,
                            edv_ctx::Buf& aux) {
  constexpr int R = Window<W>::kRows, E = Window<W>::kEntries;
  constexpr uint64_t per_key = (uint64_t)R * kRowWords * 4 + (uint64_t)R * E * 10 * 4;
  const uint64_t max_slice = kKeyBuildScratch / per_key > 0 ? kKeyBuildScratch / per_key : 1;
  const uint64_t slice = nkeys < max_slice ? nkeys : max_slice;
  const size_t need = slice * R * kRowWords * 4 + slice * R * E * 10 * 4;
  if (aux.cap < need) HIP_TRY(hipStreamSynchronize(st));
  int r;
  if ((r = ensure(aux, need))) return r;
  uint32_t* rows = (uint32_t*)aux.p;
  uint32_t* pre = rows + slice * R * kRowWords;
  for (uint64_t k0 = 0; k0 < nkeys; k0 += slice) {
    const uint64_t kn = nkeys - k0 < slice ? nkeys - k0 : slice;
    hipLaunchKernelGGL(edv_key_rows_kernel<W>, dim3((uint32_t)div_up(kn, kBlock)), dim3(kBlock), 0, st, d_pk + 32 * k0,
                       kn, rows, ctx->d_key_valid, d_ids + k0, ctx->d_key_pk);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(edv_comb_fill_kernel<W>, dim3((uint32_t)div_up(kn * R * FillShape<W>::NCH, kBlock)),
                       dim3(kBlock), 0, st, rows, kn * R, ctx->d_key_tab, pre, (uint64_t)0, ctx->key_cap, d_ids + k0);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

static int keys_build(edv_ctx* ctx, uint64_t first, uint64_t nkeys, hipStream_t st) {
  if (!nkeys) return 0;
  edv_ctx::Buf& aux = st == ctx->stream_build ? ctx->b_build : ctx->b_aux;
#define EDV_BUILD_CASE(W) \
  case W:                 \
    return keys_build_w<W>(ctx, first, nkeys, st, aux);
  switch (ctx->key_w) {
    EDV_KEY_WINDOWS(EDV_BUILD_CASE)
    default:
      return set_err(EDV_EINVAL, "key window %d", ctx->key_w);
  }
#undef EDV_BUILD_CASE
}

static int launch_verify_keyed(edv_ctx* ctx, const void* d_sig, const void* d_kidx, const void* d_msgs,
                               const void* d_off, uint64_t n, void* d_words, hipStream_t st) {
  if (n == 0) return 0;
  if (ctx->key_count == 0) return set_err(EDV_EINVAL, "no registered keys");
  const uint64_t* off = (const uint64_t*)d_off;
  return launch_pipeline(ctx, true, d_sig, d_kidx, d_msgs, off, off + 1, n, d_words, st);
}

// Pinned host memory handed out by edv_host_alloc (process-wide: the blocks
// are allocated portable, so every context's copy engine can read them).  A
// host-pointer verify whose source range lies inside one block copies it to
// the device straight from there, with no CPU staging copy.
struct PinnedBlock {
  const uint8_t* p;
  size_t n;
};
std::mutex g_pinned_mu;
std::vector<PinnedBlock> g_pinned;

static bool pinned_range(const void* p, size_t n) {
  if (!p) return false;
  const uint8_t* a = (const uint8_t*)p;
  std::lock_guard<std::mutex> g(g_pinned_mu);
  for (const PinnedBlock& b : g_pinned)
    if (a >= b.p && a + n <= b.p + b.n) return true;
  return false;
}

// Host-pointer verify: chunks of kHostChunk requests, two slots of device
// buffers.  Chunk c: its inputs go to the device on stream_copy -- straight
// from the caller's memory when it lies in edv_host_alloc'd pinned blocks,
// otherwise through a CPU copy into the slot's pinned staging first -- then
// (after the H2D event) the signature-slot decode if any, the kernels and the
// bitmask D2H on the context stream.  So the copies of chunk c + 1 run while
// chunk c's kernels do.  Offsets are copied as given: the kernels see the
// device message buffer at (base - msg_off[c0]), so no offset is rebased on
// the host.  key_bytes: 32 (pk32) or 4 (key ids); sig_stride: 64 (R || S) or
// EDV_SIG_SLOT96.
constexpr uint64_t kHostChunk = 1ull << 18;

// memcpy into the pinned staging on up to 8 host threads (8 MiB or more each;
// the caller and pooled helpers, host_pool.h): one thread copies a pageable
// source at ~15 GB/s, below the H2D rate, so a 2^18-request chunk of 200-byte
// messages (~70 MB) would otherwise take longer to stage than to transfer and
// verify.
static void stage_copy(void* dst, const void* src, size_t n) {
  constexpr size_t kPerThread = 8u << 20;
  const unsigned hw = std::thread::hardware_concurrency();
  size_t t = n / kPerThread;
  if (t > 8) t = 8;
  if (hw && t > hw) t = hw;
  if (t <= 1) {
    memcpy(dst, src, n);
    return;
  }
  const size_t per = (n / t + 63) & ~(size_t)63;
  HostPool::get().run((int)t, [&](int w) {
    const size_t a = (size_t)w * per, b = ((size_t)w + 1) * per < n ? ((size_t)w + 1) * per : n;
    if (a < b) memcpy((char*)dst + a, (const char*)src + a, b - a);
  });
}

// A slot's chunk done: its bits into its submission's buffer, the slot free.
static int drain_slot(edv_ctx* ctx, int sl) {
  edv_ctx::SlotUse& u = ctx->slot_use[sl];
  if (!u.ticket) return 0;
  HIP_TRY(hipEventSynchronize(ctx->ev_done[sl]));
  for (edv_ctx::Pending& p : ctx->pending)
    if (p.ticket == u.ticket) {
      if (u.bytes) {  // c0 is a multiple of 64 (kHostChunk)
        const uint8_t* b = (const uint8_t*)ctx->h_bits[sl].p;
        uint8_t* o = p.bits.data() + u.c0 / 8;
        for (uint64_t k = 0; k < u.cn; ++k)
          if (b[k]) o[k >> 3] |= (uint8_t)(1u << (k & 7));
      } else {
        memcpy(p.bits.data() + u.c0 / 8, ctx->h_bits[sl].p, (u.cn + 7) / 8);
      }
      break;
    }
  u.ticket = 0;
  return 0;
}

static int host_submit(edv_ctx* ctx, bool keyed, const uint8_t* sig, uint64_t sig_stride, const uint8_t* keys,
                       const uint8_t* msgs, const uint64_t* msg_off, uint64_t n, uint64_t* ticket_out) {
  using clk = std::chrono::steady_clock;
  const auto t_call = clk::now();
  double stage_s = 0.0;
  const uint64_t key_bytes = keyed ? 4 : 32;
  const bool slots = sig_stride == EDV_SIG_SLOT96;
  for (uint64_t i = 0; i < n; ++i)
    if (msg_off[i + 1] < msg_off[i]) return set_err(EDV_EINVAL, "msg_off[%llu] decreasing", (unsigned long long)i);
  if (msg_off[n] > msg_off[0] && !msgs) return set_err(EDV_EINVAL, "null msgs");
  if (keyed && ctx->key_count == 0) return set_err(EDV_EINVAL, "no registered keys");
  const bool sig_direct = pinned_range(sig, sig_stride * n);
  const bool key_direct = pinned_range(keys, key_bytes * n);
  const bool msg_direct = msg_off[n] == msg_off[0] || pinned_range(msgs + msg_off[0], msg_off[n] - msg_off[0]);
  const bool off_direct = pinned_range(msg_off, 8 * (n + 1));
  ctx->last_direct = (sig_direct ? 1 : 0) | (key_direct ? 2 : 0) | (msg_direct ? 4 : 0) | (off_direct ? 8 : 0);
  ctx->last_h2d_bytes = 0;
  const uint64_t ticket = ctx->next_ticket++;
  // at most kMaxPending uncollected submissions: a caller that submits more before collecting gets an
  // error here rather than a silently dropped verdict set at collect time
  if (ctx->pending.size() >= kMaxPending)
    return set_err(EDV_EINVAL, "%llu submissions outstanding: collect before submitting more",
                   (unsigned long long)ctx->pending.size());
  ctx->pending.push_back(edv_ctx::Pending{ticket, n, std::vector<uint8_t>((size_t)((n + 7) / 8), 0)});
  // a source the copy engine reads: the caller's pinned memory, or the slot's staging after a CPU copy
  auto source = [&](bool direct, edv_ctx::Buf& stage, const uint8_t* src, uint64_t bytes, bool threaded,
                    const uint8_t** out) -> int {
    if (direct || !bytes) {
      *out = src;
      return 0;
    }
    int r = ensure_pinned(stage, bytes + 16);
    if (r) return r;
    const auto t0 = clk::now();
    if (threaded)
      stage_copy(stage.p, src, bytes);
    else
      memcpy(stage.p, src, bytes);
    stage_s += std::chrono::duration<double>(clk::now() - t0).count();
    *out = (const uint8_t*)stage.p;
    return 0;
  };
  auto run = [&]() -> int {
    int r;
    for (uint64_t c0 = 0; c0 < n; c0 += kHostChunk) {
      const int sl = (int)(ctx->next_slot++ % edv_ctx::kSlots);
      if ((r = drain_slot(ctx, sl))) return r;  // the slot's previous chunk (this or an earlier submission)
      const uint64_t cn = (n - c0) < kHostChunk ? (n - c0) : kHostChunk;
      const uint64_t m0 = msg_off[c0], mbytes = msg_off[c0 + cn] - m0, nwords = div_up(cn, 64);
      if ((r = ensure_pinned(ctx->h_bits[sl], 8 * nwords)) || (r = ensure(ctx->d_sig[sl], 64 * cn)) ||
          (r = ensure(ctx->d_key[sl], key_bytes * cn)) || (r = ensure(ctx->d_msg[sl], mbytes + 16)) ||
          (r = ensure(ctx->d_off[sl], 8 * (cn + 1))) || (r = ensure(ctx->d_bits[sl], 8 * nwords)) ||
          (slots && (r = ensure(ctx->d_slot[sl], sig_stride * cn))))
        return r;
      // a small chunk (a message the verify-ahead missed): its four inputs packed into one pinned
      // block and ONE copy on the compute stream, instead of four copies on the copy stream and a
      // cross-stream wait -- each small DMA costs microseconds of latency, not bandwidth
      const uint64_t a16 = 16;
      const uint64_t o_key = div_up(sig_stride * cn, a16) * a16, o_off = o_key + div_up(key_bytes * cn, a16) * a16,
                     o_msg = o_off + div_up(8 * (cn + 1), a16) * a16, c_bytes = o_msg + mbytes;
      if (cn <= ctx->small_max && c_bytes <= kCompactBytes) {
        if ((r = ensure_pinned(ctx->h_msg[sl], c_bytes + 16)) || (r = ensure(ctx->d_msg[sl], c_bytes + 16))) return r;
        char* hb = (char*)ctx->h_msg[sl].p;
        const auto t0 = clk::now();
        memcpy(hb, sig + sig_stride * c0, sig_stride * cn);
        memcpy(hb + o_key, keys + key_bytes * c0, key_bytes * cn);
        memcpy(hb + o_off, msg_off + c0, 8 * (cn + 1));
        if (mbytes) memcpy(hb + o_msg, msgs + m0, mbytes);
        stage_s += std::chrono::duration<double>(clk::now() - t0).count();
        hipStream_t st = ctx->stream;
        const bool zc = keyed && !slots && ctx->small_zero_copy;  // the kernel reads hb over PCIe
        char* db = zc ? hb : (char*)ctx->d_msg[sl].p;
        if (!zc) HIP_TRY(hipMemcpyAsync(db, hb, c_bytes, hipMemcpyHostToDevice, st));
        ctx->last_h2d_bytes += c_bytes;
        void* d_sig_use = db;
        if (slots) {
          hipLaunchKernelGGL(edv_b58_sig_kernel, dim3((uint32_t)div_up(cn, kBlock)), dim3(kBlock), 0, st,
                             (const uint8_t*)db, cn, (uint8_t*)ctx->d_sig[sl].p);
          HIP_TRY(hipGetLastError());
          d_sig_use = ctx->d_sig[sl].p;
        }
        const uint64_t* d_off = (const uint64_t*)(db + o_off);
        const uint8_t* d_msg_base = (const uint8_t*)db + o_msg - m0;
        set_bucketing(ctx, ctx->bucket_mode == 2 && lengths_mixed(msg_off + c0, cn));
        if (keyed) {  // verdict bytes straight into the slot's pinned host buffer
          if ((r = ensure_pinned(ctx->h_bits[sl], cn))) return r;
          r = launch_small(ctx, d_sig_use, db + o_key, d_msg_base, d_off, d_off + 1, cn, nullptr, st,
                           (uint8_t*)ctx->h_bits[sl].p);
        } else {
          r = launch_pipeline(ctx, keyed, d_sig_use, db + o_key, d_msg_base, d_off, d_off + 1, cn, ctx->d_bits[sl].p,
                              st);
        }
        if (r) return r;
        if (!keyed)
          HIP_TRY(hipMemcpyAsync(ctx->h_bits[sl].p, ctx->d_bits[sl].p, 8 * nwords, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipEventRecord(ctx->ev_done[sl], st));
        ctx->slot_use[sl] = edv_ctx::SlotUse{ticket, c0, cn, keyed};
        continue;
      }
      const uint8_t *s_sig, *s_key, *s_msg, *s_off;
      if ((r = source(sig_direct, ctx->h_sig[sl], sig + sig_stride * c0, sig_stride * cn, true, &s_sig)) ||
          (r = source(key_direct, ctx->h_key[sl], keys + key_bytes * c0, key_bytes * cn, false, &s_key)) ||
          (r = source(msg_direct, ctx->h_msg[sl], msgs ? msgs + m0 : nullptr, mbytes, true, &s_msg)) ||
          (r = source(off_direct, ctx->h_off[sl], (const uint8_t*)(msg_off + c0), 8 * (cn + 1), false, &s_off)))
        return r;
      set_bucketing(ctx, ctx->bucket_mode == 2 && lengths_mixed(msg_off + c0, cn));
      hipStream_t cs = ctx->stream_copy;
      void* d_sig_in = slots ? ctx->d_slot[sl].p : ctx->d_sig[sl].p;
      HIP_TRY(hipMemcpyAsync(d_sig_in, s_sig, sig_stride * cn, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipMemcpyAsync(ctx->d_key[sl].p, s_key, key_bytes * cn, hipMemcpyHostToDevice, cs));
      if (mbytes) HIP_TRY(hipMemcpyAsync(ctx->d_msg[sl].p, s_msg, mbytes, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipMemcpyAsync(ctx->d_off[sl].p, s_off, 8 * (cn + 1), hipMemcpyHostToDevice, cs));
      HIP_TRY(hipEventRecord(ctx->ev_h2d[sl], cs));
      ctx->last_h2d_bytes += sig_stride * cn + key_bytes * cn + mbytes + 8 * (cn + 1);
      hipStream_t st = ctx->stream;
      HIP_TRY(hipStreamWaitEvent(st, ctx->ev_h2d[sl], 0));
      if (slots) {
        hipLaunchKernelGGL(edv_b58_sig_kernel, dim3((uint32_t)div_up(cn, kBlock)), dim3(kBlock), 0, st,
                           (const uint8_t*)ctx->d_slot[sl].p, cn, (uint8_t*)ctx->d_sig[sl].p);
        HIP_TRY(hipGetLastError());
      }
      const uint64_t* d_off = (const uint64_t*)ctx->d_off[sl].p;
      // the offsets are the caller's (starting at m0): the kernels address msgs + off[i]
      const uint8_t* d_msg_base = (const uint8_t*)ctx->d_msg[sl].p - m0;
      if (keyed && cn <= ctx->small_max)
        r = launch_small(ctx, ctx->d_sig[sl].p, ctx->d_key[sl].p, d_msg_base, d_off, d_off + 1, cn, ctx->d_bits[sl].p,
                         st);
      else
        r = launch_pipeline(ctx, keyed, ctx->d_sig[sl].p, ctx->d_key[sl].p, d_msg_base, d_off, d_off + 1, cn,
                            ctx->d_bits[sl].p, st);
      if (r) return r;
      HIP_TRY(hipMemcpyAsync(ctx->h_bits[sl].p, ctx->d_bits[sl].p, 8 * nwords, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipEventRecord(ctx->ev_done[sl], st));
      ctx->slot_use[sl] = edv_ctx::SlotUse{ticket, c0, cn};
    }
    return 0;
  };
  int r = run();
  ctx->last_stage_ms = stage_s * 1e3;
  ctx->last_call_ms = std::chrono::duration<double, std::milli>(clk::now() - t_call).count();
  if (r) {  // nothing of a failed submission stays queued
    for (int sl = 0; sl < edv_ctx::kSlots; ++sl)
      if (ctx->slot_use[sl].ticket == ticket) (void)drain_slot(ctx, sl);
    for (size_t k = 0; k < ctx->pending.size(); ++k)
      if (ctx->pending[k].ticket == ticket) {
        ctx->pending.erase(ctx->pending.begin() + (long)k);
        break;
      }
    return r;
  }
  *ticket_out = ticket;
  return 0;
}

static int host_collect(edv_ctx* ctx, uint64_t ticket, uint8_t* accept_bits) {
  size_t k = 0;
  while (k < ctx->pending.size() && ctx->pending[k].ticket != ticket) ++k;
  if (k == ctx->pending.size()) return set_err(EDV_EINVAL, "no pending submission %llu", (unsigned long long)ticket);
  int r;
  for (int sl = 0; sl < edv_ctx::kSlots; ++sl)
    if (ctx->slot_use[sl].ticket == ticket && (r = drain_slot(ctx, sl))) return r;
  edv_ctx::Pending& p = ctx->pending[k];
  const uint64_t n = p.n;
  if (n) {
    memcpy(accept_bits, p.bits.data(), (size_t)((n + 7) / 8));
    if (n & 7) accept_bits[n / 8] &= (uint8_t)((1u << (n & 7)) - 1);
  }
  ctx->pending.erase(ctx->pending.begin() + (long)k);
  return 0;
}

static int host_verify(edv_ctx* ctx, bool keyed, const uint8_t* sig, uint64_t sig_stride, const uint8_t* keys,
                       const uint8_t* msgs, const uint64_t* msg_off, uint64_t n, uint8_t* accept_bits) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  uint64_t ticket = 0;
  int r = host_submit(ctx, keyed, sig, sig_stride, keys, msgs, msg_off, n, &ticket);
  if (r) return r;
  r = host_collect(ctx, ticket, accept_bits);
  ctx->last_call_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  return r;
}

namespace edv_internal {
int begin(edv_ctx* ctx, hipStream_t* stream) {
  int r = set_device(ctx);
  if (r) return r;
  *stream = ctx->stream;
  return 0;
}
uint64_t& bls_pair_max(edv_ctx* ctx) { return ctx->bls_pair_max; }
uint64_t& bls_wave_max(edv_ctx* ctx) { return ctx->bls_wave_max; }
int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace edv_internal

extern "C" {

int edv_keys_add(edv_ctx* ctx, const uint8_t* pk32, uint64_t nkeys, uint64_t* first_id) {
  int r = set_device(ctx);
  if (r) return r;
  if (nkeys && !pk32) return set_err(EDV_EINVAL, "null pk32");
  if (ctx->key_count + nkeys > 0xffffffffull) return set_err(EDV_EINVAL, "too many keys");
  if ((r = keys_reserve(ctx, ctx->key_count + nkeys))) return r;
  const uint64_t first = ctx->key_count;
  if (nkeys) {
    HIP_TRY(hipMemcpyAsync(ctx->d_key_pk + 32 * first, pk32, 32 * nkeys, hipMemcpyHostToDevice, ctx->stream));
    if ((r = keys_build(ctx, first, nkeys, ctx->stream))) return r;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  ctx->key_count += nkeys;
  if (first_id) *first_id = first;
  return 0;
}

int edv_keys_add_device(edv_ctx* ctx, const void* d_pk32, uint64_t nkeys, uint64_t* first_id, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (nkeys && !d_pk32) return set_err(EDV_EINVAL, "null d_pk32");
  if (ctx->key_count + nkeys > 0xffffffffull) return set_err(EDV_EINVAL, "too many keys");
  if ((r = keys_reserve(ctx, ctx->key_count + nkeys))) return r;
  const uint64_t first = ctx->key_count;
  hipStream_t st = pick_stream(ctx, stream);
  if (nkeys) {
    HIP_TRY(hipMemcpyAsync(ctx->d_key_pk + 32 * first, d_pk32, 32 * nkeys, hipMemcpyDeviceToDevice, st));
    if ((r = keys_build(ctx, first, nkeys, st))) return r;
  }
  ctx->key_count += nkeys;
  if (first_id) *first_id = first;
  return 0;
}

int edv_keys_set(edv_ctx* ctx, uint64_t first_id, const uint8_t* pk32, uint64_t nkeys) {
  int r = set_device(ctx);
  if (r) return r;
  if (nkeys && !pk32) return set_err(EDV_EINVAL, "null pk32");
  if (first_id > ctx->key_count || nkeys > ctx->key_count - first_id)
    return set_err(EDV_EINVAL, "keys [%llu, %llu) outside the %llu registered", (unsigned long long)first_id,
                   (unsigned long long)(first_id + nkeys), (unsigned long long)ctx->key_count);
  if (nkeys) {
    // in-flight verifies may still read the old tables of these slots
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyAsync(ctx->d_key_pk + 32 * first_id, pk32, 32 * nkeys, hipMemcpyHostToDevice, ctx->stream));
    if ((r = keys_build(ctx, first_id, nkeys, ctx->stream))) return r;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  return 0;
}

// Asynchronous registration.  The pk upload and the table builds go on stream_build (its own
// scratch, b_build), an event closes each call, and the host returns at once; the caller routes a
// building id's requests elsewhere until edv_keys_ready says its ticket is done.
static int build_ticket(edv_ctx* ctx, uint64_t* ticket) {
  hipEvent_t ev = nullptr;
  HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const hipError_t e = hipEventRecord(ev, ctx->stream_build);
  if (e != hipSuccess) {
    (void)hipEventDestroy(ev);
    return set_err(EDV_EHIP, "hipEventRecord: %s", hipGetErrorString(e));
  }
  ctx->builds.push_back(edv_ctx::BuildEv{++ctx->build_ticket, ev});
  if (ticket) *ticket = ctx->build_ticket;
  return 0;
}

int edv_keys_add_async(edv_ctx* ctx, const uint8_t* pk32, uint64_t nkeys, uint64_t* first_id, uint64_t* ticket) {
  int r = set_device(ctx);
  if (r) return r;
  if (nkeys && !pk32) return set_err(EDV_EINVAL, "null pk32");
  if (ctx->key_count + nkeys > 0xffffffffull) return set_err(EDV_EINVAL, "too many keys");
  // a regrowth of the store waits for everything (it copies the built tables); rare: capacity doubles
  if ((r = keys_reserve(ctx, ctx->key_count + nkeys))) return r;
  const uint64_t first = ctx->key_count;
  if (nkeys) {
    HIP_TRY(hipMemcpyAsync(ctx->d_key_pk + 32 * first, pk32, 32 * nkeys, hipMemcpyHostToDevice, ctx->stream_build));
    if ((r = keys_build(ctx, first, nkeys, ctx->stream_build))) return r;
  }
  if ((r = build_ticket(ctx, ticket))) return r;
  ctx->key_count += nkeys;
  if (first_id) *first_id = first;
  return 0;
}

int edv_keys_set_async(edv_ctx* ctx, uint64_t first_id, const uint8_t* pk32, uint64_t nkeys, uint64_t* ticket) {
  int r = set_device(ctx);
  if (r) return r;
  if (nkeys && !pk32) return set_err(EDV_EINVAL, "null pk32");
  if (first_id > ctx->key_count || nkeys > ctx->key_count - first_id)
    return set_err(EDV_EINVAL, "keys [%llu, %llu) outside the %llu registered", (unsigned long long)first_id,
                   (unsigned long long)(first_id + nkeys), (unsigned long long)ctx->key_count);
  if (nkeys) {
    // the rebuild starts after the work already queued on the context's streams (verifies that may
    // still read these slots' old tables); the host does not wait
    hipStream_t qs[4] = {ctx->stream, ctx->stream2, ctx->stream_copy, ctx->stream_key};
    for (int k = 0; k < 4; ++k) {
      HIP_TRY(hipEventRecord(ctx->ev_fence[k], qs[k]));
      HIP_TRY(hipStreamWaitEvent(ctx->stream_build, ctx->ev_fence[k], 0));
    }
    HIP_TRY(hipMemcpyAsync(ctx->d_key_pk + 32 * first_id, pk32, 32 * nkeys, hipMemcpyHostToDevice,
                           ctx->stream_build));
    if ((r = keys_build(ctx, first_id, nkeys, ctx->stream_build))) return r;
  }
  return build_ticket(ctx, ticket);
}

int edv_keys_set_many_async(edv_ctx* ctx, const uint32_t* ids, const uint8_t* pk32, uint64_t nkeys,
                            uint64_t* ticket) {
  int r = set_device(ctx);
  if (r) return r;
  if (nkeys && (!ids || !pk32)) return set_err(EDV_EINVAL, "null pointer");
  for (uint64_t k = 0; k < nkeys; ++k)
    if (ids[k] >= ctx->key_count)
      return set_err(EDV_EINVAL, "key id %u outside the %llu registered", ids[k], (unsigned long long)ctx->key_count);
  {  // distinct ids: two builds of one slot in one launch would race
    std::vector<uint32_t> sorted(ids, ids + nkeys);
    std::sort(sorted.begin(), sorted.end());
    for (uint64_t k = 1; k < nkeys; ++k)
      if (sorted[k] == sorted[k - 1]) return set_err(EDV_EINVAL, "key id %u twice", sorted[k]);
  }
  if (nkeys) {
    const int slot = ctx->many_next;
    ctx->many_next = (slot + 1) % edv_ctx::kManyRing;
    edv_ctx::Buf &hb = ctx->h_many[slot], &db = ctx->d_many[slot];
    const uint64_t bytes = 36 * nkeys;  // encodings, then ids
    if (ctx->ev_many[slot]) HIP_TRY(hipEventSynchronize(ctx->ev_many[slot]));  // its last copy has read hb
    else HIP_TRY(hipEventCreateWithFlags(&ctx->ev_many[slot], hipEventDisableTiming));
    if ((r = ensure_pinned(hb, bytes))) return r;
    if (db.cap < bytes) {  // a build queued earlier may still read the old device buffer
      HIP_TRY(hipStreamSynchronize(ctx->stream_build));
      if ((r = ensure(db, bytes))) return r;
    }
    memcpy(hb.p, pk32, 32 * nkeys);
    memcpy((uint8_t*)hb.p + 32 * nkeys, ids, 4 * nkeys);
    // the rebuild starts after the work already queued on the context's streams (verifies that may
    // still read these slots' old tables); the host does not wait
    hipStream_t qs[4] = {ctx->stream, ctx->stream2, ctx->stream_copy, ctx->stream_key};
    for (int k = 0; k < 4; ++k) {
      HIP_TRY(hipEventRecord(ctx->ev_fence[k], qs[k]));
      HIP_TRY(hipStreamWaitEvent(ctx->stream_build, ctx->ev_fence[k], 0));
    }
    HIP_TRY(hipMemcpyAsync(db.p, hb.p, bytes, hipMemcpyHostToDevice, ctx->stream_build));
    HIP_TRY(hipEventRecord(ctx->ev_many[slot], ctx->stream_build));
    const uint8_t* d_pk = (const uint8_t*)db.p;
    const uint32_t* d_ids = (const uint32_t*)(d_pk + 32 * nkeys);
    edv_ctx::Buf& aux = ctx->b_build;
#define EDV_MANY_CASE(W)                                                                  \
  case W:                                                                                 \
    r = keys_build_ids_w<W>(ctx, d_pk, d_ids, nkeys, ctx->stream_build, aux);            \
    break;
    switch (ctx->key_w) {
      EDV_KEY_WINDOWS(EDV_MANY_CASE)
      default:
        return set_err(EDV_EINVAL, "key window %d", ctx->key_w);
    }
#undef EDV_MANY_CASE
    if (r) return r;
  }
  return build_ticket(ctx, ticket);
}

int edv_keys_ready(edv_ctx* ctx, uint64_t ticket) {
  if (!ctx) return set_err(EDV_EINVAL, "null context");  // (a query: the resident kernel stays)
  HIP_TRY(hipSetDevice(ctx->device));
  while (ticket > ctx->build_done && !ctx->builds.empty()) {
    const hipError_t e = hipEventQuery(ctx->builds.front().ev);
    if (e == hipErrorNotReady) return 0;
    if (e != hipSuccess) return set_err(EDV_EHIP, "key-table build: %s", hipGetErrorString(e));
    ctx->build_done = ctx->builds.front().ticket;
    (void)hipEventDestroy(ctx->builds.front().ev);
    ctx->builds.pop_front();
  }
  return ticket <= ctx->build_done ? 1 : 0;
}

int edv_keys_sync(edv_ctx* ctx) {
  int r = set_device(ctx);
  if (r) return r;
  if (ctx->builds.empty()) return 0;
  HIP_TRY(hipStreamSynchronize(ctx->stream_build));
  return edv_keys_ready(ctx, ctx->build_ticket) == 1 ? 0 : set_err(EDV_EHIP, "key-table builds did not drain");
}

uint64_t edv_keys_count(edv_ctx* ctx) { return ctx ? ctx->key_count : 0; }

int edv_keys_reset(edv_ctx* ctx) {
  int r = set_device(ctx);
  if (r) return r;
  // a pending asynchronous build must not write a slot the next registration reuses
  if ((r = edv_keys_sync(ctx))) return r;
  ctx->key_count = 0;
  return 0;
}

int edv_keys_set_window(edv_ctx* ctx, int w) {
  int r = set_device(ctx);
  if (r) return r;
  if (!key_window_ok(w)) return set_err(EDV_EINVAL, "key window %d (4, 6, 8, 10, 12, 13, 14 or 16)", w);
  if (ctx->key_count) return set_err(EDV_EINVAL, "key window change with %llu keys registered (edv_keys_reset first)",
                                     (unsigned long long)ctx->key_count);
  if (w == ctx->key_w) return 0;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  if ((r = edv_keys_sync(ctx))) return r;
  if (ctx->d_key_tab) (void)hipFree(ctx->d_key_tab);
  if (ctx->d_key_pk) (void)hipFree(ctx->d_key_pk);
  if (ctx->d_key_valid) (void)hipFree(ctx->d_key_valid);
  ctx->d_key_tab = nullptr;
  ctx->d_key_pk = nullptr;
  ctx->d_key_valid = nullptr;
  ctx->key_cap = 0;
  ctx->key_w = w;
  return 0;
}

int edv_keys_window(edv_ctx* ctx) { return ctx ? ctx->key_w : -1; }

int edv_verify_batch_keyed_device(edv_ctx* ctx, const void* d_sig64, const void* d_key_idx, const void* d_msgs,
                                  const void* d_msg_off, uint64_t n, void* d_accept_words, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n && (!d_sig64 || !d_key_idx || !d_msgs || !d_msg_off || !d_accept_words))
    return set_err(EDV_EINVAL, "null device pointer");
  set_bucketing(ctx, false);
  return launch_verify_keyed(ctx, d_sig64, d_key_idx, d_msgs, d_msg_off, n, d_accept_words, pick_stream(ctx, stream));
}

int edv_verify_spans_device(edv_ctx* ctx, const void* d_sig64, const void* d_keys, int keyed, const void* d_msgs,
                            const void* d_msg_start, const void* d_msg_end, uint64_t n, void* d_accept_words,
                            void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n && (!d_sig64 || !d_keys || !d_msgs || !d_msg_start || !d_msg_end || !d_accept_words))
    return set_err(EDV_EINVAL, "null device pointer");
  if (n && keyed && ctx->key_count == 0) return set_err(EDV_EINVAL, "no registered keys");
  set_bucketing(ctx, false);
  return launch_pipeline(ctx, keyed != 0, d_sig64, d_keys, d_msgs, (const uint64_t*)d_msg_start,
                         (const uint64_t*)d_msg_end, n, d_accept_words, pick_stream(ctx, stream));
}

int edv_verify_batch_keyed(edv_ctx* ctx, const uint8_t* sig64, const uint32_t* key_idx, const uint8_t* msgs,
                           const uint64_t* msg_off, uint64_t n, uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!sig64 || !key_idx || !msg_off || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  return host_verify(ctx, true, sig64, 64, (const uint8_t*)key_idx, msgs, msg_off, n, accept_bits);
}

inline void cpu_relax() { __builtin_ia32_pause(); }

// edv_verify_one through the resident kernel: 0 with *accept set, 1 when this request must take the
// launch path instead (message too long, resident path off or broken), or an EDV_E* error.
int verify_one_resident(edv_ctx* ctx, const uint8_t* sig64, uint32_t key_id, const uint8_t* msg, uint64_t mlen,
                        uint8_t* accept) {
  if (!ctx->res_on || mlen > kResMsgMax || ctx->key_count == 0) return 1;
  using rclk = std::chrono::steady_clock;
  if (!ctx->res_box) {
    HIP_TRY(hipSetDevice(ctx->device));
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(ResBox), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      ctx->res_on = false;
      return 1;
    }
    memset(p, 0, sizeof(ResBox));
    ctx->res_box = (ResBox*)p;
  }
  ResBox* b = ctx->res_box;
  auto wait_gone = [&]() -> int {  // a kernel asked to leave: until it has (bounded: it polls every ~us)
    const auto t0 = rclk::now();
    while (__atomic_load_n(&b->running, __ATOMIC_ACQUIRE) != 0) {
      if (rclk::now() - t0 > std::chrono::seconds(2)) {
        HIP_TRY(hipStreamSynchronize(ctx->stream_res));
        break;
      }
      cpu_relax();
    }
    ctx->res_launched = ctx->res_stopping = false;
    return 0;
  };
  int r;
  if (ctx->res_launched && ctx->res_w != ctx->key_w && !ctx->res_stopping) {  // another window: another kernel
    __atomic_store_n(&b->stop, (uint64_t)1, __ATOMIC_RELEASE);
    ctx->res_stopping = true;
  }
  if (ctx->res_launched && ctx->res_stopping && (r = wait_gone())) return r;
  auto launch = [&](uint64_t answered) -> int {  // answered: the last request the host has its verdict of
    HIP_TRY(hipSetDevice(ctx->device));  // (only here: a request to a running kernel makes no HIP call)
    __atomic_store_n(&b->stop, (uint64_t)0, __ATOMIC_RELAXED);
    __atomic_store_n(&b->done_seq, answered, __ATOMIC_RELAXED);
    __atomic_store_n(&b->running, 1u, __ATOMIC_RELEASE);
    // idle exit after 200 us without a request (100 MHz wall clock): a burst of cache misses keeps it,
    // and anything queued behind it on a shared hardware queue waits at most that long
    const uint64_t idle = 20000;
#define EDV_RES_CASE(W)                                                                                   \
  case W:                                                                                                 \
    hipLaunchKernelGGL(edv_resident_kernel<W>, dim3(1), dim3(kSmallThreads), 0, ctx->stream_res, b,      \
                       ctx->d_btab_comb32, ctx->d_ident, idle);                                           \
    break;
    switch (ctx->key_w) {
      EDV_KEY_WINDOWS(EDV_RES_CASE)
      default:
        __atomic_store_n(&b->running, 0u, __ATOMIC_RELEASE);
        return set_err(EDV_EINVAL, "key window %d", ctx->key_w);
    }
#undef EDV_RES_CASE
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      __atomic_store_n(&b->running, 0u, __ATOMIC_RELEASE);
      return set_err(EDV_EHIP, "resident kernel launch: %s", hipGetErrorString(e));
    }
    ctx->res_launched = true;
    ctx->res_stopping = false;
    ctx->res_w = ctx->key_w;
    ++ctx->res_launches;
    return 0;
  };
  if (ctx->res_launched && __atomic_load_n(&b->running, __ATOMIC_ACQUIRE) == 0) ctx->res_launched = false;  // idled out
  if (!ctx->res_launched && (r = launch(ctx->res_seq))) return r;
  // the request, then its number
  b->mlen = mlen;
  b->key_id = key_id;
  b->key_count = (uint32_t)ctx->key_count;
  b->key_tab = ctx->d_key_tab;
  b->key_pk = ctx->d_key_pk;
  b->key_valid = ctx->d_key_valid;
  b->key_cap = ctx->key_cap;
  memcpy(b->sig, sig64, 64);
  if (mlen) memcpy(b->msg, msg, (size_t)mlen);
  const uint64_t seq = ++ctx->res_seq;
  __atomic_store_n(&b->req_seq, seq, __ATOMIC_RELEASE);
  const auto t0 = rclk::now();
  uint32_t spins = 0;
  while (__atomic_load_n(&b->done_seq, __ATOMIC_ACQUIRE) != seq) {
    cpu_relax();
    if ((++spins & 255) != 0) continue;
    if (__atomic_load_n(&b->running, __ATOMIC_ACQUIRE) == 0 &&
        __atomic_load_n(&b->done_seq, __ATOMIC_ACQUIRE) != seq) {
      // it idled out just before the request arrived: a fresh kernel picks the request up
      ctx->res_launched = false;
      if ((r = launch(seq - 1))) return r;
    }
    if (rclk::now() - t0 > std::chrono::seconds(5)) {  // never expected: stop using it on this context
      resident_yield(ctx);
      ctx->res_on = false;
      return set_err(EDV_EHIP, "resident kernel did not answer request %llu within 5 s", (unsigned long long)seq);
    }
  }
  *accept = __atomic_load_n(&b->verdict, __ATOMIC_ACQUIRE) ? 1 : 0;
  ++ctx->res_served;
  return 0;
}

int edv_verify_one(edv_ctx* ctx, const uint8_t* sig64, uint32_t key_id, const uint8_t* msg, uint64_t mlen,
                   uint8_t* accept) {
  if (!ctx) return set_err(EDV_EINVAL, "null context");
  if (!sig64 || !accept || (mlen && !msg)) return set_err(EDV_EINVAL, "null pointer");
  const int r = verify_one_resident(ctx, sig64, key_id, msg, mlen, accept);
  if (r <= 0) return r;
  // the launch path: one request through edv_verify_small_kernel
  uint64_t off[2] = {0, mlen};
  *accept = 0;
  return edv_verify_batch_keyed(ctx, sig64, &key_id, msg, off, 1, accept);
}

int edv_verify_batch_keyed_slots(edv_ctx* ctx, const uint8_t* sig_slots, const uint32_t* key_idx, const uint8_t* msgs,
                                 const uint64_t* msg_off, uint64_t n, uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!sig_slots || !key_idx || !msg_off || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  return host_verify(ctx, true, sig_slots, EDV_SIG_SLOT96, (const uint8_t*)key_idx, msgs, msg_off, n, accept_bits);
}

int edv_verify_batch_slots(edv_ctx* ctx, const uint8_t* sig_slots, const uint8_t* pk32, const uint8_t* msgs,
                           const uint64_t* msg_off, uint64_t n, uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!sig_slots || !pk32 || !msg_off || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  return host_verify(ctx, false, sig_slots, EDV_SIG_SLOT96, pk32, msgs, msg_off, n, accept_bits);
}

int edv_stage_reserve(edv_ctx* ctx, uint64_t bytes) {
  int r = set_device(ctx);
  if (r) return r;
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  if (ctx->set_ticket[ctx->cur_set])
    return set_err(EDV_EBUSY, "staging set %d holds an uncollected submission", ctx->cur_set);
  ctx->stage_err = 0;
  ctx->last_ok[ctx->cur_set] = false;  // the puts that follow overwrite the last batch's messages
  if (ctx->d_stage().cap < bytes) {
    HIP_TRY(hipStreamSynchronize(ctx->stream_copy));  // earlier puts may still write the old buffer
    HIP_TRY(hipStreamSynchronize(ctx->stream));       // ... and earlier verifies read it
    if ((r = ensure(ctx->d_stage(), bytes))) return r;
  }
  return 0;
}

int edv_stage_select(edv_ctx* ctx, int set) {
  int r = set_device(ctx);
  if (r) return r;
  if (set < 0 || set >= edv_ctx::kSets) return set_err(EDV_EINVAL, "staging set %d (0 or 1)", set);
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  ctx->cur_set = set;
  return 0;
}

int edv_stage_put(edv_ctx* ctx, const void* src, uint64_t nbytes, uint64_t off) {
  if (!ctx) return set_err(EDV_EINVAL, "null context");
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  if (!nbytes) return 0;
  int r = 0;
  if (!src || off > ctx->d_stage().cap || nbytes > ctx->d_stage().cap - off)
    r = set_err(EDV_EINVAL, "stage_put [%llu, +%llu) outside the %llu-byte staging buffer", (unsigned long long)off,
                (unsigned long long)nbytes, (unsigned long long)ctx->d_stage().cap);
  else if (!pinned_range(src, nbytes))
    r = set_err(EDV_EINVAL, "stage_put source is not edv_host_alloc memory");
  else if (hipSetDevice(ctx->device) != hipSuccess ||
           hipMemcpyAsync((char*)ctx->d_stage().p + off, src, nbytes, hipMemcpyHostToDevice, ctx->stream_copy) !=
               hipSuccess)
    r = set_err(EDV_EHIP, "stage_put copy failed");
  if (r && !ctx->stage_err) ctx->stage_err = r;
  return r;
}

int edv_verify_staged_submit(edv_ctx* ctx, int keyed, const uint8_t* keys, uint64_t slot_off, uint64_t msg_base,
                             const uint64_t* msg_start, const uint64_t* msg_end, uint64_t n, uint64_t* ticket) {
  int r = set_device(ctx);
  if (r) return r;
  if (!ticket || (n && (!keys || !msg_start || !msg_end))) return set_err(EDV_EINVAL, "null pointer");
  const int set = ctx->cur_set;
  {
    std::lock_guard<std::mutex> lk(ctx->stage_mu);
    if (ctx->stage_err) return set_err(ctx->stage_err, "an earlier stage_put failed");
    if (ctx->set_ticket[set]) return set_err(EDV_EBUSY, "staging set %d holds an uncollected submission", set);
  }
  if (keyed && n && ctx->key_count == 0) return set_err(EDV_EINVAL, "no registered keys");
  const uint64_t cap = ctx->d_stage().cap;
  if (n && (slot_off > cap || n > (cap - slot_off) / EDV_SIG_SLOT96)) return set_err(EDV_EINVAL, "slots outside staging");
  uint64_t bad = 0;  // the kernels read msg_base + [start, end): inside the staging buffer
  for (uint64_t i = 0; i < n; ++i) bad |= (uint64_t)(msg_start[i] > msg_end[i]) | (uint64_t)(msg_end[i] > cap - msg_base);
  if (bad) return set_err(EDV_EINVAL, "a message span outside staging");
  const uint64_t key_bytes = keyed ? 4 : 32, nwords = div_up(n, 64);
  if ((r = ensure_pinned(ctx->sh_bits[set], 8 * nwords + 8)) || (r = ensure(ctx->s_key[set], key_bytes * n)) ||
      (r = ensure(ctx->d_spans[set], 16 * n)) || (r = ensure(ctx->s_sig[set], 64 * n)) ||
      (r = ensure(ctx->s_bits[set], 8 * nwords)))
    return r;
  const uint64_t tk = ctx->next_ticket++;
  if (n) {
    // the key ids and the spans straight from the caller's memory when it is pinned (the
    // authenticator gathers the ids and the scan writes the spans, starts then ends, into
    // edv_host_alloc blocks); else through the set's pinned staging, copied by the pooled threads
    const bool keys_direct = pinned_range(keys, key_bytes * n);
    const bool spans_direct = msg_end == msg_start + n && pinned_range(msg_start, 16 * n);
    const void* src_key = keys;
    const void* src_spans = msg_start;
    if (!keys_direct) {
      if ((r = ensure_pinned(ctx->sh_key[set], key_bytes * n))) return r;
      stage_copy(ctx->sh_key[set].p, keys, key_bytes * n);
      src_key = ctx->sh_key[set].p;
    }
    if (!spans_direct) {
      if ((r = ensure_pinned(ctx->sh_off[set], 16 * n))) return r;
      stage_copy(ctx->sh_off[set].p, msg_start, 8 * n);
      stage_copy((char*)ctx->sh_off[set].p + 8 * n, msg_end, 8 * n);
      src_spans = ctx->sh_off[set].p;
    }
    ctx->last_direct = (keys_direct ? 2 : 0) | (spans_direct ? 8 : 0);
    hipStream_t cs = ctx->stream_copy, st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->s_key[set].p, src_key, key_bytes * n, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipMemcpyAsync(ctx->d_spans[set].p, src_spans, 16 * n, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipEventRecord(ctx->ev_sh2d[set], cs));  // after every put queued before this call
    HIP_TRY(hipStreamWaitEvent(st, ctx->ev_sh2d[set], 0));
    const uint8_t* stage = (const uint8_t*)ctx->d_stage().p;
    hipLaunchKernelGGL(edv_b58_sig_kernel, dim3((uint32_t)div_up(n, kBlock)), dim3(kBlock), 0, st, stage + slot_off,
                       n, (uint8_t*)ctx->s_sig[set].p);
    HIP_TRY(hipGetLastError());
    const uint64_t* ms = (const uint64_t*)ctx->d_spans[set].p;
    set_bucketing(ctx, false);
    if (keyed && n <= ctx->small_max)
      r = launch_small(ctx, ctx->s_sig[set].p, ctx->s_key[set].p, stage + msg_base, ms, ms + n, n,
                       ctx->s_bits[set].p, st);
    else
      r = launch_pipeline(ctx, keyed != 0, ctx->s_sig[set].p, ctx->s_key[set].p, stage + msg_base, ms, ms + n, n,
                          ctx->s_bits[set].p, st);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(ctx->sh_bits[set].p, ctx->s_bits[set].p, 8 * nwords, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(ctx->ev_sdone[set], st));
  }
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  ctx->set_ticket[set] = tk;
  ctx->set_n[set] = n;
  ctx->last_n[set] = n;
  ctx->last_msg_base[set] = msg_base;
  ctx->last_ok[set] = n > 0;
  *ticket = tk;
  return 0;
}

int edv_verify_staged_begin(edv_ctx* ctx, int keyed, uint64_t n, uint64_t* ticket) {
  int r = set_device(ctx);
  if (r) return r;
  if (!ticket) return set_err(EDV_EINVAL, "null pointer");
  const int set = ctx->cur_set;
  {
    std::lock_guard<std::mutex> lk(ctx->stage_mu);
    if (ctx->set_ticket[set]) return set_err(EDV_EBUSY, "staging set %d holds an uncollected submission", set);
    if (ctx->part_set >= 0) return set_err(EDV_EINVAL, "a batch of parts is open (set %d)", ctx->part_set);
  }
  if (keyed && n && ctx->key_count == 0) return set_err(EDV_EINVAL, "no registered keys");
  const uint64_t key_bytes = keyed ? 4 : 32, nwords = div_up(n, 64);
  // every buffer the parts use, sized here on the caller's thread (the parts only launch)
  if ((r = ensure_pinned(ctx->sh_bits[set], 8 * nwords + 8)) || (r = ensure(ctx->s_key[set], key_bytes * n)) ||
      (r = ensure(ctx->d_spans[set], 16 * n)) || (r = ensure(ctx->s_sig[set], 64 * n)) ||
      (r = ensure(ctx->s_bits[set], 8 * nwords)))
    return r;
  if (n) HIP_TRY(hipMemsetAsync(ctx->s_bits[set].p, 0, 8 * nwords, ctx->stream));
  set_bucketing(ctx, false);
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  const uint64_t tk = ctx->next_ticket++;
  ctx->set_ticket[set] = tk;
  ctx->set_n[set] = n;
  ctx->last_ok[set] = false;  // (a speculative batch's parts may not cover it: no subsets of it)
  ctx->part_set = set;
  ctx->part_keyed = keyed != 0;
  ctx->part_err = 0;
  ctx->part_msg.clear();
  ctx->part_launched = 0;
  *ticket = tk;
  return 0;
}

int edv_verify_staged_part(edv_ctx* ctx, const void* keys, uint64_t slot_off, uint64_t msg_base,
                           const uint64_t* spans, uint64_t n, uint64_t lo, uint64_t hi) {
  if (!ctx) return set_err(EDV_EINVAL, "null context");
  std::lock_guard<std::mutex> lk(ctx->stage_mu);  // one part at a time, ordered with the puts
  const int set = ctx->part_set;
  int r = 0;
  auto fail = [&](int code) {
    if (!ctx->part_err) {
      ctx->part_err = code;
      ctx->part_msg = g_err;  // (g_err is this thread's; edv_verify_staged_end reports it on the caller's)
    }
    return code;
  };
  if (set < 0) return fail(set_err(EDV_EINVAL, "no batch of parts is open"));
  if (ctx->part_err) return ctx->part_err;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(set_err(EDV_EHIP, "hipSetDevice"));
  if (n != ctx->set_n[set] || lo > hi || hi > n || (lo & 63) || !keys || !spans)
    return fail(set_err(EDV_EINVAL, "part [%llu, %llu) of %llu", (unsigned long long)lo, (unsigned long long)hi,
                        (unsigned long long)n));
  if (lo == hi) return 0;
  const uint64_t cap = ctx->d_stage_set[set].cap, m = hi - lo;
  if (ctx->stage_err) return fail(ctx->stage_err);
  if (slot_off > cap || hi > (cap - slot_off) / EDV_SIG_SLOT96) return fail(set_err(EDV_EINVAL, "slots outside staging"));
  const uint64_t *ms_h = spans + lo, *me_h = spans + n + lo;
  uint64_t bad = 0;  // the kernels read msg_base + [start, end): inside the staging buffer
  for (uint64_t i = 0; i < m; ++i) bad |= (uint64_t)(ms_h[i] > me_h[i]) | (uint64_t)(me_h[i] > cap - msg_base);
  if (bad) return fail(set_err(EDV_EINVAL, "a message span outside staging"));
  const bool keyed = ctx->part_keyed;
  const uint64_t key_bytes = keyed ? 4 : 32;
  if (!pinned_range((const uint8_t*)keys + key_bytes * lo, key_bytes * m) || !pinned_range(ms_h, 8 * m) ||
      !pinned_range(me_h, 8 * m))
    return fail(set_err(EDV_EINVAL, "part inputs are not edv_host_alloc memory"));
  hipStream_t cs = ctx->stream_copy, st = ctx->stream;
  uint64_t* d_ms = (uint64_t*)ctx->d_spans[set].p;
  uint8_t* d_key = (uint8_t*)ctx->s_key[set].p + key_bytes * lo;
  if (hipMemcpyAsync(d_key, (const uint8_t*)keys + key_bytes * lo, key_bytes * m, hipMemcpyHostToDevice, cs) ||
      hipMemcpyAsync(d_ms + lo, ms_h, 8 * m, hipMemcpyHostToDevice, cs) ||
      hipMemcpyAsync(d_ms + n + lo, me_h, 8 * m, hipMemcpyHostToDevice, cs) ||
      hipEventRecord(ctx->ev_sh2d[set], cs) ||  // after every put queued before this part
      hipStreamWaitEvent(st, ctx->ev_sh2d[set], 0))
    return fail(set_err(EDV_EHIP, "part copies"));
  const uint8_t* stage = (const uint8_t*)ctx->d_stage_set[set].p;
  uint8_t* sig = (uint8_t*)ctx->s_sig[set].p + 64 * lo;
  hipLaunchKernelGGL(edv_b58_sig_kernel, dim3((uint32_t)div_up(m, kBlock)), dim3(kBlock), 0, st,
                     stage + slot_off + EDV_SIG_SLOT96 * lo, m, sig);
  if (hipGetLastError() != hipSuccess) return fail(set_err(EDV_EHIP, "part b58 launch"));
  r = launch_pipeline(ctx, keyed, sig, d_key, stage + msg_base, d_ms + lo, d_ms + n + lo, m,
                      (unsigned long long*)ctx->s_bits[set].p + lo / 64, st);
  if (r) return fail(r);
  ++ctx->part_launched;
  return 0;
}

int edv_verify_staged_end(edv_ctx* ctx) {
  int r = set_device(ctx);
  if (r) return r;
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  const int set = ctx->part_set;
  if (set < 0) return set_err(EDV_EINVAL, "no batch of parts is open");
  ctx->part_set = -1;
  const uint64_t nwords = div_up(ctx->set_n[set], 64);
  if (nwords) {
    HIP_TRY(hipMemcpyAsync(ctx->sh_bits[set].p, ctx->s_bits[set].p, 8 * nwords, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipEventRecord(ctx->ev_sdone[set], ctx->stream));
  }
  if (ctx->part_err) return set_err(ctx->part_err, "a part of this batch failed: %s", ctx->part_msg.c_str());
  return 0;
}

int edv_verify_staged_collect(edv_ctx* ctx, uint64_t ticket, uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  int set = -1;
  for (int k = 0; k < edv_ctx::kSets; ++k)
    if (ticket && ctx->set_ticket[k] == ticket) set = k;
  if (set < 0) return set_err(EDV_EINVAL, "no staged submission %llu", (unsigned long long)ticket);
  const uint64_t n = ctx->set_n[set];
  if (n && !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  if (n) {
    HIP_TRY(hipEventSynchronize(ctx->ev_sdone[set]));
    memcpy(accept_bits, ctx->sh_bits[set].p, (size_t)((n + 7) / 8));
    if (n & 7) accept_bits[n / 8] &= (uint8_t)((1u << (n & 7)) - 1);
  }
  std::lock_guard<std::mutex> lk(ctx->stage_mu);
  ctx->set_ticket[set] = 0;
  ctx->set_n[set] = 0;
  return 0;
}

int edv_verify_staged(edv_ctx* ctx, int keyed, const uint8_t* keys, uint64_t slot_off, uint64_t msg_base,
                      const uint64_t* msg_start, const uint64_t* msg_end, uint64_t n, uint8_t* accept_bits) {
  if (n && !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  uint64_t ticket = 0;
  int r = edv_verify_staged_submit(ctx, keyed, keys, slot_off, msg_base, msg_start, msg_end, n, &ticket);
  if (r) return r;
  return edv_verify_staged_collect(ctx, ticket, accept_bits);
}

int edv_verify_staged_subset(edv_ctx* ctx, const uint32_t* idx, const uint8_t* pk32, uint64_t m,
                             uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  if (m == 0) return 0;
  if (!idx || !pk32 || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  const int set = ctx->cur_set;
  uint64_t n = 0, base = 0;
  {
    std::lock_guard<std::mutex> lk(ctx->stage_mu);
    if (ctx->set_ticket[set]) return set_err(EDV_EBUSY, "staging set %d holds an uncollected submission", set);
    if (!ctx->last_ok[set]) return set_err(EDV_EINVAL, "staging set %d holds no submitted staged batch", set);
    n = ctx->last_n[set];
    base = ctx->last_msg_base[set];
  }
  uint64_t bad = 0;
  for (uint64_t j = 0; j < m; ++j) bad |= (uint64_t)(idx[j] >= n);
  if (bad) return set_err(EDV_EINVAL, "a subset index outside the staged batch of %llu", (unsigned long long)n);
  const uint64_t nwords = div_up(m, 64);
  // the keys first (16-byte aligned for the general path's loads), then the indices
  if ((r = ensure_pinned(ctx->sub_h, 36 * m)) || (r = ensure(ctx->sub_d_in, 36 * m)) ||
      (r = ensure(ctx->sub_d_sig, 64 * m)) || (r = ensure(ctx->sub_d_spans, 16 * m)) ||
      (r = ensure(ctx->sub_d_words, 8 * nwords)) || (r = ensure_pinned(ctx->sub_h_bits, 8 * nwords)))
    return r;
  stage_copy(ctx->sub_h.p, pk32, 32 * m);
  stage_copy((uint8_t*)ctx->sub_h.p + 32 * m, idx, 4 * m);
  hipStream_t st = ctx->stream;
  HIP_TRY(hipMemcpyAsync(ctx->sub_d_in.p, ctx->sub_h.p, 36 * m, hipMemcpyHostToDevice, st));
  const uint8_t* d_pk = (const uint8_t*)ctx->sub_d_in.p;
  const uint32_t* d_idx = (const uint32_t*)(d_pk + 32 * m);
  uint64_t* d_sp = (uint64_t*)ctx->sub_d_spans.p;
  hipLaunchKernelGGL(edv_subset_gather_kernel, dim3((uint32_t)div_up(m, kBlock)), dim3(kBlock), 0, st, d_idx, m, n,
                     (const uint8_t*)ctx->s_sig[set].p, (const uint64_t*)ctx->d_spans[set].p,
                     (uint8_t*)ctx->sub_d_sig.p, d_sp);
  HIP_TRY(hipGetLastError());
  set_bucketing(ctx, false);
  r = launch_pipeline(ctx, false, ctx->sub_d_sig.p, d_pk, (const uint8_t*)ctx->d_stage_set[set].p + base, d_sp,
                      d_sp + m, m, ctx->sub_d_words.p, st);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(ctx->sub_h_bits.p, ctx->sub_d_words.p, 8 * nwords, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  memcpy(accept_bits, ctx->sub_h_bits.p, (size_t)((m + 7) / 8));
  if (m & 7) accept_bits[m / 8] &= (uint8_t)((1u << (m & 7)) - 1);
  return 0;
}

int edv_verify_submit(edv_ctx* ctx, int keyed, const uint8_t* sig, int sig_format, const uint8_t* keys,
                      const uint8_t* msgs, const uint64_t* msg_off, uint64_t n, uint64_t* ticket) {
  int r = set_device(ctx);
  if (r) return r;
  if (!ticket || !msg_off || (n && (!sig || !keys))) return set_err(EDV_EINVAL, "null pointer");
  if (sig_format != 64 && sig_format != EDV_SIG_SLOT96) return set_err(EDV_EINVAL, "sig_format %d", sig_format);
  return host_submit(ctx, keyed != 0, sig, (uint64_t)sig_format, keys, msgs, msg_off, n, ticket);
}

int edv_verify_collect(edv_ctx* ctx, uint64_t ticket, uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  if (!accept_bits) return set_err(EDV_EINVAL, "null accept_bits");
  return host_collect(ctx, ticket, accept_bits);
}

int edv_host_alloc(edv_ctx* ctx, uint64_t bytes, void** out) {
  int r = set_device(ctx);
  if (r) return r;
  if (!out) return set_err(EDV_EINVAL, "null out");
  *out = nullptr;
  if (bytes == 0) return set_err(EDV_EINVAL, "zero bytes");
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocPortable);
  if (e != hipSuccess) return set_err(EDV_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
  {
    std::lock_guard<std::mutex> g(g_pinned_mu);
    g_pinned.push_back(PinnedBlock{(const uint8_t*)p, (size_t)bytes});
  }
  *out = p;
  return 0;
}

int edv_host_free(void* p) {
  if (!p) return 0;
  {
    std::lock_guard<std::mutex> g(g_pinned_mu);
    size_t k = 0;
    while (k < g_pinned.size() && g_pinned[k].p != p) ++k;
    if (k == g_pinned.size()) return set_err(EDV_EINVAL, "not an edv_host_alloc block");
    g_pinned.erase(g_pinned.begin() + (long)k);
  }
  HIP_TRY(hipHostFree(p));
  return 0;
}


}  // extern "C"

extern "C" {

const char* edv_version(void) { return EDV_VERSION; }
int edv_base_window(void) { return kBaseW; }
const char* edv_last_error(void) { return g_err.c_str(); }

int edv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

edv_ctx* edv_create(int device) {
  int ndev = edv_device_count();
  if (device < 0 || device >= ndev) {
    set_err(EDV_ENODEV, "device %d out of range (%d HIP devices)", device, ndev);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_err(EDV_ENODEV, "device %d is not gfx950 (%s)", device, prop.gcnArchName);
    return nullptr;
  }
  edv_ctx* ctx = new edv_ctx();
  ctx->device = device;
  auto fail = [&](const char* what, hipError_t e) -> edv_ctx* {
    set_err(EDV_EHIP, "%s: %s", what, hipGetErrorString(e));
    edv_destroy(ctx);
    return nullptr;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
  // A blocking stream: it is ordered against the legacy NULL stream, which is
  // where PyTorch's default-stream copies that produce our inputs run.
  if ((e = hipStreamCreate(&ctx->stream)) != hipSuccess) return fail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking)) != hipSuccess)
    return fail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithFlags(&ctx->stream_copy, hipStreamNonBlocking)) != hipSuccess)
    return fail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithFlags(&ctx->stream_key, hipStreamNonBlocking)) != hipSuccess)
    return fail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithFlags(&ctx->stream_build, hipStreamNonBlocking)) != hipSuccess)
    return fail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithFlags(&ctx->stream_res, hipStreamNonBlocking)) != hipSuccess)
    return fail("hipStreamCreate", e);
  for (hipEvent_t& f : ctx->ev_fence)
    if ((e = hipEventCreateWithFlags(&f, hipEventDisableTiming)) != hipSuccess) return fail("hipEventCreate", e);
  for (int sb = 0; sb < edv_ctx::kSub; ++sb)
    if ((e = hipEventCreateWithFlags(&ctx->ev_kfork[sb], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->ev_kjoin[sb], hipEventDisableTiming)) != hipSuccess)
      return fail("hipEventCreate", e);
  for (int k = 0; k < edv_ctx::kSets; ++k)
    if ((e = hipEventCreateWithFlags(&ctx->ev_sh2d[k], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->ev_sdone[k], hipEventDisableTiming)) != hipSuccess)
      return fail("hipEventCreate", e);
  for (int k = 0; k < edv_ctx::kSlots; ++k)
    if ((e = hipEventCreateWithFlags(&ctx->ev_h2d[k], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->ev_done[k], hipEventDisableTiming)) != hipSuccess)
      return fail("hipEventCreate", e);
  for (int sb = 0; sb < edv_ctx::kSub; ++sb)
    for (int k = 0; k < edv_ctx::kEv; ++k)
      if ((e = hipEventCreate(&ctx->ev_sub[sb][k])) != hipSuccess) return fail("hipEventCreate", e);
  for (int k = 0; k < 2; ++k)
    if ((e = hipEventCreateWithFlags(&ctx->ev_join[k], hipEventDisableTiming)) != hipSuccess)
      return fail("hipEventCreate", e);
  if ((e = hipMalloc(&ctx->d_btab_comb, sizeof(BASE_COMB_U32))) != hipSuccess) return fail("hipMalloc", e);
  if ((e = hipMalloc(&ctx->d_ident, sizeof(kNielsIdentityHost))) != hipSuccess) return fail("hipMalloc", e);
  if ((e = hipMemcpy(ctx->d_ident, kNielsIdentityHost, sizeof(kNielsIdentityHost), hipMemcpyHostToDevice)) !=
      hipSuccess)
    return fail("hipMemcpy", e);
  if ((e = hipMemcpy(ctx->d_btab_comb, BASE_COMB_U32, sizeof(BASE_COMB_U32), hipMemcpyHostToDevice)) != hipSuccess)
    return fail("hipMemcpy", e);
  {
    // W = 8 base-point comb table, built on the device by the key-table kernels
    constexpr int rowsB = Window<kBaseW>::kRows, EB = Window<kBaseW>::kEntries;
    uint32_t *rows = nullptr, *pre = nullptr;
    if ((e = hipMalloc(&ctx->d_btab_comb32, (size_t)kBaseTabWords * 4)) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc(&rows, rowsB * kRowWords * 4)) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc(&pre, (size_t)rowsB * EB * 10 * 4)) != hipSuccess) return fail("hipMalloc", e);
    hipLaunchKernelGGL(edv_base_rows_kernel, dim3(1), dim3(64), 0, ctx->stream, rows);
    hipLaunchKernelGGL(edv_comb_fill_kernel<kBaseW>, dim3((uint32_t)div_up(rowsB * FillShape<kBaseW>::NCH, kBlock)),
                       dim3(kBlock), 0, ctx->stream, rows, (uint64_t)rowsB, ctx->d_btab_comb32, pre, 0ull, 1ull);
    e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(rows);
    (void)hipFree(pre);
    if (e != hipSuccess) return fail("base table build", e);
  }
  ctx->scratch_lanes = kMaxLanes;
  if ((e = hipMalloc(&ctx->d_scratch, ctx->scratch_lanes / kBlock * (uint64_t)kRegionBytes)) != hipSuccess)
    return fail("hipMalloc(scratch)", e);
  if ((e = hipMalloc(&ctx->d_hsoa, ctx->scratch_lanes * 8 * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(h)", e);
  if ((e = hipMalloc(&ctx->d_flags, ctx->scratch_lanes)) != hipSuccess) return fail("hipMalloc(flags)", e);
  if ((e = hipMalloc(&ctx->d_pt, ctx->scratch_lanes * 30 * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(pt)", e);
  if ((e = hipMalloc(&ctx->d_pre, ctx->scratch_lanes * 10 * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(pre)", e);
  if ((e = hipMalloc(&ctx->d_perm, ctx->scratch_lanes * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(perm)", e);
  if ((e = hipMalloc(&ctx->d_kperm, ctx->scratch_lanes * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(kperm)", e);
  if ((e = hipMalloc(&ctx->d_ok8, ctx->scratch_lanes)) != hipSuccess) return fail("hipMalloc(ok8)", e);
  if ((e = hipMalloc(&ctx->d_lenkey, 2 * ctx->scratch_lanes)) != hipSuccess) return fail("hipMalloc(lenkey)", e);
  if ((e = hipMalloc(&ctx->d_dedup, 6 * ctx->scratch_lanes * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(dedup)", e);
  if ((e = hipMalloc(&ctx->d_key_ok, ctx->scratch_lanes)) != hipSuccess) return fail("hipMalloc(key_ok)", e);
  if ((e = hipMalloc(&ctx->d_ucount, edv_ctx::kSub * sizeof(uint32_t))) != hipSuccess)
    return fail("hipMalloc(ucount)", e);
  if ((e = rocprim::radix_sort_pairs_desc(nullptr, ctx->sort_tmp_bytes, ctx->d_lenkey, ctx->d_lenkey + kMaxLanes,
                                          rocprim::counting_iterator<uint32_t>(0), ctx->d_perm,
                                          (uint32_t)ctx->scratch_lanes, 0, kLenKeyBits, ctx->stream)) != hipSuccess)
    return fail("radix sort size", e);
  ctx->sort_tmp_bytes = (ctx->sort_tmp_bytes + 255) & ~(size_t)255;
  if ((e = hipMalloc(&ctx->d_sort_tmp, edv_ctx::kSub * ctx->sort_tmp_bytes)) != hipSuccess)
    return fail("hipMalloc(sort)", e);
  if (const char* w = getenv("EDV_KEY_WINDOW")) {
    const int kw = atoi(w);
    if (key_window_ok(kw)) ctx->key_w = kw;
  }
  return ctx;
}

void edv_destroy(edv_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  resident_yield(ctx);  // the resident kernel leaves at its next poll; its stream is drained first
  if (ctx->stream_res) (void)hipStreamSynchronize(ctx->stream_res);
  if (ctx->stream_res) (void)hipStreamDestroy(ctx->stream_res);
  if (ctx->res_box) (void)hipHostFree(ctx->res_box);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream_copy) (void)hipStreamSynchronize(ctx->stream_copy);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  if (ctx->stream_key) (void)hipStreamSynchronize(ctx->stream_key);
  if (ctx->stream_build) (void)hipStreamSynchronize(ctx->stream_build);
  for (edv_ctx::Buf* b : {&ctx->b_sig, &ctx->b_pk, &ctx->b_msg, &ctx->b_off, &ctx->b_bits, &ctx->b_aux, &ctx->b_build,
                          &ctx->sub_h, &ctx->sub_d_in, &ctx->sub_d_sig, &ctx->sub_d_spans, &ctx->sub_d_words,
                          &ctx->sub_h_bits})
    free_buf(*b);
  for (int k = 0; k < edv_ctx::kSets; ++k) {
    for (edv_ctx::Buf* b : {&ctx->d_stage_set[k], &ctx->d_spans[k], &ctx->s_sig[k], &ctx->s_key[k], &ctx->s_bits[k],
                            &ctx->sh_key[k], &ctx->sh_off[k], &ctx->sh_bits[k]})
      free_buf(*b);
    if (ctx->ev_sh2d[k]) (void)hipEventDestroy(ctx->ev_sh2d[k]);
    if (ctx->ev_sdone[k]) (void)hipEventDestroy(ctx->ev_sdone[k]);
  }
  for (edv_ctx::BuildEv& b : ctx->builds) (void)hipEventDestroy(b.ev);
  for (int k = 0; k < edv_ctx::kManyRing; ++k) {
    free_buf(ctx->h_many[k]);
    free_buf(ctx->d_many[k]);
    if (ctx->ev_many[k]) (void)hipEventDestroy(ctx->ev_many[k]);
  }
  for (hipEvent_t f : ctx->ev_fence)
    if (f) (void)hipEventDestroy(f);
  for (int k = 0; k < edv_ctx::kSlots; ++k) {
    for (edv_ctx::Buf* b : {&ctx->h_sig[k], &ctx->h_key[k], &ctx->h_msg[k], &ctx->h_off[k], &ctx->h_bits[k],
                            &ctx->d_sig[k], &ctx->d_key[k], &ctx->d_msg[k], &ctx->d_off[k], &ctx->d_bits[k],
                            &ctx->d_slot[k]})
      free_buf(*b);
    if (ctx->ev_h2d[k]) (void)hipEventDestroy(ctx->ev_h2d[k]);
    if (ctx->ev_done[k]) (void)hipEventDestroy(ctx->ev_done[k]);
  }
  if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
  if (ctx->d_hsoa) (void)hipFree(ctx->d_hsoa);
  if (ctx->d_flags) (void)hipFree(ctx->d_flags);
  if (ctx->d_pt) (void)hipFree(ctx->d_pt);
  if (ctx->d_perm) (void)hipFree(ctx->d_perm);
  if (ctx->d_kperm) (void)hipFree(ctx->d_kperm);
  if (ctx->d_ok8) (void)hipFree(ctx->d_ok8);
  if (ctx->d_kbin) (void)hipFree(ctx->d_kbin);
  if (ctx->d_kscan_tmp) (void)hipFree(ctx->d_kscan_tmp);
  if (ctx->d_gunits) (void)hipFree(ctx->d_gunits);
  if (ctx->d_goff) (void)hipFree(ctx->d_goff);
  if (ctx->d_scan_tmp) (void)hipFree(ctx->d_scan_tmp);
  if (ctx->d_arena) (void)hipFree(ctx->d_arena);
  if (ctx->d_lenkey) (void)hipFree(ctx->d_lenkey);
  if (ctx->d_dedup) (void)hipFree(ctx->d_dedup);
  if (ctx->d_key_ok) (void)hipFree(ctx->d_key_ok);
  if (ctx->d_ucount) (void)hipFree(ctx->d_ucount);
  if (ctx->d_sort_tmp) (void)hipFree(ctx->d_sort_tmp);
  if (ctx->d_ident) (void)hipFree(ctx->d_ident);
  if (ctx->d_pre) (void)hipFree(ctx->d_pre);
  if (ctx->d_btab_comb) (void)hipFree(ctx->d_btab_comb);
  if (ctx->d_btab_comb32) (void)hipFree(ctx->d_btab_comb32);
  if (ctx->d_key_pk) (void)hipFree(ctx->d_key_pk);
  if (ctx->d_key_valid) (void)hipFree(ctx->d_key_valid);
  if (ctx->d_key_tab) (void)hipFree(ctx->d_key_tab);
  for (int sb = 0; sb < edv_ctx::kSub; ++sb) {
    for (int k = 0; k < edv_ctx::kEv; ++k)
      if (ctx->ev_sub[sb][k]) (void)hipEventDestroy(ctx->ev_sub[sb][k]);
    if (ctx->ev_kfork[sb]) (void)hipEventDestroy(ctx->ev_kfork[sb]);
    if (ctx->ev_kjoin[sb]) (void)hipEventDestroy(ctx->ev_kjoin[sb]);
  }
  for (int k = 0; k < 2; ++k)
    if (ctx->ev_join[k]) (void)hipEventDestroy(ctx->ev_join[k]);
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->stream_key) (void)hipStreamDestroy(ctx->stream_key);
  if (ctx->stream_copy) (void)hipStreamDestroy(ctx->stream_copy);
  if (ctx->stream_build) (void)hipStreamDestroy(ctx->stream_build);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int edv_synchronize(edv_ctx* ctx) {
  int r = set_device(ctx);
  if (r) return r;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int edv_verify_batch_device(edv_ctx* ctx, const void* d_sig64, const void* d_pk32, const void* d_msgs,
                            const void* d_msg_off, uint64_t n, void* d_accept_words, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n && (!d_sig64 || !d_pk32 || !d_msgs || !d_msg_off || !d_accept_words))
    return set_err(EDV_EINVAL, "null device pointer");
  set_bucketing(ctx, false);
  return launch_verify(ctx, d_sig64, d_pk32, d_msgs, d_msg_off, n, d_accept_words, pick_stream(ctx, stream));
}

// Options and statistics (include/edverify.h: edv_options, edv_stats).
namespace {
int phases_into(edv_ctx* ctx, double* out4) {  // the last timed launch's phase sums (waits for its events)
  for (int k = 0; k < 4; ++k) out4[k] = 0.0;
  if (ctx->small_timed) {  // launch_small: the one kernel is the comb phase
    float t = 0.f;
    HIP_TRY(hipEventSynchronize(ctx->ev_sub[0][3]));
    HIP_TRY(hipEventElapsedTime(&t, ctx->ev_sub[0][0], ctx->ev_sub[0][3]));
    out4[2] = t;
    return 0;
  }
  for (int sb = 0; sb < ctx->last_nsub; ++sb) {
    HIP_TRY(hipEventSynchronize(ctx->ev_sub[sb][edv_ctx::kEv - 1]));
    for (int k = 0; k < edv_ctx::kEv - 1; ++k) {
      float t = 0.f;
      HIP_TRY(hipEventElapsedTime(&t, ctx->ev_sub[sb][k], ctx->ev_sub[sb][k + 1]));
      out4[k] += t;
    }
  }
  return 0;
}
}  // namespace

void edv_default_options(edv_options* out) {
  if (!out) return;
  memset(out, 0, sizeof *out);
  out->pipeline = 1;
  out->length_buckets = 2;
  out->key_sort = 2;
  out->resident = 1;
  out->small_batch = 256;
  out->unit_arena_bytes = kMaxLanes * 80ull * sizeof(Chunk16);
  out->bls_pair_lanes = 32768;
  out->bls_wave_checks = 8192;
}

int edv_get_options(edv_ctx* ctx, edv_options* out) {
  if (!ctx || !out) return set_err(EDV_EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  out->pipeline = ctx->max_sub;
  out->length_buckets = ctx->bucket_mode;
  out->key_sort = ctx->key_sort;
  out->resident = ctx->res_on ? 1 : 0;
  out->small_batch = ctx->small_max;
  out->unit_arena_bytes = ctx->arena_want * sizeof(Chunk16);
  out->bls_pair_lanes = ctx->bls_pair_max;
  out->bls_wave_checks = ctx->bls_wave_max;
  return 0;
}

int edv_set_options(edv_ctx* ctx, const edv_options* o) {
  if (!ctx || !o) return set_err(EDV_EINVAL, "null argument");
  // every field checked before any is applied: a refused call leaves the context as it was
  if (o->pipeline < 1 || o->pipeline > edv_ctx::kSub)
    return set_err(EDV_EINVAL, "pipeline %d (1..%d sub-batches)", o->pipeline, edv_ctx::kSub);
  if (o->length_buckets < 0 || o->length_buckets > 3)
    return set_err(EDV_EINVAL, "length_buckets %d (0 off, 1 on, 2 auto, 3 on + packed units)", o->length_buckets);
  if (o->key_sort < 0 || o->key_sort > 2) return set_err(EDV_EINVAL, "key_sort %d (0 off, 1 on, 2 auto)", o->key_sort);
  if (o->resident < 0 || o->resident > 1) return set_err(EDV_EINVAL, "resident %d (0 off, 1 on)", o->resident);
  if (o->small_batch > 65536)
    return set_err(EDV_EINVAL, "small_batch %llu (at most 65536)", (unsigned long long)o->small_batch);
  if (!o->resident) resident_yield(ctx);
  ctx->max_sub = o->pipeline;
  ctx->bucket_mode = o->length_buckets;
  ctx->key_sort = o->key_sort;
  ctx->res_on = o->resident != 0;
  ctx->small_max = o->small_batch;
  ctx->arena_want = o->unit_arena_bytes / sizeof(Chunk16);
  ctx->bls_pair_max = o->bls_pair_lanes;
  ctx->bls_wave_max = o->bls_wave_checks;
  return 0;
}

int edv_get_stats(edv_ctx* ctx, edv_stats* out) {
  if (!ctx || !out) return set_err(EDV_EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  if (ctx->timed) {
    int r = phases_into(ctx, out->phase_ms);
    if (r) return r;
    out->phases_valid = 1;
  }
  out->launch_count = ctx->last_nsub;
  out->chunk_items = ctx->last_chunk_n;
  out->host_call_ms = ctx->last_call_ms;
  out->host_stage_ms = ctx->last_stage_ms;
  out->host_h2d_bytes = ctx->last_h2d_bytes;
  out->host_direct = (uint32_t)ctx->last_direct;
  out->resident_launches = ctx->res_launches;
  out->resident_served = ctx->res_served;
  out->resident_service_us = ctx->res_box ? (double)__atomic_load_n(&ctx->res_box->service_ticks, __ATOMIC_ACQUIRE) / 100.0
                                          : 0.0;
  return 0;
}

#if EDV_SMALL_PROFILE
int edv_small_profile(uint64_t* out10) {  // probe builds only (not in include/edverify.h)
  HIP_TRY(hipMemcpyFromSymbol(out10, HIP_SYMBOL(g_small_prof), 10 * sizeof(uint64_t)));
  return 0;
}
#endif

int edv_verify_batch(edv_ctx* ctx, const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msgs,
                     const uint64_t* msg_off, uint64_t n, uint8_t* accept_bits) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!sig64 || !pk32 || !msg_off || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  return host_verify(ctx, false, sig64, 64, pk32, msgs, msg_off, n, accept_bits);
}

int edv_sign_open_batch(edv_ctx* ctx, const uint8_t* sm, const uint64_t* sm_off, const uint8_t* pk32, uint64_t n,
                        uint8_t* accept_bits) {
  if (!ctx) return set_err(EDV_EINVAL, "null context");
  if (n == 0) return 0;
  if (!sm_off || !pk32 || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  // crypto_sign_open: smlen < 64 -> reject; else sig = sm[0:64], m = sm[64:].
  std::vector<uint8_t> sig(64 * n, 0), too_short(n, 0), msgs;
  std::vector<uint64_t> off(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = sm_off[i], b = sm_off[i + 1];
    if (b < a) return set_err(EDV_EINVAL, "sm_off[%llu] decreasing", (unsigned long long)i);
    if (b - a < 64) {
      too_short[i] = 1;
    } else {
      if (!sm) return set_err(EDV_EINVAL, "null sm");
      memcpy(&sig[64 * i], sm + a, 64);
      msgs.insert(msgs.end(), sm + a + 64, sm + b);
    }
    off[i + 1] = msgs.size();
  }
  int r = edv_verify_batch(ctx, sig.data(), pk32, msgs.data(), off.data(), n, accept_bits);
  if (r) return r;
  for (uint64_t i = 0; i < n; ++i)
    if (too_short[i]) accept_bits[i / 8] &= (uint8_t)~(1u << (i % 8));
  return 0;
}

int edv_seed_keypair_batch(edv_ctx* ctx, const uint8_t* seeds32, uint64_t n, uint8_t* pk32_out, uint8_t* sk64_out) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!seeds32 || !pk32_out || !sk64_out) return set_err(EDV_EINVAL, "null pointer");
  if ((r = ensure(ctx->b_sig, 64 * n)) || (r = ensure(ctx->b_pk, 32 * n)) || (r = ensure(ctx->b_aux, 32 * n))) return r;
  hipStream_t st = ctx->stream;
  HIP_TRY(hipMemcpyAsync(ctx->b_aux.p, seeds32, 32 * n, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(edv_keypair_kernel, dim3((uint32_t)div_up(n, kBlock)), dim3(kBlock), 0, st,
                     (const uint8_t*)ctx->b_aux.p, n, ctx->d_btab_comb, (uint8_t*)ctx->b_pk.p, (uint8_t*)ctx->b_sig.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(pk32_out, ctx->b_pk.p, 32 * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(sk64_out, ctx->b_sig.p, 64 * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return 0;
}

int edv_sign_batch_device(edv_ctx* ctx, const void* d_sk64, const void* d_key_idx, const void* d_msgs,
                          const void* d_msg_off, uint64_t n, void* d_sig64_out, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!d_sk64 || !d_key_idx || !d_msgs || !d_msg_off || !d_sig64_out) return set_err(EDV_EINVAL, "null device pointer");
  hipStream_t st = pick_stream(ctx, stream);
  const uint64_t* off = (const uint64_t*)d_msg_off;
  hipLaunchKernelGGL(edv_sign_kernel, dim3((uint32_t)div_up(n, kBlock)), dim3(kBlock), 0, st, (const uint8_t*)d_sk64,
                     (const uint32_t*)d_key_idx, (const uint8_t*)d_msgs, off, off + 1, n, ctx->d_btab_comb,
                     (uint8_t*)d_sig64_out);
  HIP_TRY(hipGetLastError());
  return 0;
}

int edv_sign_spans_device(edv_ctx* ctx, const void* d_sk64, const void* d_key_idx, const void* d_msgs,
                          const void* d_msg_start, const void* d_msg_end, uint64_t n, void* d_sig64_out,
                          void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!d_sk64 || !d_key_idx || !d_msgs || !d_msg_start || !d_msg_end || !d_sig64_out)
    return set_err(EDV_EINVAL, "null device pointer");
  hipStream_t st = pick_stream(ctx, stream);
  hipLaunchKernelGGL(edv_sign_kernel, dim3((uint32_t)div_up(n, kBlock)), dim3(kBlock), 0, st, (const uint8_t*)d_sk64,
                     (const uint32_t*)d_key_idx, (const uint8_t*)d_msgs, (const uint64_t*)d_msg_start,
                     (const uint64_t*)d_msg_end, n, ctx->d_btab_comb, (uint8_t*)d_sig64_out);
  HIP_TRY(hipGetLastError());
  return 0;
}

int edv_sha256_spans_device(edv_ctx* ctx, const void* d_msgs, const void* d_msg_start, const void* d_msg_end,
                            uint64_t n, void* d_out32, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!d_msgs || !d_msg_start || !d_msg_end || !d_out32) return set_err(EDV_EINVAL, "null device pointer");
  hipStream_t st = pick_stream(ctx, stream);
  hipLaunchKernelGGL(edv_sha256_kernel, dim3((uint32_t)div_up(n, kBlock)), dim3(kBlock), 0, st,
                     (const uint8_t*)d_msgs, (const uint64_t*)d_msg_start, (const uint64_t*)d_msg_end, n,
                     (uint8_t*)d_out32);
  HIP_TRY(hipGetLastError());
  return 0;
}

int edv_sha256_batch(edv_ctx* ctx, const uint8_t* msgs, const uint64_t* msg_off, uint64_t n, uint8_t* out32) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!msg_off || !out32) return set_err(EDV_EINVAL, "null pointer");
  for (uint64_t i = 0; i < n; ++i)
    if (msg_off[i + 1] < msg_off[i]) return set_err(EDV_EINVAL, "msg_off[%llu] decreasing", (unsigned long long)i);
  const uint64_t m0 = msg_off[0], mbytes = msg_off[n] - m0;
  if (mbytes && !msgs) return set_err(EDV_EINVAL, "null msgs");
  if ((r = ensure(ctx->b_msg, mbytes + 16)) || (r = ensure(ctx->b_off, 8 * (n + 1))) || (r = ensure(ctx->b_sig, 32 * n)))
    return r;
  hipStream_t st = ctx->stream;
  std::vector<uint64_t> off(n + 1);
  for (uint64_t i = 0; i <= n; ++i) off[i] = msg_off[i] - m0;
  if (mbytes) HIP_TRY(hipMemcpyAsync(ctx->b_msg.p, msgs + m0, mbytes, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->b_off.p, off.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
  const uint64_t* d_off = (const uint64_t*)ctx->b_off.p;
  if ((r = edv_sha256_spans_device(ctx, ctx->b_msg.p, d_off, d_off + 1, n, ctx->b_sig.p, st))) return r;
  HIP_TRY(hipMemcpyAsync(out32, ctx->b_sig.p, 32 * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return 0;
}

int edv_sign_batch(edv_ctx* ctx, const uint8_t* sk64, const uint32_t* key_idx, const uint8_t* msgs,
                   const uint64_t* msg_off, uint64_t n, uint8_t* sig64_out) {
  int r = set_device(ctx);
  if (r) return r;
  if (n == 0) return 0;
  if (!sk64 || !key_idx || !msg_off || !sig64_out) return set_err(EDV_EINVAL, "null pointer");
  uint32_t nkeys = 0;
  for (uint64_t i = 0; i < n; ++i) nkeys = key_idx[i] + 1 > nkeys ? key_idx[i] + 1 : nkeys;
  const uint64_t m0 = msg_off[0], mbytes = msg_off[n] - m0;
  std::vector<uint64_t> off(n + 1);
  for (uint64_t i = 0; i <= n; ++i) off[i] = msg_off[i] - m0;
  if ((r = ensure(ctx->b_sig, 64 * n)) || (r = ensure(ctx->b_pk, 64 * (uint64_t)nkeys)) ||
      (r = ensure(ctx->b_msg, mbytes + 16)) || (r = ensure(ctx->b_off, 8 * (n + 1))) || (r = ensure(ctx->b_aux, 4 * n)))
    return r;
  hipStream_t st = ctx->stream;
  HIP_TRY(hipMemcpyAsync(ctx->b_pk.p, sk64, 64 * (uint64_t)nkeys, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->b_aux.p, key_idx, 4 * n, hipMemcpyHostToDevice, st));
  if (mbytes) HIP_TRY(hipMemcpyAsync(ctx->b_msg.p, msgs + m0, mbytes, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->b_off.p, off.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
  if ((r = edv_sign_batch_device(ctx, ctx->b_pk.p, ctx->b_aux.p, ctx->b_msg.p, ctx->b_off.p, n, ctx->b_sig.p, st)))
    return r;
  HIP_TRY(hipMemcpyAsync(sig64_out, ctx->b_sig.p, 64 * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return 0;
}

static void quorum_thresholds(uint32_t nv, uint32_t* q_prepare, uint32_t* q_commit) {
  // plenum/common/util.py:217-228 getMaxFailures; plenum/server/quorums.py:19-21
  const uint32_t f = nv >= 4 ? (nv - 1) / 3 : 0;
  *q_prepare = nv - f - 1;
  *q_commit = nv - f;
}

int edv_tally_finish_device(edv_ctx* ctx, const void* d_ballot, uint32_t n_keys, uint32_t n_validators,
                            void* d_counts, void* d_quorum, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n_keys == 0) return 0;
  if (!d_ballot || !d_counts || !d_quorum || n_validators == 0) return set_err(EDV_EINVAL, "bad tally arguments");
  uint32_t qp, qc;
  quorum_thresholds(n_validators, &qp, &qc);
  hipStream_t st = pick_stream(ctx, stream);
  hipLaunchKernelGGL(edv_tally_count_kernel, dim3((uint32_t)div_up(n_keys, kBlock)), dim3(kBlock), 0, st,
                     (const uint8_t*)d_ballot, n_keys, n_validators, qp, qc, (uint32_t*)d_counts, (uint8_t*)d_quorum);
  HIP_TRY(hipGetLastError());
  return 0;
}

int edv_tally_device(edv_ctx* ctx, const void* d_key, const void* d_voter, const void* d_phase, const void* d_valid,
                     const void* d_primary, uint64_t n_votes, uint32_t n_keys, uint32_t n_validators, void* d_ballot, void* d_counts,
                     void* d_quorum, void* stream) {
  int r = set_device(ctx);
  if (r) return r;
  if (n_keys == 0) return 0;
  if (!d_ballot || n_validators == 0 || n_validators > 255) return set_err(EDV_EINVAL, "bad tally arguments");
  hipStream_t st = pick_stream(ctx, stream);
  HIP_TRY(hipMemsetAsync(d_ballot, 0, (size_t)n_keys * 2 * n_validators, st));
  if (n_votes) {
    if (!d_key || !d_voter || !d_phase || !d_valid) return set_err(EDV_EINVAL, "null vote pointer");
    hipLaunchKernelGGL(edv_tally_scatter_kernel, dim3((uint32_t)div_up(n_votes, kBlock)), dim3(kBlock), 0, st,
                       (const uint32_t*)d_key, (const uint8_t*)d_voter, (const uint8_t*)d_phase,
                       (const uint8_t*)d_valid, (const uint8_t*)d_primary, n_votes, n_keys, n_validators,
                       (uint8_t*)d_ballot);
    HIP_TRY(hipGetLastError());
  }
  return edv_tally_finish_device(ctx, d_ballot, n_keys, n_validators, d_counts, d_quorum, st);
}

int edv_tally(edv_ctx* ctx, const uint32_t* key, const uint8_t* voter, const uint8_t* phase, const uint8_t* valid,
              const uint8_t* primary, uint64_t n_votes, uint32_t n_keys, uint32_t n_validators, uint32_t* counts_out, uint8_t* quorum_out) {
  int r = set_device(ctx);
  if (r) return r;
  if (n_keys == 0) return 0;
  if (!counts_out || !quorum_out) return set_err(EDV_EINVAL, "null output");
  void *d_key = nullptr, *d_voter = nullptr, *d_phase = nullptr, *d_valid = nullptr, *d_ballot = nullptr,
       *d_counts = nullptr, *d_quorum = nullptr, *d_primary = nullptr;
  auto cleanup = [&]() {
    for (void* p : {d_key, d_voter, d_phase, d_valid, d_ballot, d_counts, d_quorum, d_primary})
      if (p) (void)hipFree(p);
  };
  hipStream_t st = ctx->stream;
  const uint64_t nv = n_votes ? n_votes : 1;
  hipError_t e = hipSuccess;
  if ((e = hipMalloc(&d_key, 4 * nv)) || (e = hipMalloc(&d_voter, nv)) || (e = hipMalloc(&d_phase, nv)) ||
      (e = hipMalloc(&d_valid, nv)) || (e = hipMalloc(&d_ballot, (size_t)n_keys * 2 * n_validators + 16)) ||
      (e = hipMalloc(&d_counts, 8ull * n_keys)) || (e = hipMalloc(&d_quorum, n_keys)) ||
      (primary && (e = hipMalloc(&d_primary, n_keys)))) {
    cleanup();
    return set_err(EDV_ENOMEM, "hipMalloc: %s", hipGetErrorString(e));
  }
  if (primary && (e = hipMemcpyAsync(d_primary, primary, n_keys, hipMemcpyHostToDevice, st))) {
    cleanup();
    return set_err(EDV_EHIP, "hipMemcpyAsync: %s", hipGetErrorString(e));
  }
  if (n_votes) {
    if ((e = hipMemcpyAsync(d_key, key, 4 * n_votes, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(d_voter, voter, n_votes, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(d_phase, phase, n_votes, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(d_valid, valid, n_votes, hipMemcpyHostToDevice, st))) {
      cleanup();
      return set_err(EDV_EHIP, "hipMemcpyAsync: %s", hipGetErrorString(e));
    }
  }
  r = edv_tally_device(ctx, d_key, d_voter, d_phase, d_valid, d_primary, n_votes, n_keys, n_validators, d_ballot, d_counts,
                       d_quorum, st);
  if (!r) {
    if ((e = hipMemcpyAsync(counts_out, d_counts, 8ull * n_keys, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(quorum_out, d_quorum, n_keys, hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      r = set_err(EDV_EHIP, "tally copy-back: %s", hipGetErrorString(e));
  }
  cleanup();
  return r;
}

}  // extern "C"
