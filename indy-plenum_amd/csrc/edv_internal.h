// edv_internal.h -- shared between the translation units of
// libplenum_edverify.so (edverify.hip, bls.hip); not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

struct edv_ctx;

namespace edv_internal {
// Make the context's device current and hand back its stream (0 or EDV_E*).
int begin(edv_ctx* ctx, hipStream_t* stream);
// Record the error text for edv_last_error() and return code.
int set_err(int code, const char* fmt, ...);
// BLS verify batches of at most this many checks take two lanes per check (edv_bls_set_pair_lanes).
uint64_t& bls_pair_max(edv_ctx* ctx);
// ... and batches of at most this many one wave per check (edv_bls_set_wave_checks).
uint64_t& bls_wave_max(edv_ctx* ctx);
}  // namespace edv_internal
