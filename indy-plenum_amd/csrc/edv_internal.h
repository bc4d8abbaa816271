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
}  // namespace edv_internal
