"""ctypes binding of libplenum_edverify.so (C ABI: include/edverify.h).

This is the only way the Python package reaches the verifier: there is no CPU
fallback.  If the shared library is missing, or no gfx950 device is visible,
every verify call raises EdVerifyUnavailable (the product fails loudly rather
than silently verifying on the host)."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "PLENUM_EDVERIFY_LIB", os.path.join(os.path.dirname(_HERE), "libplenum_edverify.so"))

# Every symbol include/edverify.h declares, with its ctypes signature.
_c = ctypes
_P = _c.c_void_p
_U64 = _c.c_uint64
_U32 = _c.c_uint32
_I = _c.c_int
SIGNATURES = {
    "edv_version": (_c.c_char_p, []),
    "edv_base_window": (_c.c_int, []),
    "edv_last_error": (_c.c_char_p, []),
    "edv_device_count": (_I, []),
    "edv_create": (_P, [_I]),
    "edv_destroy": (None, [_P]),
    "edv_synchronize": (_I, [_P]),
    "edv_default_options": (None, [_P]),
    "edv_get_options": (_I, [_P, _P]),
    "edv_set_options": (_I, [_P, _P]),
    "edv_get_stats": (_I, [_P, _P]),
    "edv_verify_batch": (_I, [_P, _P, _P, _P, _P, _U64, _P]),
    "edv_sign_open_batch": (_I, [_P, _P, _P, _P, _U64, _P]),
    "edv_verify_batch_device": (_I, [_P, _P, _P, _P, _P, _U64, _P, _P]),
    "edv_stage_reserve": (_I, [_P, _U64]),
    "edv_stage_put": (_I, [_P, _P, _U64, _U64]),
    "edv_verify_staged": (_I, [_P, _I, _P, _U64, _U64, _P, _P, _U64, _P]),
    "edv_stage_select": (_I, [_P, _I]),
    "edv_verify_staged_submit": (_I, [_P, _I, _P, _U64, _U64, _P, _P, _U64, _P]),
    "edv_verify_staged_collect": (_I, [_P, _U64, _P]),
    "edv_verify_staged_begin": (_I, [_P, _I, _U64, _P]),
    "edv_verify_staged_part": (_I, [_P, _P, _U64, _U64, _P, _U64, _U64, _U64]),
    "edv_verify_staged_end": (_I, [_P]),
    "edv_verify_staged_subset": (_I, [_P, _P, _P, _U64, _P]),
    "edv_keys_add": (_I, [_P, _P, _U64, _P]),
    "edv_keys_add_device": (_I, [_P, _P, _U64, _P, _P]),
    "edv_keys_set": (_I, [_P, _U64, _P, _U64]),
    "edv_keys_add_async": (_I, [_P, _P, _U64, _P, _P]),
    "edv_keys_set_async": (_I, [_P, _U64, _P, _U64, _P]),
    "edv_keys_set_many_async": (_I, [_P, _P, _P, _U64, _P]),
    "edv_keys_ready": (_I, [_P, _U64]),
    "edv_keys_sync": (_I, [_P]),
    "edv_keys_count": (_U64, [_P]),
    "edv_keys_reset": (_I, [_P]),
    "edv_keys_set_window": (_I, [_P, _I]),
    "edv_keys_window": (_I, [_P]),
    "edv_verify_batch_keyed": (_I, [_P, _P, _P, _P, _P, _U64, _P]),
    "edv_verify_batch_keyed_device": (_I, [_P, _P, _P, _P, _P, _U64, _P, _P]),
    "edv_verify_one": (_I, [_P, _P, _U32, _P, _U64, _P]),
    "edv_verify_spans_device": (_I, [_P, _P, _P, _I, _P, _P, _P, _U64, _P, _P]),
    "edv_verify_batch_slots": (_I, [_P, _P, _P, _P, _P, _U64, _P]),
    "edv_verify_batch_keyed_slots": (_I, [_P, _P, _P, _P, _P, _U64, _P]),
    "edv_verify_submit": (_I, [_P, _I, _P, _I, _P, _P, _P, _U64, _P]),
    "edv_verify_collect": (_I, [_P, _U64, _P]),
    "edv_host_alloc": (_I, [_P, _U64, _P]),
    "edv_host_free": (_I, [_P]),
    "edv_seed_keypair_batch": (_I, [_P, _P, _U64, _P, _P]),
    "edv_sign_batch_device": (_I, [_P, _P, _P, _P, _P, _U64, _P, _P]),
    "edv_sign_spans_device": (_I, [_P, _P, _P, _P, _P, _P, _U64, _P, _P]),
    "edv_sign_batch": (_I, [_P, _P, _P, _P, _P, _U64, _P]),
    "edv_sha256_spans_device": (_I, [_P, _P, _P, _P, _U64, _P, _P]),
    "edv_sha256_batch": (_I, [_P, _P, _P, _U64, _P]),
    "edv_tally_device": (_I, [_P, _P, _P, _P, _P, _P, _U64, _U32, _U32, _P, _P, _P, _P]),
    "edv_tally_finish_device": (_I, [_P, _P, _U32, _U32, _P, _P, _P]),
    "edv_tally": (_I, [_P, _P, _P, _P, _P, _P, _U64, _U32, _U32, _P, _P]),
    "edv_bls_verify_batch": (_I, [_P, _P, _P, _P, _P, _P, _P, _U64, _P]),
    "edv_bls_aggregate": (_I, [_P, _P, _P, _U64, _P]),
    "edv_bls_sign_batch": (_I, [_P, _P, _P, _P, _U64, _P]),
    "edv_bls_keygen_batch": (_I, [_P, _P, _P, _U64, _P]),
}


class EdVerifyUnavailable(RuntimeError):
    """The HIP verify library or a gfx950 device is not available."""


class EdVerifyError(RuntimeError):
    """A library call returned a negative EDV_E* code."""

    def __init__(self, code, msg):
        super().__init__("edverify error %d: %s" % (code, msg))
        self.code = code


class EdvOptions(ctypes.Structure):
    """include/edverify.h edv_options."""
    _fields_ = [("pipeline", ctypes.c_int32), ("length_buckets", ctypes.c_int32), ("key_sort", ctypes.c_int32),
                ("resident", ctypes.c_int32), ("small_batch", ctypes.c_uint64), ("unit_arena_bytes", ctypes.c_uint64),
                ("bls_pair_lanes", ctypes.c_uint64), ("bls_wave_checks", ctypes.c_uint64)]


class EdvStats(ctypes.Structure):
    """include/edverify.h edv_stats."""
    _fields_ = [("phase_ms", ctypes.c_double * 4), ("launch_count", ctypes.c_int32), ("phases_valid", ctypes.c_int32),
                ("chunk_items", ctypes.c_uint64), ("host_call_ms", ctypes.c_double), ("host_stage_ms", ctypes.c_double),
                ("host_h2d_bytes", ctypes.c_uint64), ("host_direct", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("resident_launches", ctypes.c_uint64), ("resident_served", ctypes.c_uint64),
                ("resident_service_us", ctypes.c_double)]


EDV_EBUSY = -5  # include/edverify.h: the staging set holds an uncollected submission


class EdVerifyBusy(EdVerifyError):
    """EDV_EBUSY: the staging set holds an uncollected submission (not a fault:
    the caller collects it first or takes another path)."""


_lib = None


def load():
    """Load (once) and return the ctypes library; raises EdVerifyUnavailable."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).
    # Whichever loads first serves the whole process, so let torch's runtime
    # load first: device pointers and stream handles then come from the one
    # runtime both sides use.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise EdVerifyUnavailable(
            "libplenum_edverify.so not built at %s (run __graft_entry__.build())" % LIB_PATH)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as ex:
        raise EdVerifyUnavailable("cannot load %s: %s" % (LIB_PATH, ex)) from ex
    lenient = os.environ.get("PLENUM_EDVERIFY_LENIENT") == "1"  # A/B tools loading older builds
    for name, (res, args) in SIGNATURES.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(code):
    if code != 0:
        cls = EdVerifyBusy if code == EDV_EBUSY else EdVerifyError
        raise cls(code, load().edv_last_error().decode(errors="replace"))
