"""EdVerifyEngine: numpy / device-pointer front end of libplenum_edverify.so.

One engine = one HIP context = one GPU (include/edverify.h).  The verify
entry points replace per-request calls of
stp_core/crypto/nacl_wrappers.py:232-242 (Verifier.verify) with one batched
launch; verdicts are libsodium 1.0.18's (crypto_sign_verify_detached == 0).
"""
import contextlib
import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import EdVerifyError, EdVerifyUnavailable, check


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def _dev(x):
    """Device pointer from a torch tensor / int / None."""
    if x is None:
        return None
    if isinstance(x, int):
        return ctypes.c_void_p(x)
    return ctypes.c_void_p(x.data_ptr())


def _stream_for(stream, *tensors):
    """Explicit stream (torch.cuda.Stream / int handle) wins; otherwise, for
    torch tensors, torch's current stream on their device, so the launch is
    ordered after the torch ops that produced the inputs; otherwise NULL (the
    context's own stream)."""
    if stream is not None:
        return ctypes.c_void_p(stream if isinstance(stream, int) else stream.cuda_stream)
    for t in tensors:
        if hasattr(t, "device") and getattr(t.device, "type", None) == "cuda":
            import torch
            return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
    return None


def pack_messages(msgs):
    """list of bytes -> (uint8 buffer, uint64 offsets[n+1])."""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=len(msgs))
    off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    buf = np.frombuffer(b"".join(msgs), dtype=np.uint8) if len(msgs) else np.zeros(0, np.uint8)
    return buf, off


def _u8(x, width=None):
    """bytes / bytearray / list of bytes / array-like -> contiguous uint8 array
    (reshaped to (-1, width) when width is given)."""
    if isinstance(x, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(x), np.uint8)
    elif isinstance(x, (list, tuple)) and x and isinstance(x[0], (bytes, bytearray)):
        a = np.frombuffer(b"".join(x), np.uint8)
    else:
        a = np.asarray(x, dtype=np.uint8)
    a = np.ascontiguousarray(a)
    return a.reshape(-1, width) if width else a.reshape(-1)


def lengths_mixed(msg_start, msg_end):
    """The auto length-bucket rule of edverify.c (lengths_mixed) for callers of
    the device-pointer entry points that hold the lengths on the host: True
    when unsorted 64-lane waves would run > 1.25x the batch's SHA-512 blocks."""
    blocks = (np.asarray(msg_end, np.int64) - np.asarray(msg_start, np.int64) + 64 + 17 + 127) // 128
    n = blocks.size
    if n == 0:
        return False
    pad = (-n) % 64
    w = np.concatenate([blocks, np.zeros(pad, np.int64)]).reshape(-1, 64)
    cnt = np.full(w.shape[0], 64, np.int64)
    cnt[-1] = 64 - pad
    return 4 * int((w.max(axis=1) * cnt).sum()) > 5 * int(blocks.sum())


SIG_SLOT = 96  # edverify.h EDV_SIG_SLOT96


class _PinnedOwner:
    """Frees an edv_host_alloc block when the last array over it is gone."""
    __slots__ = ("lib", "ptr")

    def __init__(self, lib, ptr):
        self.lib, self.ptr = lib, ptr

    def __del__(self):
        try:
            self.lib.edv_host_free(ctypes.c_void_p(self.ptr))
        except Exception:
            pass


def unpack_bits(bits, n):
    return np.unpackbits(np.asarray(bits, dtype=np.uint8), bitorder="little")[:n].astype(bool)


class EdVerifyEngine:
    """Batched Ed25519 verify / sign / vote tally on one MI355X."""

    def __init__(self, device=0):
        lib = _lib.load()
        ndev = lib.edv_device_count()
        if ndev <= device:
            raise EdVerifyUnavailable("no HIP device %d (found %d)" % (device, ndev))
        ctx = lib.edv_create(device)
        if not ctx:
            raise EdVerifyUnavailable(lib.edv_last_error().decode(errors="replace"))
        self._lib = lib
        self._ctx = ctypes.c_void_p(ctx)
        self.device = device
        self._one_args = threading.local()  # verify_one_keyed's reusable ctypes arguments
        try:  # verify_one_keyed through the host extension: (function, edv_verify_one address, context)
            from ._hostpack import verify_one as _native_one
            self._one_native = (_native_one, ctypes.cast(self._lib.edv_verify_one, ctypes.c_void_p).value,
                                self._ctx.value)
        except (ImportError, AttributeError):
            self._one_native = None

    # ------------------------------------------------------------- lifecycle
    def close(self):
        self._one_native = None  # (it holds the context's address)
        if getattr(self, "_ctx", None):
            self._lib.edv_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def version(self):
        return self._lib.edv_version().decode()

    def synchronize(self):
        check(self._lib.edv_synchronize(self._ctx))

    # ---------------------------------------------------------------- verify
    def verify_bits(self, sig64, pk32, msgs, msg_off):
        """Packed accept bitmask ((n + 7) // 8 bytes, LSB-first)."""
        sig64 = _u8(sig64, 64)
        pk32 = _u8(pk32, 32)
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        n = sig64.shape[0]
        if pk32.shape[0] != n or msg_off.shape[0] != n + 1:
            raise ValueError("shape mismatch: sig %d, pk %d, off %d" % (n, pk32.shape[0], msg_off.shape[0]))
        if n and int(msg_off[-1]) > msgs.shape[0]:
            raise ValueError("msg_off exceeds message buffer")
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        if n:
            check(self._lib.edv_verify_batch(self._ctx, _ptr(sig64), _ptr(pk32), _ptr(msgs) if msgs.size else None,
                                             _ptr(msg_off), n, _ptr(bits)))
        return bits

    def verify_batch(self, sig64, pk32, msgs, msg_off, sig_slot=64):
        """Bool array: accepted[i] == (crypto_sign_verify_detached(...) == 0).
        sig_slot=96: sig64 holds EDV_SIG_SLOT96 slots (base58 text decoded on
        the GPU, edverify.h)."""
        if sig_slot == SIG_SLOT:
            return self._verify_slots(False, sig64, pk32, msgs, msg_off)
        sig64 = _u8(sig64, 64)
        return unpack_bits(self.verify_bits(sig64, pk32, msgs, msg_off), sig64.shape[0])

    supports_sig_slots = True

    def _verify_slots(self, keyed, slots, keys, msgs, msg_off):
        slots = _u8(slots, SIG_SLOT)
        keys = np.ascontiguousarray(keys, dtype=np.uint32) if keyed else _u8(keys, 32)
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        n = slots.shape[0]
        if keys.shape[0] != n or msg_off.shape[0] != n + 1:
            raise ValueError("shape mismatch: slots %d, keys %d, off %d" % (n, keys.shape[0], msg_off.shape[0]))
        if n and int(msg_off[-1]) > msgs.shape[0]:
            raise ValueError("msg_off exceeds message buffer")
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        if n:
            fn = self._lib.edv_verify_batch_keyed_slots if keyed else self._lib.edv_verify_batch_slots
            check(fn(self._ctx, _ptr(slots), _ptr(keys), _ptr(msgs) if msgs.size else None, _ptr(msg_off), n,
                     _ptr(bits)))
        return unpack_bits(bits, n)

    def verify_submit(self, sig, keys, msgs, msg_off, keyed, sig_slot=64):
        """Queue a host-pointer verify and return a handle for verify_collect
        (edv_verify_submit): inputs in host_alloc memory are read by DMA later
        and must not change until then (the handle keeps the arrays alive).
        keyed: keys are uint32 key ids, else n x 32 key bytes."""
        sig = _u8(sig, sig_slot)
        keys = np.ascontiguousarray(keys, dtype=np.uint32) if keyed else _u8(keys, 32)
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        n = sig.shape[0]
        if keys.shape[0] != n or msg_off.shape[0] != n + 1:
            raise ValueError("shape mismatch: sig %d, keys %d, off %d" % (n, keys.shape[0], msg_off.shape[0]))
        if n and int(msg_off[-1]) > msgs.shape[0]:
            raise ValueError("msg_off exceeds message buffer")
        ticket = ctypes.c_uint64()
        check(self._lib.edv_verify_submit(self._ctx, 1 if keyed else 0, _ptr(sig), int(sig_slot), _ptr(keys),
                                          _ptr(msgs) if msgs.size else None, _ptr(msg_off), n,
                                          ctypes.byref(ticket)))
        return (ticket.value, n, (sig, keys, msgs, msg_off))

    def verify_collect(self, handle):
        """Wait for a verify_submit and return its bool verdicts."""
        ticket, n, _keep = handle
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        check(self._lib.edv_verify_collect(self._ctx, ticket, _ptr(bits) if n else ctypes.c_void_p(1)))
        return unpack_bits(bits, n)

    # ------------------------------------------------------- staged inputs
    supports_staging = True

    def stage_reserve(self, nbytes):
        """A device staging buffer of >= nbytes (edv_stage_reserve)."""
        check(self._lib.edv_stage_reserve(self._ctx, int(nbytes)))

    def stager(self):
        """(edv_stage_put address, context address): what the native scan
        calls from its workers to queue each chunk's copies."""
        return (ctypes.cast(self._lib.edv_stage_put, ctypes.c_void_p).value, self._ctx.value)

    def verify_staged(self, keyed, keys, slot_off, msg_base, msg_start, msg_end):
        """Verdicts of n staged requests (edv_verify_staged): slots at staging
        offset slot_off, message i at msg_base + [msg_start[i], msg_end[i])."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32) if keyed else _u8(keys, 32)
        ms = np.ascontiguousarray(msg_start, dtype=np.uint64)
        me = np.ascontiguousarray(msg_end, dtype=np.uint64)
        n = ms.shape[0]
        if keys.shape[0] != n or me.shape[0] != n:
            raise ValueError("shape mismatch: keys %d, starts %d, ends %d" % (keys.shape[0], n, me.shape[0]))
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        check(self._lib.edv_verify_staged(self._ctx, 1 if keyed else 0, _ptr(keys), int(slot_off), int(msg_base),
                                          _ptr(ms), _ptr(me), n, _ptr(bits) if n else ctypes.c_void_p(1)))
        return unpack_bits(bits, n)

    def stage_select(self, staging_set):
        """Make staging set 0 or 1 current (edv_stage_select): batch k + 1 is
        staged into one set while batch k's kernels read the other."""
        check(self._lib.edv_stage_select(self._ctx, int(staging_set)))

    def verify_staged_submit(self, keyed, keys, slot_off, msg_base, msg_start, msg_end):
        """edv_verify_staged without the wait: a handle for verify_staged_collect.
        The inputs must stay untouched until the collect."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32) if keyed else _u8(keys, 32)
        ms = np.ascontiguousarray(msg_start, dtype=np.uint64)
        me = np.ascontiguousarray(msg_end, dtype=np.uint64)
        n = ms.shape[0]
        if keys.shape[0] != n or me.shape[0] != n:
            raise ValueError("shape mismatch: keys %d, starts %d, ends %d" % (keys.shape[0], n, me.shape[0]))
        ticket = ctypes.c_uint64()
        check(self._lib.edv_verify_staged_submit(self._ctx, 1 if keyed else 0, _ptr(keys), int(slot_off),
                                                 int(msg_base), _ptr(ms), _ptr(me), n, ctypes.byref(ticket)))
        return (ticket.value, n, (keys, ms, me))

    def verify_staged_collect(self, handle):
        """The verdicts of a verify_staged_submit (edv_verify_staged_collect)."""
        ticket, n, _keep = handle
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        check(self._lib.edv_verify_staged_collect(self._ctx, ticket, _ptr(bits) if n else ctypes.c_void_p(1)))
        return unpack_bits(bits, n)

    supports_staged_parts = True

    def verify_staged_begin(self, keyed, n):
        """Take the current staging set for an n-item batch verified in parts
        (edv_verify_staged_begin): a handle for verify_staged_collect once
        verify_staged_end has run."""
        ticket = ctypes.c_uint64()
        check(self._lib.edv_verify_staged_begin(self._ctx, 1 if keyed else 0, int(n), ctypes.byref(ticket)))
        return (ticket.value, int(n), None)

    def parter(self):
        """(edv_verify_staged_part address, context address): what the native
        scan's copier calls for each part of the batch it has staged."""
        return (ctypes.cast(self._lib.edv_verify_staged_part, ctypes.c_void_p).value, self._ctx.value)

    def verify_staged_end(self):
        """Queue the verdicts' copy after the last part (edv_verify_staged_end);
        raises if a part failed (collect the handle all the same)."""
        check(self._lib.edv_verify_staged_end(self._ctx))

    supports_staged_subset = True

    def verify_staged_subset(self, idx, pk32):
        """Verdicts of items idx of the last staged batch of the current set
        again, on the general path with their own key bytes pk32 (m x 32)
        (edv_verify_staged_subset): only idx and the keys cross PCIe."""
        idx = np.ascontiguousarray(idx, dtype=np.uint32)
        pk32 = _u8(pk32, 32)
        m = idx.shape[0]
        if pk32.shape[0] != m:
            raise ValueError("shape mismatch: idx %d, keys %d" % (m, pk32.shape[0]))
        bits = np.zeros((m + 7) // 8, dtype=np.uint8)
        if m:
            check(self._lib.edv_verify_staged_subset(self._ctx, _ptr(idx), _ptr(pk32), m, _ptr(bits)))
        return unpack_bits(bits, m)

    def host_alloc(self, nbytes):
        """nbytes of pinned host memory (edv_host_alloc) as a writable ctypes
        array; host-pointer verifies copy inputs inside it to the device with no
        staging copy.  Freed when the array (and every view of it) is gone."""
        p = ctypes.c_void_p()
        check(self._lib.edv_host_alloc(self._ctx, int(nbytes), ctypes.byref(p)))
        arr = (ctypes.c_ubyte * int(nbytes)).from_address(p.value)
        arr._owner = _PinnedOwner(self._lib, p.value)
        return arr

    def last_host_stats(self):
        """The last host-pointer verify: dict(call_ms, stage_ms, h2d_bytes,
        direct) -- stage_ms is the CPU copy into pinned staging (0 when every
        input came from host_alloc memory)."""
        st = self.stats()
        d = int(st["host_direct"])
        return {"call_ms": st["host_call_ms"], "stage_ms": st["host_stage_ms"], "h2d_bytes": int(st["host_h2d_bytes"]),
                "direct": {"sig": bool(d & 1), "keys": bool(d & 2), "msgs": bool(d & 4), "offsets": bool(d & 8)}}

    def sign_open_batch(self, sm, sm_off, pk32):
        """crypto_sign_open verdicts over signed messages sm_i = sig || msg
        (exactly VerifyKey.verify(signature + msg), nacl_wrappers.py:100-108)."""
        sm = _u8(sm)
        sm_off = np.ascontiguousarray(sm_off, dtype=np.uint64)
        pk32 = _u8(pk32, 32)
        n = pk32.shape[0]
        if sm_off.shape[0] != n + 1:
            raise ValueError("sm_off must have n + 1 entries")
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        if n:
            check(self._lib.edv_sign_open_batch(self._ctx, _ptr(sm) if sm.size else None, _ptr(sm_off), _ptr(pk32),
                                                n, _ptr(bits)))
        return unpack_bits(bits, n)

    def verify_batch_device(self, d_sig64, d_pk32, d_msgs, d_msg_off, n, d_accept_words, stream=None):
        """Asynchronous verify on device buffers (torch tensors or raw pointers)."""
        st = _stream_for(stream, d_sig64, d_accept_words)
        check(self._lib.edv_verify_batch_device(self._ctx, _dev(d_sig64), _dev(d_pk32), _dev(d_msgs),
                                                _dev(d_msg_off), n, _dev(d_accept_words), st))

    # ------------------------------------------------------- options / stats
    # edverify.h edv_options: every knob in one struct, read and written whole (edv_set_options checks
    # every field before applying any); options(**kw) sets some for a with-block and puts the previous
    # values back however the block ends.
    _OPTION_NAMES = ("pipeline", "length_buckets", "key_sort", "resident", "small_batch", "unit_arena_bytes",
                     "bls_pair_lanes", "bls_wave_checks")
    _MODES = {"length_buckets": {"auto": 2, "on": 1, "off": 0, "packed": 3}, "key_sort": {"auto": 2, "on": 1, "off": 0}}

    def get_options(self):
        o = _lib.EdvOptions()
        check(self._lib.edv_get_options(self._ctx, ctypes.byref(o)))
        return {k: getattr(o, k) for k in self._OPTION_NAMES}

    def set_options(self, **kw):
        """Change some options (names of edv_options; modes also as "auto" / "on" / "off" / "packed",
        booleans as 1 / 0); an invalid value raises and changes nothing."""
        unknown = set(kw) - set(self._OPTION_NAMES)
        if unknown:
            raise ValueError("unknown options: %s" % sorted(unknown))
        cur = self.get_options()
        for k, v in kw.items():
            cur[k] = int(self._MODES.get(k, {}).get(v, v))
        check(self._lib.edv_set_options(self._ctx, ctypes.byref(_lib.EdvOptions(**cur))))

    @contextlib.contextmanager
    def options(self, **kw):
        before = self.get_options()
        self.set_options(**kw)
        try:
            yield self
        finally:
            check(self._lib.edv_set_options(self._ctx, ctypes.byref(_lib.EdvOptions(**before))))

    @staticmethod
    def default_options():
        o = _lib.EdvOptions()
        _lib.load().edv_default_options(ctypes.byref(o))
        return {k: getattr(o, k) for k in EdVerifyEngine._OPTION_NAMES}

    def stats(self):
        """edv_get_stats as a dict (waits for the last timed launch's events)."""
        st = _lib.EdvStats()
        check(self._lib.edv_get_stats(self._ctx, ctypes.byref(st)))
        out = {k: getattr(st, k) for k, _ in _lib.EdvStats._fields_ if k not in ("phase_ms", "reserved")}
        out["phase_ms"] = tuple(st.phase_ms)
        return out

    def last_phases_ms(self):
        """(hash, table, dsm-or-comb, encode) milliseconds of the last verify
        launch, from HIP events on the launch streams: per phase the sum over
        the last chunk's sub-batch launches (see last_launch_count)."""
        st = self.stats()
        if not st["phases_valid"]:
            raise EdVerifyError(-1, "no timed verify launch yet")
        return st["phase_ms"]

    def last_phase_ms(self):
        """(hash, table, dsm) milliseconds of the last verify launch (HIP events)."""
        return self.last_phases_ms()[:3]

    def last_launch_count(self):
        """Kernel launches per phase (sub-batches) in the last verify chunk."""
        return int(self.stats()["launch_count"])

    def last_chunk_items(self):
        """Requests in the last verify chunk (what last_phases_ms covers)."""
        return int(self.stats()["chunk_items"])

    def set_pipeline(self, sub_batches):
        """Sub-batches per chunk (1..4; 1 = kernels run one at a time)."""
        self.set_options(pipeline=sub_batches)

    def set_small_batch(self, max_requests):
        """Keyed host-pointer verifies of at most max_requests requests take the
        low-latency kernel (default 256, 0 = never)."""
        self.set_options(small_batch=max_requests)

    def set_key_sort(self, mode):
        """Key-sorted comb order on the key-table path: False/0 off, True/1
        on, "auto"/2 (the default: sub-batches of 4,096 requests or more)."""
        self.set_options(key_sort=mode)

    def set_length_buckets(self, mode):
        """Hash lanes sorted by SHA-512 block count: False/0 off, True/1 on,
        "auto"/2 (the default; host-offset calls decide per batch, edverify.h),
        "packed"/3 sorted and packed into the length-bucketed SoA unit layout."""
        self.set_options(length_buckets=mode)

    def set_unit_arena(self, nbytes):
        """Unit-arena size of the packed mode in bytes (groups beyond it are
        hashed in place)."""
        self.set_options(unit_arena_bytes=nbytes)

    # ------------------------------------------------------------------ BLS
    # BN254 BLS (indy-crypto's Bls, bls_crypto_indy_crypto.py:59-90); G1 / G2
    # points as the 128-byte wire forms of edverify.h.
    def bls_verify_batch(self, sig128, msgs, msg_off, vk128, gen128, vk_off=None):
        """Bool array: e(sig_i, gen) == e(H(m_i), vk_i); with vk_off, vk_i is the
        sum of vk128[vk_off[i]:vk_off[i+1]] (verify_multi_sig)."""
        sig128 = _u8(sig128, 128)
        n = sig128.shape[0]
        vk128 = _u8(vk128, 128)
        gen128 = _u8(gen128)
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        if msg_off.shape[0] != n + 1 or gen128.size != 128:
            raise ValueError("msg_off needs n + 1 entries and gen 128 bytes")
        if vk_off is not None:
            vk_off = np.ascontiguousarray(vk_off, dtype=np.uint64)
            if vk_off.shape[0] != n + 1 or int(vk_off[-1]) > vk128.shape[0]:
                raise ValueError("vk_off needs n + 1 entries within vk128")
        elif vk128.shape[0] != n:
            raise ValueError("one verkey per item without vk_off")
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        if n:
            check(self._lib.edv_bls_verify_batch(self._ctx, _ptr(sig128), _ptr(msgs) if msgs.size else None,
                                                 _ptr(msg_off), _ptr(vk128), _ptr(vk_off), _ptr(gen128), n,
                                                 _ptr(bits)))
        return unpack_bits(bits, n)

    def bls_set_pair_lanes(self, max_checks):
        """Verify batches of at most max_checks use two lanes per check (lower
        latency); 0 = one lane per check always (edv_options.bls_pair_lanes)."""
        self.set_options(bls_pair_lanes=max_checks)

    def bls_set_wave_checks(self, max_checks):
        """Verify batches of at most max_checks run one wave per check (the
        check as a straight-line program over the wave's lanes: the latency
        form); 0 = never (edv_options.bls_wave_checks)."""
        self.set_options(bls_wave_checks=max_checks)

    def bls_aggregate(self, sig128, sig_off):
        """out[i] = sum of sig128[sig_off[i]:sig_off[i+1]] (create_multi_sig)."""
        sig128 = _u8(sig128, 128)
        sig_off = np.ascontiguousarray(sig_off, dtype=np.uint64)
        m = sig_off.shape[0] - 1
        out = np.zeros((m, 128), dtype=np.uint8)
        if m > 0:
            check(self._lib.edv_bls_aggregate(self._ctx, _ptr(sig128), _ptr(sig_off), m, _ptr(out)))
        return out

    def bls_sign_batch(self, sk32, msgs, msg_off):
        """[sk_i] H(m_i) as 128-byte G1 (sk: 32-byte big-endian scalars < r)."""
        sk32 = _u8(sk32, 32)
        n = sk32.shape[0]
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        out = np.zeros((n, 128), dtype=np.uint8)
        if n:
            check(self._lib.edv_bls_sign_batch(self._ctx, _ptr(sk32), _ptr(msgs) if msgs.size else None,
                                               _ptr(msg_off), n, _ptr(out)))
        return out

    def bls_keygen_batch(self, sk32, gen128):
        """[sk_i] gen as 128-byte G2 verkeys."""
        sk32 = _u8(sk32, 32)
        gen128 = _u8(gen128)
        n = sk32.shape[0]
        out = np.zeros((n, 128), dtype=np.uint8)
        if n:
            check(self._lib.edv_bls_keygen_batch(self._ctx, _ptr(sk32), _ptr(gen128), n, _ptr(out)))
        return out

    # ------------------------------------------------------------ key tables
    def keys_set_window(self, w):
        """Comb window of the key tables: 4 (64 KiB/key, 64 additions per
        verify), 6 (172 KiB, 43), 8 (512 KiB, 32), 10 (1.6 MiB, 26; the
        default), 12, 13 (10 MiB, 20), 14 or 16 (64 MiB, 16).  Only with no
        keys registered."""
        check(self._lib.edv_keys_set_window(self._ctx, int(w)))

    @property
    def keys_window(self):
        return int(self._lib.edv_keys_window(self._ctx))

    def keys_add(self, pk32):
        """Register public keys (a fixed-base comb table each, edverify.h);
        returns the first key id (ids are consecutive)."""
        pk32 = _u8(pk32, 32)
        first = ctypes.c_uint64()
        check(self._lib.edv_keys_add(self._ctx, _ptr(pk32), pk32.shape[0], ctypes.byref(first)))
        return first.value

    def keys_add_device(self, d_pk32, nkeys, stream=None):
        first = ctypes.c_uint64()
        check(self._lib.edv_keys_add_device(self._ctx, _dev(d_pk32), nkeys, ctypes.byref(first),
                                            _stream_for(stream, d_pk32)))
        return first.value

    def keys_set(self, first_id, pk32):
        """Rebuild registered slots first_id.. with new keys (LRU eviction)."""
        pk32 = _u8(pk32, 32)
        check(self._lib.edv_keys_set(self._ctx, int(first_id), _ptr(pk32), pk32.shape[0]))

    def keys_add_async(self, pk32):
        """Register keys without waiting for their tables (edv_keys_add_async):
        returns (first id, ticket); the ids may be used by keyed verifies only
        once keys_ready(ticket)."""
        pk32 = _u8(pk32, 32)
        first, ticket = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._lib.edv_keys_add_async(self._ctx, _ptr(pk32), pk32.shape[0], ctypes.byref(first),
                                           ctypes.byref(ticket)))
        return first.value, ticket.value

    def keys_set_many_async(self, ids, pk32):
        """Rebuild slots ids[k] (distinct) with keys pk32[k], all in one call,
        without waiting (edv_keys_set_many_async); returns the ticket."""
        pk32 = _u8(pk32, 32)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        if ids.shape[0] != pk32.shape[0]:
            raise ValueError("shape mismatch: %d ids, %d keys" % (ids.shape[0], pk32.shape[0]))
        ticket = ctypes.c_uint64()
        check(self._lib.edv_keys_set_many_async(self._ctx, _ptr(ids), _ptr(pk32), ids.shape[0], ctypes.byref(ticket)))
        return ticket.value

    def keys_set_async(self, first_id, pk32):
        """Rebuild slots first_id.. with new keys without waiting; returns the ticket."""
        pk32 = _u8(pk32, 32)
        ticket = ctypes.c_uint64()
        check(self._lib.edv_keys_set_async(self._ctx, int(first_id), _ptr(pk32), pk32.shape[0],
                                           ctypes.byref(ticket)))
        return ticket.value

    def keys_ready(self, ticket):
        r = self._lib.edv_keys_ready(self._ctx, int(ticket))
        check(min(r, 0))
        return r == 1

    def keys_sync(self):
        check(self._lib.edv_keys_sync(self._ctx))

    def keys_count(self):
        return int(self._lib.edv_keys_count(self._ctx))

    keys_generation = 0  # bumped by keys_reset: a KeyStore (keystore.py) drops its ids

    def keys_reset(self):
        check(self._lib.edv_keys_reset(self._ctx))
        self.keys_generation += 1

    def verify_batch_keyed(self, sig64, key_idx, msgs, msg_off, sig_slot=64):
        """Verdicts against registered key ids (same predicate as verify_batch);
        sig_slot=96 as verify_batch."""
        if sig_slot == SIG_SLOT:
            return self._verify_slots(True, sig64, key_idx, msgs, msg_off)
        sig64 = _u8(sig64, 64)
        key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        n = sig64.shape[0]
        if key_idx.shape[0] != n or msg_off.shape[0] != n + 1:
            raise ValueError("shape mismatch")
        if n and int(msg_off[-1]) > msgs.shape[0]:
            raise ValueError("msg_off exceeds message buffer")
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        if n:
            check(self._lib.edv_verify_batch_keyed(self._ctx, _ptr(sig64), _ptr(key_idx),
                                                   _ptr(msgs) if msgs.size else None, _ptr(msg_off), n, _ptr(bits)))
        return unpack_bits(bits, n)

    def verify_one_keyed(self, sig64, key_id, msg):
        """One request against registered key `key_id` (bytes in, bool out): the
        per-message authenticate() path, the same library call as verify_batch_keyed
        without the numpy packing around it."""
        if len(sig64) != 64:
            raise ValueError("sig64 must be 64 bytes")
        # (edv_verify_one: the resident kernel's mailbox, or one launch of the small kernel)
        one = self._one_native
        if one is not None:  # the native call (csrc/hostpack.cpp verify_one): no ctypes conversions
            try:
                return one[0](one[1], one[2], sig64, int(key_id), msg)
            except RuntimeError as ex:
                code = int(str(ex).split()[-1]) if str(ex).split()[-1].lstrip("-").isdigit() else -1
                raise EdVerifyError(code, self._lib.edv_last_error().decode(errors="replace")) from None
        # argument objects of this thread, reused from call to call (building them costs microseconds)
        tl = self._one_args.__dict__
        if "ok" not in tl:
            tl["ok"] = ctypes.c_uint8()
            tl["ok_p"] = ctypes.byref(tl["ok"])
        tl["ok"].value = 0
        check(self._lib.edv_verify_one(self._ctx, bytes(sig64), int(key_id), bytes(msg) if msg else None, len(msg),
                                       tl["ok_p"]))
        return bool(tl["ok"].value & 1)

    def verify_batch_keyed_device(self, d_sig64, d_key_idx, d_msgs, d_msg_off, n, d_accept_words, stream=None):
        st = _stream_for(stream, d_sig64, d_accept_words)
        check(self._lib.edv_verify_batch_keyed_device(self._ctx, _dev(d_sig64), _dev(d_key_idx), _dev(d_msgs),
                                                      _dev(d_msg_off), n, _dev(d_accept_words), st))

    def verify_spans_device(self, d_sig64, d_keys, keyed, d_msgs, d_msg_start, d_msg_end, n, d_accept_words,
                            stream=None):
        """Verify with message spans (item i = msgs[start[i]:end[i]]): the
        signatures of a multi-signature request share one message copy.
        keyed: d_keys are uint32 key ids, else n x 32 key bytes."""
        st = _stream_for(stream, d_sig64, d_accept_words)
        check(self._lib.edv_verify_spans_device(self._ctx, _dev(d_sig64), _dev(d_keys), 1 if keyed else 0,
                                                _dev(d_msgs), _dev(d_msg_start), _dev(d_msg_end), n,
                                                _dev(d_accept_words), st))

    # ------------------------------------------------------------------ sign
    def seed_keypair_batch(self, seeds32):
        seeds32 = _u8(seeds32, 32)
        n = seeds32.shape[0]
        pk = np.zeros((n, 32), np.uint8)
        sk = np.zeros((n, 64), np.uint8)
        if n:
            check(self._lib.edv_seed_keypair_batch(self._ctx, _ptr(seeds32), n, _ptr(pk), _ptr(sk)))
        return pk, sk

    def sign_batch(self, sk64, key_idx, msgs, msg_off):
        sk64 = _u8(sk64, 64)
        key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        n = key_idx.shape[0]
        if n and int(key_idx.max()) >= sk64.shape[0]:
            raise ValueError("key_idx out of range")
        sig = np.zeros((n, 64), np.uint8)
        if n:
            check(self._lib.edv_sign_batch(self._ctx, _ptr(sk64), _ptr(key_idx), _ptr(msgs) if msgs.size else None,
                                           _ptr(msg_off), n, _ptr(sig)))
        return sig

    def sign_batch_device(self, d_sk64, d_key_idx, d_msgs, d_msg_off, n, d_sig_out, stream=None):
        st = _stream_for(stream, d_sk64, d_sig_out)
        check(self._lib.edv_sign_batch_device(self._ctx, _dev(d_sk64), _dev(d_key_idx), _dev(d_msgs),
                                              _dev(d_msg_off), n, _dev(d_sig_out), st))

    def sign_spans_device(self, d_sk64, d_key_idx, d_msgs, d_msg_start, d_msg_end, n, d_sig_out, stream=None):
        """Deterministic signatures over message spans (item i = msgs[start[i]:end[i]])."""
        st = _stream_for(stream, d_sig_out)
        check(self._lib.edv_sign_spans_device(self._ctx, _dev(d_sk64), _dev(d_key_idx), _dev(d_msgs),
                                              _dev(d_msg_start), _dev(d_msg_end), n, _dev(d_sig_out), st))

    # -------------------------------------------------------------- digests
    def sha256_batch(self, msgs, msg_off):
        """SHA-256 of each message (host buffers): n x 32 uint8."""
        msgs = _u8(msgs)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        n = msg_off.shape[0] - 1
        out = np.zeros((max(n, 0), 32), np.uint8)
        if n > 0:
            if int(msg_off[-1]) > msgs.shape[0]:
                raise ValueError("msg_off exceeds message buffer")
            check(self._lib.edv_sha256_batch(self._ctx, _ptr(msgs) if msgs.size else None, _ptr(msg_off), n,
                                              _ptr(out)))
        return out

    def sha256_spans_device(self, d_msgs, d_msg_start, d_msg_end, n, d_out32, stream=None):
        st = _stream_for(stream, d_out32)
        check(self._lib.edv_sha256_spans_device(self._ctx, _dev(d_msgs), _dev(d_msg_start), _dev(d_msg_end), n,
                                                _dev(d_out32), st))

    # ----------------------------------------------------------------- tally
    def tally(self, key, voter, phase, valid, n_keys, n_validators, primary=None):
        """Distinct-voter PREPARE/COMMIT counts and quorum flags per key.
        primary: per-key voter index of the view's primary (0xff = none) --
        its PREPARE never counts (replica.py:1289-1291); None = no primary.
        Returns (counts uint32[n_keys, 2], prepare_quorum bool[n_keys],
        commit_quorum bool[n_keys])."""
        key = np.ascontiguousarray(key, dtype=np.uint32)
        voter = np.ascontiguousarray(voter, dtype=np.uint8)
        phase = np.ascontiguousarray(phase, dtype=np.uint8)
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        nv = key.shape[0]
        if not (voter.shape[0] == phase.shape[0] == valid.shape[0] == nv):
            raise ValueError("vote arrays differ in length")
        if primary is not None:
            primary = np.ascontiguousarray(primary, dtype=np.uint8)
            if primary.shape[0] != n_keys:
                raise ValueError("primary must have n_keys entries")
        counts = np.zeros((n_keys, 2), np.uint32)
        quorum = np.zeros(n_keys, np.uint8)
        if n_keys:
            check(self._lib.edv_tally(self._ctx, _ptr(key), _ptr(voter), _ptr(phase), _ptr(valid), _ptr(primary),
                                      nv, n_keys, n_validators, _ptr(counts), _ptr(quorum)))
        return counts, (quorum & 1).astype(bool), (quorum & 2).astype(bool)

    def tally_device(self, d_key, d_voter, d_phase, d_valid, n_votes, n_keys, n_validators, d_ballot, d_counts,
                     d_quorum, stream=None, d_primary=None):
        check(self._lib.edv_tally_device(self._ctx, _dev(d_key), _dev(d_voter), _dev(d_phase), _dev(d_valid),
                                         _dev(d_primary), n_votes, n_keys, n_validators, _dev(d_ballot),
                                         _dev(d_counts), _dev(d_quorum), _stream_for(stream, d_ballot)))

    def tally_finish_device(self, d_ballot, n_keys, n_validators, d_counts, d_quorum, stream=None):
        check(self._lib.edv_tally_finish_device(self._ctx, _dev(d_ballot), n_keys, n_validators, _dev(d_counts),
                                                _dev(d_quorum), _stream_for(stream, d_ballot)))
