"""CPU test double with EdVerifyEngine's verify / key-store interface,
answering with the C oracle (oracle/_build/libed25519_oracle.so).  Used ONLY
to test host-side logic (check order, exception mapping, batching, key-store
ownership, sharding) without a GPU; the product has no CPU path.  Plain
numpy + ctypes, so the Python 3.9 reference checks (tests/golden/) use it too.
`calls` counts verify launches (one per batch call)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


_BASELINE = []


class StagingSetBusy(RuntimeError):
    """What the library's EDV_EBUSY raises (plenum_amd._lib.EdVerifyBusy): the
    staging set holds an uncollected submission."""
    code = -5


def _not_held(held, s):
    if held[s] is not None:
        raise StagingSetBusy("staging set %d holds an uncollected submission" % s)


def _baseline_lib():
    if not _BASELINE:
        _BASELINE.append(ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_baseline.so")))
    return _BASELINE[0]


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def load_oracle():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libed25519_oracle.so"))
    lib.oracle_verify_detached.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.oracle_sign_open.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    return lib


class OracleEngine:
    def __init__(self, lib=None):
        self.lib = lib or load_oracle()
        self.calls = 0
        self.keyed_calls = 0
        self.keys = []
        self.window = 10
        self.keys_generation = 0
        self.fail_keys_add = False

    def keys_reset(self):
        self.keys = []
        self.keys_generation += 1

    def keys_set_window(self, w):
        assert not self.keys
        self.window = w

    def keys_add(self, pk32):
        if self.fail_keys_add:
            raise RuntimeError("edverify error -3: key store allocation failed (test)")
        first = len(self.keys)
        self.keys.extend(bytes(r) for r in np.asarray(pk32, np.uint8).reshape(-1, 32))
        return first

    def keys_set(self, first_id, pk32):
        rows = [bytes(r) for r in np.asarray(pk32, np.uint8).reshape(-1, 32)]
        assert first_id + len(rows) <= len(self.keys)
        self.keys[first_id:first_id + len(rows)] = rows

    def keys_count(self):
        return len(self.keys)

    # signature slots (edverify.h EDV_SIG_SLOT96), decoded here the way the
    # slot contract states: text -> its 512-bit big-endian base58 value
    supports_sig_slots = True
    slot_text_items = 0
    _B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"

    def host_alloc(self, nbytes):
        """Plain host memory standing in for edv_host_alloc's pinned blocks."""
        self.host_allocs = getattr(self, "host_allocs", 0) + 1
        return (ctypes.c_ubyte * int(nbytes))()

    def _sig64(self, sig, sig_slot):
        if sig_slot == 64:
            return sig
        assert sig_slot == 96
        slots = np.asarray(sig, np.uint8).reshape(-1, 96)
        out = np.zeros((slots.shape[0], 64), np.uint8)
        for i, s in enumerate(slots):
            t = int(s[95])
            if t == 0:
                out[i] = s[:64]
                continue
            v = 0
            for c in bytes(s[:t]).decode("ascii"):
                v = v * 58 + self._B58.index(c)
            assert v < 1 << 512, "slot text beyond 64 bytes"
            out[i] = np.frombuffer(v.to_bytes(64, "big"), np.uint8)
            self.slot_text_items += 1
        return out

    def verify_batch_keyed(self, sig64, key_idx, msgs, msg_off, sig_slot=64):
        sig64 = self._sig64(sig64, sig_slot)
        self.keyed_calls += 1
        pk = np.frombuffer(b"".join(self.keys[int(k)] if int(k) < len(self.keys) else b"\0" * 32
                                    for k in key_idx), np.uint8).reshape(-1, 32)
        ok = self._verify(sig64, pk, msgs, msg_off)
        self.calls += 1
        return ok & np.array([int(k) < len(self.keys) for k in key_idx], bool)

    def sign_open_batch(self, sm, sm_off, pk32):
        self.calls += 1
        sm = bytes(sm) if not isinstance(sm, np.ndarray) else sm.tobytes()
        pk32 = np.asarray(pk32, dtype=np.uint8).reshape(-1, 32) if not isinstance(pk32, list) else \
            np.frombuffer(b"".join(pk32), np.uint8).reshape(-1, 32)
        off = [int(x) for x in sm_off]
        return np.array([self.lib.oracle_sign_open(sm[off[i]:off[i + 1]], off[i + 1] - off[i], pk32[i].tobytes()) == 0
                         for i in range(len(off) - 1)], dtype=bool)

    def verify_submit(self, sig, keys, msgs, msg_off, keyed, sig_slot=64):
        self.submits = getattr(self, "submits", 0) + 1
        inflight = getattr(self, "in_flight", 0) + 1
        if inflight > 64:  # edverify.hip kMaxPending: the library refuses a 65th uncollected ticket
            raise RuntimeError("64 submissions outstanding")
        self.in_flight = inflight
        self.max_in_flight = max(getattr(self, "max_in_flight", 0), inflight)
        if keyed:
            return self.verify_batch_keyed(sig, keys, msgs, msg_off, sig_slot=sig_slot)
        return self.verify_batch(sig, keys, msgs, msg_off, sig_slot=sig_slot)

    def verify_collect(self, handle):
        self.in_flight -= 1
        return handle

    def verify_batch(self, sig64, pk32, msgs, msg_off, sig_slot=64):
        self.calls += 1
        return self._verify(self._sig64(sig64, sig_slot), pk32, msgs, msg_off)

    def _verify(self, sig64, pk32, msgs, msg_off):
        sig64 = np.ascontiguousarray(np.asarray(sig64, np.uint8).reshape(-1, 64))
        pk32 = np.ascontiguousarray(np.asarray(pk32, np.uint8).reshape(-1, 32))
        off = np.ascontiguousarray(np.asarray(msg_off, np.uint64))
        n = len(off) - 1
        if n >= 64:  # the same C oracle on every host CPU (oracle/cpu_baseline.c, use_sodium = 0)
            buf = np.frombuffer(bytes(msgs) if not isinstance(msgs, np.ndarray) else msgs.tobytes(), np.uint8)
            buf = np.concatenate([buf, np.zeros(16, np.uint8)])
            ok = np.zeros(n, np.uint8)
            secs = ctypes.c_double()
            P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
            assert _baseline_lib().cpu_baseline_run(P(sig64), P(pk32), P(buf), P(off), ctypes.c_uint64(n),
                                                    _threads(), 0, P(ok), ctypes.byref(secs)) == 0
            return ok.astype(bool)
        msgs = bytes(msgs) if not isinstance(msgs, np.ndarray) else msgs.tobytes()
        o = [int(x) for x in off]
        return np.array([self.lib.oracle_verify_detached(sig64[i].tobytes(), msgs[o[i]:o[i + 1]],
                                                         o[i + 1] - o[i], pk32[i].tobytes()) == 0
                         for i in range(n)], dtype=bool)


class OracleBlsEngine:
    """The BLS half of EdVerifyEngine (bls_verify_batch, bls_aggregate,
    bls_sign_batch, bls_keygen_batch) answered by oracle/bls_bn254_oracle.py
    (pure Python, ~0.5 s per check).  `calls` counts launches."""

    def __init__(self):
        import sys
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import bls_bn254_oracle
        self.o = bls_bn254_oracle
        self.calls = 0

    def bls_verify_batch(self, sig128, msgs, msg_off, vk128, gen128, vk_off=None):
        o = self.o
        self.calls += 1
        sig128 = np.asarray(sig128, np.uint8).reshape(-1, 128)
        vk128 = np.asarray(vk128, np.uint8).reshape(-1, 128)
        msgs = np.asarray(msgs, np.uint8)
        gen = o.g2_from_bytes(np.asarray(gen128, np.uint8).tobytes())
        out = []
        for i in range(sig128.shape[0]):
            k0, k1 = (int(vk_off[i]), int(vk_off[i + 1])) if vk_off is not None else (i, i + 1)
            acc = None
            for k in range(k0, k1):
                acc = o.g2_add(acc, o.g2_from_bytes(vk128[k].tobytes()))
            m = msgs[int(msg_off[i]):int(msg_off[i + 1])].tobytes()
            out.append(o.verify(o.g1_from_bytes(sig128[i].tobytes()), m, acc, gen))
        return np.asarray(out, bool)

    def bls_aggregate(self, sig128, sig_off):
        o = self.o
        self.calls += 1
        sig128 = np.asarray(sig128, np.uint8).reshape(-1, 128)
        out = []
        for i in range(len(sig_off) - 1):
            pts = [o.g1_from_bytes(sig128[k].tobytes()) for k in range(int(sig_off[i]), int(sig_off[i + 1]))]
            out.append(np.frombuffer(o.g1_to_bytes(o.aggregate(pts)), np.uint8))
        return np.asarray(out, np.uint8).reshape(-1, 128)

    def bls_sign_batch(self, sk32, msgs, msg_off):
        o = self.o
        self.calls += 1
        sk32 = np.asarray(sk32, np.uint8).reshape(-1, 32)
        msgs = np.asarray(msgs, np.uint8)
        return np.asarray([np.frombuffer(o.g1_to_bytes(o.sign(msgs[int(msg_off[i]):int(msg_off[i + 1])].tobytes(),
                                                               int.from_bytes(sk32[i].tobytes(), "big"))), np.uint8)
                           for i in range(sk32.shape[0])], np.uint8)

    def bls_keygen_batch(self, sk32, gen128):
        o = self.o
        self.calls += 1
        sk32 = np.asarray(sk32, np.uint8).reshape(-1, 32)
        gen = o.g2_from_bytes(np.asarray(gen128, np.uint8).tobytes())
        return np.asarray([np.frombuffer(o.g2_to_bytes(o.keygen(int.from_bytes(sk32[i].tobytes(), "big"), gen)),
                                         np.uint8) for i in range(sk32.shape[0])], np.uint8)


class AsyncOracleEngine(OracleEngine):
    """OracleEngine with edv_keys_add_async's contract: a registration returns
    at once with a ticket and its build stays in flight until finish_builds()
    (or keys_sync); a keyed verify of an id still building fails the test (the
    product must route it to the general path), and the synchronous
    keys_add / keys_set raise (the request path must never wait on a build)."""

    def __init__(self, lib=None):
        super().__init__(lib)
        self.issued = 0
        self.done = 0
        self.building = {}  # id -> ticket
        self.sync_calls = 0

    def keys_add(self, pk32):
        raise AssertionError("synchronous keys_add on the request path")

    def keys_set(self, first_id, pk32):
        raise AssertionError("synchronous keys_set on the request path")

    def keys_add_async(self, pk32):
        first = OracleEngine.keys_add(self, pk32)
        self.issued += 1
        for i in range(first, len(self.keys)):
            self.building[i] = self.issued
        return first, self.issued

    def keys_set_async(self, first_id, pk32):
        OracleEngine.keys_set(self, first_id, pk32)
        self.issued += 1
        for i in range(first_id, first_id + np.asarray(pk32, np.uint8).reshape(-1, 32).shape[0]):
            self.building[i] = self.issued
        return self.issued

    def keys_set_many_async(self, ids, pk32):
        pk32 = np.asarray(pk32, np.uint8).reshape(-1, 32)
        ids = [int(i) for i in ids]
        assert len(set(ids)) == len(ids) == pk32.shape[0]
        for i, k in zip(ids, pk32):
            OracleEngine.keys_set(self, i, k.reshape(1, 32))
        self.issued += 1
        self.many_calls = getattr(self, "many_calls", 0) + 1
        for i in ids:
            self.building[i] = self.issued
        return self.issued

    def keys_ready(self, ticket):
        return ticket <= self.done

    def finish_builds(self):
        self.done = self.issued
        self.building.clear()

    def keys_sync(self):
        self.sync_calls += 1
        self.finish_builds()

    def keys_reset(self):
        super().keys_reset()
        self.finish_builds()

    def verify_batch_keyed(self, sig64, key_idx, msgs, msg_off, sig_slot=64):
        busy = [int(k) for k in key_idx if int(k) in self.building]
        assert not busy, "keyed verify of ids still building: %s" % sorted(set(busy))[:8]
        return super().verify_batch_keyed(sig64, key_idx, msgs, msg_off, sig_slot)


class StagingOracleEngine(OracleEngine):
    """OracleEngine with edv_stage_reserve / edv_stage_put / edv_verify_staged:
    the staging buffer is host memory and the put a memcpy done by
    oracle/_build/libstage_double.so, which the native scan calls from its
    worker threads exactly as it calls the library's edv_stage_put."""
    supports_staging = True

    def __init__(self, lib=None):
        super().__init__(lib)
        self._put = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libstage_double.so")).stage_double_put
        self.sets = [(ctypes.c_ubyte * 0)(), (ctypes.c_ubyte * 0)()]  # edv_stage_select's two staging sets
        self.cur = 0
        self.held = [None, None]  # the uncollected submission of each set
        self.staged_calls = 0
        self.submits_staged = 0
        self._last = [None, None]  # each set's last staged batch: (slot_off, msg_base, starts, ends)
        self.subset_calls = 0

    @property
    def stage(self):
        return self.sets[self.cur]

    def stage_select(self, staging_set):
        assert staging_set in (0, 1)
        self.cur = staging_set

    def stage_reserve(self, nbytes):
        _not_held(self.held, self.cur)
        self._last[self.cur] = None  # (edv_verify_staged_subset refuses the set from here)
        if len(self.stage) < nbytes:
            self.sets[self.cur] = (ctypes.c_ubyte * int(nbytes))()

    def verify_staged_submit(self, keyed, keys, slot_off, msg_base, msg_start, msg_end):
        _not_held(self.held, self.cur)
        self.submits_staged += 1
        ok = self.verify_staged(keyed, keys, slot_off, msg_base, msg_start, msg_end)
        self.held[self.cur] = ok
        return (self.cur, ok)

    def verify_staged_collect(self, handle):
        if isinstance(handle, _Parts):
            return self._collect_parts(handle)
        s, ok = handle
        assert self.held[s] is ok
        self.held[s] = None
        return ok

    # -- edv_verify_staged_begin / _part / _end (stage_double_part snapshots each part)
    supports_staged_parts = True
    part_fail_at = 0  # make the k-th part call fail (tests)

    def verify_staged_begin(self, keyed, n):
        assert keyed
        _not_held(self.held, self.cur)
        if n and not self.keys:  # edv_verify_staged_begin: EDV_EINVAL "no registered keys"
            raise RuntimeError("edverify error -1: no registered keys")
        h = _Parts(self.cur, n, self.part_fail_at)
        self.held[self.cur] = h
        self._last[self.cur] = None
        self.parts_begun = getattr(self, "parts_begun", 0) + 1
        self._open = h
        return h

    def parter(self):
        fn = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libstage_double.so")).stage_double_part
        return (ctypes.cast(fn, ctypes.c_void_p).value, ctypes.addressof(self._open.c))

    def verify_staged_end(self):
        h, self._open = self._open, None
        h.ended = True
        if h.c.bad or (h.c.fail_at and h.c.calls >= h.c.fail_at):
            raise RuntimeError("a part failed")

    def _collect_parts(self, h):
        assert self.held[h.set] is h and h.ended
        self.held[h.set] = None
        n, cov = h.n, int(h.c.covered)
        ok = np.zeros(n, bool)
        if cov:
            st = np.frombuffer(self.sets[h.set], np.uint8)
            keys = np.ctypeslib.as_array(h.keys)[:cov]
            spans = np.ctypeslib.as_array(h.spans)
            ok[:cov] = self._verify_span_items(st, keys, spans[:cov], spans[n:n + cov], h)
        return ok

    def _verify_span_items(self, st, keys, ms, me, h):
        # the slots sit at the staging's slot offset; the scan reserved them after the messages
        slot_off = self._slot_off_of(h)
        n = len(ms)
        slots = st[slot_off:slot_off + 96 * n].reshape(-1, 96)
        parts = [st[int(a):int(b)].tobytes() for a, b in zip(ms, me)]
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(p) for p in parts])
        buf = np.frombuffer(b"".join(parts), np.uint8)
        self.parts_verified = getattr(self, "parts_verified", 0) + n
        return self.verify_batch_keyed(slots, keys, buf, off, sig_slot=96)

    def _slot_off_of(self, h):
        return int(h.c.slot_off)

    def stager(self):
        return (ctypes.cast(self._put, ctypes.c_void_p).value, ctypes.addressof(self.stage))

    supports_staged_subset = True

    def verify_staged_subset(self, idx, pk32):
        """edv_verify_staged_subset: items idx of the set's last staged batch, general path."""
        last = self._last[self.cur]
        assert last is not None and self.held[self.cur] is None, "no staged batch to take a subset of"
        slot_off, msg_base, ms, me = last
        idx = np.asarray(idx, np.int64)
        assert idx.size == 0 or int(idx.max()) < len(ms)
        self.subset_calls += 1
        st = np.frombuffer(self.stage, np.uint8)
        slots = st[slot_off:slot_off + 96 * len(ms)].reshape(-1, 96)[idx]
        parts = [st[msg_base + int(ms[i]):msg_base + int(me[i])].tobytes() for i in idx]
        off = np.zeros(len(idx) + 1, np.uint64)
        off[1:] = np.cumsum([len(p) for p in parts])
        return self.verify_batch(slots, np.asarray(pk32, np.uint8).reshape(-1, 32),
                                 np.frombuffer(b"".join(parts), np.uint8), off, sig_slot=96)

    def verify_staged(self, keyed, keys, slot_off, msg_base, msg_start, msg_end):
        self.staged_calls += 1
        self._last[self.cur] = (int(slot_off), int(msg_base), np.array(msg_start, np.uint64),
                                np.array(msg_end, np.uint64))
        st = np.frombuffer(self.stage, np.uint8)
        n = len(msg_start)
        slots = st[slot_off:slot_off + 96 * n].reshape(-1, 96)
        parts = [st[msg_base + int(a):msg_base + int(b)].tobytes() for a, b in zip(msg_start, msg_end)]
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(p) for p in parts])
        buf = np.frombuffer(b"".join(parts), np.uint8)
        if keyed:
            return self.verify_batch_keyed(slots, keys, buf, off, sig_slot=96)
        return self.verify_batch(slots, keys, buf, off, sig_slot=96)


class _PartC(ctypes.Structure):
    _fields_ = [("keys", ctypes.c_void_p), ("spans", ctypes.c_void_p), ("n", ctypes.c_uint64),
                ("covered", ctypes.c_uint64), ("calls", ctypes.c_uint64), ("fail_at", ctypes.c_uint64),
                ("bad", ctypes.c_uint64), ("slot_off", ctypes.c_uint64)]


class _Parts:
    """A speculative staged batch of StagingOracleEngine (the double's edv_verify_staged_begin
    handle): the part snapshots stage_double_part writes."""

    def __init__(self, s, n, fail_at):
        self.set, self.n, self.ended = s, n, False
        self.keys = (ctypes.c_uint32 * max(n, 1))()
        self.spans = (ctypes.c_uint64 * max(2 * n, 1))()
        self.c = _PartC(ctypes.addressof(self.keys), ctypes.addressof(self.spans), n, 0, 0, fail_at, 0, 0)
