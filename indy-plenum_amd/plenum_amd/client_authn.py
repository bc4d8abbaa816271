"""Client authenticators with the reference API, verified in GPU batches.

Reference: plenum/server/client_authn.py:22-154 (ClientAuthNr, NaclAuthNr,
SimpleAuthNr).  `authenticate(msg, identifier=None, signature=None)` keeps the
reference's exact check order and exception classes:
  :72-80  signature present            -> EmptySignature / MissingSignature
  :81-87  identifier present           -> EmptyIdentifier / MissingIdentifier
  :88-91  b58decode(signature)         -> InvalidSignatureFormat (from the b58 error)
  :92     serializeForSig(msg, ['signature'])
  :93     getVerkey(identifier)        -> UnknownIdentifier (SimpleAuthNr :142-154)
  :95-97  verkey is None               -> CouldNotAuthenticate
  :99     DidVerifier(verkey, identifier)  (InvalidKey -> CouldNotAuthenticate)
  :100-102 verify(sig, ser) false      -> InvalidSignature
  :105-106 anything else               -> CouldNotAuthenticate from ex
The verify step is libsodium's crypto_sign_open(sig || ser, pk)
(nacl_wrappers.py:232-242, :108), run by libplenum_edverify.so on the GPU.

GpuAuthMixin carries ALL of it -- authenticate, the batch machinery, the
verdict cache, the key-table routing -- and relies on its host class only for
getVerkey / addIdr (and the `clients` / `state` they use).  Mixed in front of
the reference's own plenum.server.client_authn.SimpleAuthNr:

    class GpuSimpleAuthNr(GpuAuthMixin, SimpleAuthNr): ...

every authenticate() goes through the engine (no libsodium call), the
exceptions are the reference's classes (exceptions.py re-exports them inside a
node), and node.py:2482's isinstance(..., SimpleAuthNr) stays true.
tests/golden/check_dropin_ref.py proves exactly this against the real
reference class.  GpuAuthNr is the same mixin over this repo's restatement of
SimpleAuthNr (standalone use).

Added on top of the reference API (the reference calls authenticate once per
message from Node.verifySignature, node.py:2294-2318):
  authenticate_batch(msgs)        one GPU launch for many requests; returns,
                                  per message, the identifier or the exception
                                  instance authenticate() would have raised.
  prefetch(msgs)                  verify-ahead: batch-verify what the node is
                                  about to authenticate (client REQUESTs and
                                  PROPAGATE payloads of one rxMsgs drain,
                                  zstack.py:528-549); later authenticate()
                                  calls hit the verdict cache.
  authenticate_multi(msg, sigs)   multi-signature requests (not in the
                                  reference snapshot: parity unpinned).
`CoreAuthNr` is an alias of GpuAuthNr; `ReqAuthenticator` aggregates
authenticators (names from BASELINE.json's north star).
"""
import contextlib
import copy
import gc
from time import perf_counter as _perf_counter
import threading
import os
from abc import abstractmethod
from collections import OrderedDict, deque
from itertools import islice
from time import monotonic
from copy import deepcopy
from typing import Dict

from .base58 import b58decode
from . import exceptions as _exc
from .exceptions import (CouldNotAuthenticate, EmptyIdentifier, EmptySignature, InsufficientCorrectSignatures,
                         InsufficientSignatures, InvalidSignature, InvalidSignatureFormat, MissingIdentifier,
                         MissingSignature, SigningException, UnknownIdentifier)
from .keystore import KeyStore, UseCounts, auto_window
from .serialization import serialize_msg_for_signing
from .verifier import DidVerifier, VerkeyCache

try:  # native batch scan (csrc/hostpack.cpp): authenticate()'s host steps for a whole batch
    from ._hostpack import gather_items as _gather_items, results_from as _results_from, scan_batch_u as _scan_batch
    from ._hostpack import gather_spans as _gather_spans
except ImportError:  # pragma: no cover - the per-message path below
    _scan_batch = _gather_items = _results_from = _gather_spans = None
try:
    from ._hostpack import (gather_u32 as _gather_u32, pack_range as _pack_range, repack_spans as _repack_spans,
                            results_ok as _results_ok, kid_map as _kid_map, kid_map_size as _kid_map_size)
except ImportError:  # pragma: no cover
    _pack_range = _repack_spans = _gather_u32 = _results_ok = _kid_map = _kid_map_size = None
try:  # the batch's per-identifier keys for the known getVerkey (SimpleAuthNr's dict lookup) in one call
    from ._hostpack import keys_known as _keys_known
except ImportError:  # pragma: no cover
    _keys_known = None
try:  # ... on the scan's worker pool, with the keys as one buffer (key store lookup, general-path keys)
    from ._hostpack import keys_known_flat as _keys_known_flat
except ImportError:  # pragma: no cover
    _keys_known_flat = None
try:  # a mixed batch's general-path items and their keys, on the worker pool
    from ._hostpack import general_items as _general_items
except ImportError:  # pragma: no cover
    _general_items = None
try:  # the node's per-message path: authenticate()'s host steps in one call; the verify-ahead's dedupe
    from ._hostpack import authn_key as _authn_key, distinct_sm as _distinct_sm
except ImportError:  # pragma: no cover
    _authn_key = _distinct_sm = None

try:  # native packing (csrc/hostpack.cpp)
    from ._hostpack import pack_sm as _pack_sm, pack_split64 as _pack_split64
except ImportError:  # pragma: no cover - same layout in Python
    import struct as _struct

    def _pack_sm(sigs, sers, keys):
        offs, pos = [0], 0
        for s_, m in zip(sigs, sers):
            pos += len(s_) + len(m)
            offs.append(pos)
        sm = b"".join(s_ + m for s_, m in zip(sigs, sers))
        return sm, _struct.pack("<%dQ" % len(offs), *offs), b"".join(keys)

    def _pack_split64(sigs, sers):
        sig64, msgs, offs, short, pos = [], [], [0], [], 0
        for s_, m in zip(sigs, sers):
            sm = s_ + m
            if len(sm) < 64:
                sig64.append(b"\0" * 64)
                short.append(1)
                sm = b""
            else:
                sig64.append(sm[:64])
                short.append(0)
                sm = sm[64:]
            msgs.append(sm)
            pos += len(sm)
            offs.append(pos)
        return b"".join(sig64), b"".join(msgs), _struct.pack("<%dQ" % len(offs), *offs), bytes(short)

SIG = 'signature'
SIGS = 'signatures'
IDENTIFIER = 'identifier'
REQ_ID = 'reqId'
VERKEY = 'verkey'


def _invalid_signatures(nf):
    """nf fresh InvalidSignature() instances.  With this package's own exception classes (no
    reference plenum importable) the constructor only records identifier = reqId = None, so the
    instances are made by BaseException.__new__ (args ()) and that one dict update -- a third of
    the constructor's cost for a batch's ~1k forgeries; the reference's classes are constructed."""
    if nf < 64 or _exc.REFERENCE:
        return [InvalidSignature() for _ in range(nf)]
    new, cls = InvalidSignature.__new__, InvalidSignature
    attrs = {"identifier": None, "reqId": None}
    out = [new(cls) for _ in range(nf)]
    for e in out:
        e.__dict__.update(attrs)
    return out


def _results_failing(ok, short, uidx_b, uniq):
    """_results_ok with a fresh InvalidSignature at every failing item (verdict False or a short
    signature), the exceptions made BEFORE the result list exists (hostpack.cpp results_ok: made
    after it, their allocations let the collector's young-generation passes walk the fresh list)."""
    import numpy as np
    okb = np.frombuffer(ok, np.uint8) if not isinstance(ok, np.ndarray) else ok.view(np.uint8)
    # (a pass is ok 1 and short 0, i.e. ok > short on the 0/1 bytes: one comparison over the batch,
    # not two plus an OR -- 1.6 against 0.26 ms per 1M on the CPU)
    nf = len(okb) - int(np.count_nonzero(okb > np.frombuffer(short, np.uint8, count=len(okb))))
    fails = _invalid_signatures(nf)
    results, failed = _results_ok(ok, short, uidx_b, uniq, fails)
    if len(failed) != nf:  # (never expected: the native pass left None at its failures)
        for i in failed:
            results[i] = InvalidSignature()
    return results, failed


@contextlib.contextmanager
def _gc_paused():
    """The cyclic collector paused for one batch call (reference counting still frees everything):
    a batch makes a few large temporary containers (the distinct identifiers, their keys: ~30k
    entries each under key churn), and every young-generation collection the call's own
    allocations set off would walk all of them -- 5-10 ms of a 250k-request batch went there.
    Collections due meanwhile run at the next allocation after the call, once the temporaries are
    gone.  The previous state is restored however the call ends."""
    was = gc.isenabled()
    if was:
        gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _known_getverkey(cls):
    """cls.getVerkey is SimpleAuthNr's -- this module's restatement or the reference's own
    (client_authn.py:142-154): clients.get(identifier), the state only when that is empty."""
    f = getattr(cls, "getVerkey", None)
    return f is SimpleAuthNr.getVerkey or (getattr(f, "__qualname__", "") == "SimpleAuthNr.getVerkey" and
                                            getattr(f, "__module__", "") == "plenum.server.client_authn")
ROLE = 'role'

KEY_STORE_BYTES = 32 << 30  # HBM for key tables: the window is the widest that fits max_keys
# Promotion priced by expected use: a key earns a table when its decayed count of verified requests
# reaches HOT_KEY_USES.  A table build costs ~BUILD_US of GPU time at the drop-in's window (W = 10)
# and a keyed verify saves ~SAVE_NS against the general path for a key of its own, so a build
# repays after BUILD_US / SAVE_NS requests; with counts halving per 2^18 requests verified, a key
# needs about that many per epoch to get there ("Key churn").  Keys with fewer
# than 1/16 of it in a batch are not counted (they cannot reach it before the decay).
HOT_KEY_USES = 64
HOT_COUNT_FLOOR = 16
_SIG_SLOT = 96  # edverify.h EDV_SIG_SLOT96: signatures as base58 text, decoded on the GPU
_PINNED_MIN_BATCH = 4096  # smaller batches keep the bytearrays (the library stages them cheaply)
_STREAM_CHUNK = 1 << 17  # requests per streamed submit: 2^17 beat 2^18 and 2^16 by 2-3 % (profiles/r06c)
_STREAM_WINDOW = 16  # streamed submits in flight before the oldest is collected (edverify.hip kMaxPending = 64)
_STAGE_MIN_BATCH = 1 << 16  # batches staged while scanned (edv_stage_put from the scan's workers)
_PART_ITEMS = 1 << 16  # a speculative staged batch's kernels go out per this many requests


_MISSING = object()
_VERDICT_ENTRY_BYTES = 240  # a verdict-cache entry's objects beyond its key and sm bytes (tuple, 2 bytes, dict slot)
_BUSY = object()  # _authenticate_staged: the staging set is held by a batch in flight
_EDV_EBUSY = -5  # include/edverify.h EDV_EBUSY (plenum_amd._lib.EdVerifyBusy.code)
_IGNORE_SIG = (SIG,)


class _Prepared:
    __slots__ = ("identifier", "sig", "ser", "key")

    def __init__(self, identifier, sig, ser, key):
        self.identifier, self.sig, self.ser, self.key = identifier, sig, ser, key


_LOCKS_LOCK = threading.Lock()


def _collect_quietly(eng, handles):
    """Collect (and so free) submitted verify tickets whose verdicts nobody will
    read -- the clean-up of a batch path that raised between submit and
    collect; their errors are not the caller's."""
    for h in handles:
        try:
            eng.verify_collect(h)
        except Exception:
            pass


def _engine_lock(eng):
    """One re-entrant lock per engine, shared by every authenticator on it:
    held from key routing (KeyStore lookup / register, whose evictions rebuild
    slots) through the verify launch, so a batch on another thread can neither
    rebind a key id this batch already resolved nor share the engine's
    staging buffers and stream with it.  (The reference is single-threaded
    asyncio, looper.py:141-151; this makes concurrent callers safe, not
    parallel.)"""
    lk = getattr(eng, "_authn_lock", None)
    if lk is None:
        with _LOCKS_LOCK:
            lk = getattr(eng, "_authn_lock", None)
            if lk is None:
                lk = threading.RLock()
                eng._authn_lock = lk
    return lk


class _GpuState:
    """Per-authenticator GPU state (created on first use).

    Threads: the engine, its key store and the scan / staging buffers are
    used only under _engine_lock.  The bookkeeping dicts -- verdicts, hot,
    pending -- are also updated outside it (authenticate()'s cache hit and
    miss, _count_verified).  Every single dict operation is atomic under the
    GIL, so concurrent callers cannot corrupt them; a race between two
    threads can at most evict one extra verdict (a later re-verify).  The
    use counts (key_uses, keystore.UseCounts) take their own lock.  The node
    calls authenticate() from its one looper thread (looper.py:141-151), as
    the reference does."""

    def __init__(self, engine=None, device=0, devices=None, verdict_cache_size=1 << 20,
                 verdict_cache_bytes=256 << 20, verdict_max_age=300.0, key_window="auto",
                 max_keys=16384, hot_key_uses=HOT_KEY_USES, key_store_bytes=KEY_STORE_BYTES, scan_threads=0,
                 pipeline_part=0, async_key_builds=True, stream=True, stage=True, speculate=True,
                 max_promotions=1024):
        self.engine = engine
        self.device = device
        self.devices = devices
        self.keys = VerkeyCache()
        # the verify-ahead verdicts: (key bytes, sm) -> bool, oldest first, bounded by entries, by
        # bytes (keys + sm + ~240 B of objects per entry) and by age (seconds since insertion; trimmed
        # on insert, per one-second epoch).  A verdict never goes stale -- it is the verdict of
        # exactly those bytes under exactly that key -- so the bounds only cap memory.
        self.verdicts = OrderedDict()
        self.verdict_cache_size = verdict_cache_size
        self.verdict_cache_bytes = verdict_cache_bytes
        self.verdict_max_age = verdict_max_age
        self.verdict_bytes = 0
        self.verdict_epochs = deque()  # [start time, entries inserted in that second], oldest first
        self.key_window = auto_window(max_keys, key_store_bytes) if key_window == "auto" else key_window
        self.max_keys = max_keys
        self.hot_key_uses = hot_key_uses
        self.key_uses_max = 1 << 16
        self.key_uses = UseCounts(self.key_uses_max)  # key -> decayed successful general-path verifies (bounded)
        self.max_promotions = max_promotions  # keys that earned a slot, registered per batch at most
        self.pending = OrderedDict()    # addIdr keys waiting for a free slot
        self.hot = OrderedDict()        # keys that earned a slot (hot_key_uses verified requests)
        self.scan_threads = scan_threads  # host threads of the native batch scan (0 = auto)
        # the scan's sig64 / message output, reused from batch to batch (grown, never shrunk:
        # fresh buffers cost a page fault per 4 KiB on every batch); a batch holds the engine
        # lock (_engine_lock) from the scan through the verify, so no other batch writes them
        self.scan_out = [bytearray(), bytearray()]
        # ... or, on an engine with pinned host memory, these (engine.host_alloc): the GPU call
        # then copies straight from them; sized from the last batch's message bytes per item
        self.pinned_out = None
        self.msg_bytes_per_item = 256.0
        # batches of 2 * pipeline_part requests or more are scanned in parts whose GPU work
        # overlaps the next part's scan (0 = never, the default: on the box's 16-CPU share the
        # per-part scan costs -- helper wake-ups, the identifier merge, the result list assembly --
        # exceeded the ~7 ms per 1M of GPU work hidden: 1M requests 23-25 M/s unparted against
        # 14 M/s in 2^17 parts and 17-18 M/s in 2^18 parts, profiles/r04c)
        self.pipeline_part = pipeline_part
        # key tables registered on the request path (addIdr keys, keys that earned a slot) build on
        # the engine's build stream while batches go on; their requests take the general path until
        # the build completes (engines without edv_keys_add_async build synchronously)
        self.async_key_builds = async_key_builds
        # batches of 2 library chunks (2^19 requests) or more pack chunk by chunk, each chunk's DMA and
        # kernels overlapping the next chunk's pack (_authenticate_streamed)
        self.stream = stream
        self.last_breakdown = None  # the last streamed batch's phases (ms)
        # stage=True (default): batches of 2^16 requests or more are staged while scanned
        # (_authenticate_staged): 35-40 against 34-37 M requests/s streamed, alternating in one
        # process on the box (profiles/r07c/e2e_ab.log) once its verdict list was built on the
        # workers; stage=False: the streamed path
        self.stage = stage
        # identifier -> (verkey as getVerkey returned it, key bytes): authenticate()'s per-message
        # DidVerifier step without the VerkeyCache call while the verkey stays the same
        self.fast_keys = {}
        self.fast_keys_max = 1 << 18  # (identifier -> (verkey, key): ~200 B each)
        self.kid_out = bytearray()  # a batch's key id per request (gather_u32 output, reused)
        # speculate=True (default): a synchronous staged batch runs its kernels under its own scan,
        # part by part, with key ids the scan takes from kid_map (identifier -> key id of the batches
        # before); after the scan every distinct identifier's id is checked against getVerkey and the
        # key store (and the store's version), and any difference re-runs the verify the ordinary way
        self.speculate = speculate
        self.kid_map = None
        self.kid_map_version = None
        self.kid_map_max = 1 << 20
        self.stats = {"batches": 0, "batch_items": 0, "cache_hits": 0, "single_verifies": 0, "keyed_items": 0,
                      "keys_registered": 0, "prefetched": 0}


class GpuAuthMixin:
    """The GPU authenticator.  Mix in front of any class with the reference
    ClientAuthNr's getVerkey / addIdr -- the reference SimpleAuthNr included
    (INTEGRATION.md); call _gpu_init() from the constructor to configure, or
    leave it for the defaults."""

    def _gpu_init(self, engine=None, device=0, **options):
        """engine: an EdVerifyEngine / MultiEngine (default: one on `device`;
        devices=[...] or "all": a MultiEngine sharding every batch over them).
        options (_GpuState): verdict_cache_size / verdict_cache_bytes /
        verdict_max_age (the verify-ahead cache's bounds: entries, bytes,
        seconds); speculate (a synchronous staged batch's kernels under its
        own scan, key ids from the batches before; default True); key_window ('auto' = widest
        comb whose max_keys tables fit key_store_bytes, e.g. 16,384 keys in
        32 GiB -> W=10, 1,000 keys -> W=14); max_keys; hot_key_uses;
        scan_threads (host threads of authenticate_batch's native scan, 0 =
        auto: up to 16, one per 2k requests); pipeline_part (batches of twice
        this many requests or more are scanned in parts whose GPU work
        overlaps the next part's scan; 0 = off); async_key_builds (key
        tables registered on the request path build in the background, their
        requests on the general path until built; default True); stream
        (batches of 2^19 requests or more pack chunk by chunk under the
        previous chunk's DMA; default True)."""
        self._edv = _GpuState(engine=engine, device=device, **options)

    @property
    def _g(self):
        g = self.__dict__.get("_edv")
        if g is None:
            g = self._edv = _GpuState()
        return g

    @property
    def engine(self):
        return self._g.engine

    @engine.setter
    def engine(self, eng):
        self._g.engine = eng

    @property
    def stats(self):
        return self._g.stats

    def _engine(self):
        g = self._g
        if g.engine is None:
            if g.devices is not None:
                from .multi import MultiEngine
                g.engine = MultiEngine(g.devices)
            else:
                from .engine import EdVerifyEngine
                g.engine = EdVerifyEngine(g.device)
        return g.engine

    # -- the reference authenticate(), verify on the GPU ----------------------
    def authenticate(self, msg: Dict, identifier: str = None, signature: str = None) -> str:
        if identifier is None and signature is None and _authn_key is not None:
            # the node's call (node.py:2310): the host steps up to getVerkey natively, then the
            # verdict cache the verify-ahead filled; anything unusual takes the path below
            if self._native_host_steps():
                k = _authn_key(msg, _IGNORE_SIG)
                if k is not None:
                    return self._authenticate_sm(k[0], k[1])
        try:
            p = self._prepare(msg, identifier, signature)
            if not self._verify_prepared(p):
                raise InvalidSignature
        except SigningException as e:
            raise e
        except Exception as ex:
            raise CouldNotAuthenticate from ex
        return p.identifier

    def _authenticate_sm(self, identifier, sm):
        """authenticate() after its host steps (client_authn.py:93-106):
        sm = b58decode(signature) || serializeForSig(msg), as authn_key
        returns them -- the same order of checks and exceptions as _prepare
        from getVerkey on."""
        g = self._g
        try:
            verkey = self.getVerkey(identifier)
            if verkey is None:
                raise CouldNotAuthenticate('Can not find verkey for DID {}'.format(identifier))
            key = self._key_of(identifier, verkey)
            if not key:  # nacl_wrappers.py:237-238: no key -> False
                raise InvalidSignature
            vk = (key, sm)
            hit = g.verdicts.get(vk)
            if hit is None:
                hit = self._verify_miss(identifier, key, sm, vk)
            else:
                g.stats["cache_hits"] += 1
            if not hit:
                raise InvalidSignature
        except SigningException as e:
            raise e
        except Exception as ex:
            raise CouldNotAuthenticate from ex
        return identifier

    def _prepare(self, msg, identifier=None, signature=None, ignore=(SIG,)):
        """Everything authenticate() does before the verify, reference order."""
        if not signature:
            try:
                signature = msg[SIG]
                if not signature:
                    raise EmptySignature(msg.get(IDENTIFIER), msg.get(REQ_ID))
            except KeyError:
                raise MissingSignature(msg.get(IDENTIFIER), msg.get(REQ_ID))
        if not identifier:
            try:
                identifier = msg[IDENTIFIER]
                if not identifier:
                    raise EmptyIdentifier(None, msg.get(REQ_ID))
            except KeyError:
                raise MissingIdentifier(identifier, msg.get(REQ_ID))
        try:
            sig = b58decode(signature)
        except Exception as ex:
            raise InvalidSignatureFormat from ex
        ser = self.serializeForSig(msg, topLevelKeysToIgnore=list(ignore))
        verkey = self.getVerkey(identifier)
        if verkey is None:
            raise CouldNotAuthenticate('Can not find verkey for DID {}'.format(identifier))
        key = self._resolve_key(verkey, identifier)
        return _Prepared(identifier, sig, ser, key)

    def serializeForSig(self, msg, topLevelKeysToIgnore=None):
        """The reference serializer's exact bytes (native, KAT-pinned)."""
        return serialize_msg_for_signing(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)

    def _key_of(self, identifier, verkey):
        """DidVerifier(verkey, identifier).key (verifier.py:21-46), remembered
        per identifier while getVerkey keeps returning the same verkey (the
        node's steady state): one dict lookup instead of the VerkeyCache call."""
        g = self._g
        fk = g.fast_keys.get(identifier)
        if fk is not None and (fk[0] is verkey or (verkey.__class__ is str and fk[0] == verkey)):
            return fk[1]
        key = self._resolve_key(verkey, identifier)
        self._remember_key(identifier, verkey, key)
        return key

    def _remember_key(self, identifier, verkey, key):
        """fast_keys[identifier] = (verkey, key): valid while getVerkey(identifier) returns this
        very verkey object.  Full: the oldest eighth goes (insertion order)."""
        if verkey.__class__ is str and key.__class__ is bytes and identifier.__class__ is str:
            fk = self._g.fast_keys
            if len(fk) >= self._g.fast_keys_max and identifier not in fk:
                for old in list(islice(fk, max(1, len(fk) // 8))):
                    del fk[old]
            fk[identifier] = (verkey, key)

    def _resolve_key(self, verkey, identifier):
        try:
            hash((verkey, identifier))
        except TypeError:
            return DidVerifier(verkey, identifier=identifier).key
        return self._g.keys.resolve(verkey, identifier)

    # -- key-table registration -------------------------------------------------
    def addIdr(self, identifier, verkey, role=None):
        super().addIdr(identifier, verkey, role)
        self._queue_key(identifier, verkey)

    def _queue_key(self, identifier, verkey):
        """addIdr'd keys take a free key-table slot at the next batch."""
        try:
            key = self._resolve_key(verkey, identifier)
        except Exception:
            return  # authenticate() raises the reference's error for this key later
        # the batch path's per-identifier key lookup hits from the first batch on (the key is
        # resolved here anyway); valid while clients[identifier] holds this verkey object
        self._remember_key(identifier, verkey, key)
        if key and len(key) == 32:
            g = self._g
            g.pending[key] = None
            while len(g.pending) > g.max_keys:
                g.pending.popitem(last=False)

    def _key_store(self):
        g = self._g
        if g.max_keys <= 0:
            return None
        return KeyStore.attach(self._engine(), g.key_window, g.max_keys)

    def _register_waiting(self, ks, batch_keys, pinned_ids=None):
        """Keys that earned a slot (may evict least-recently-used keys not in
        this batch: batch_keys, or their ids pinned_ids) and addIdr keys (free
        slots only), registered before the batch routes its items (asynchronous
        builds by default)."""
        g = self._g
        n_reg = 0
        if g.hot:  # at most max_promotions per batch (each a table build on the device)
            got = ks.register(list(g.hot)[:g.max_promotions], pinned=batch_keys, evict=True,
                              asynchronous=g.async_key_builds, pinned_ids=pinned_ids)
            g.stats["keys_registered"] += len(got)
            n_reg += len(got)
            g.hot.clear()
        if g.pending:
            room = ks.free_slots()
            if room > 0:
                got = ks.register([k for k in g.pending if k not in ks][:room], evict=False,
                                  asynchronous=g.async_key_builds)
                g.stats["keys_registered"] += len(got)
                n_reg += len(got)
            g.pending.clear()
        return n_reg

    def keys_settle(self):
        """Register the addIdr keys waiting for a slot and wait until every
        queued key-table build has finished (e.g. after genesis NYMs, before a
        timed run); batches never need this for correctness."""
        g = self._g
        ks = self._key_store()
        if ks is None:
            return 0
        with _engine_lock(self._engine()):
            if g.pending:
                room = ks.free_slots()
                if room > 0:
                    got = ks.register([k for k in g.pending if k not in ks][:room], evict=False,
                                      asynchronous=g.async_key_builds)
                    g.stats["keys_registered"] += len(got)
                g.pending.clear()
            ks.settle()
        return len(ks)

    def _route(self, todo):
        """Register waiting keys, then split items into (keyed + ids, general)."""
        g = self._g
        ks = self._key_store()
        if ks is None:
            return [], [], todo
        batch_keys = [p.key for p in todo]
        if g.hot:  # earned a slot: may evict least-recently-used keys not in this batch
            got = ks.register(list(g.hot)[:g.max_promotions], pinned=batch_keys, evict=True,
                              asynchronous=g.async_key_builds)
            g.stats["keys_registered"] += len(got)
            g.hot.clear()
        if g.pending:  # addIdr keys: free slots only
            room = ks.free_slots()
            if room > 0:
                take = [k for k in g.pending if k not in ks][:room]
                got = ks.register(take, evict=False, asynchronous=g.async_key_builds)
                g.stats["keys_registered"] += len(got)
            g.pending.clear()  # registered, or no room: later keys get in by use (hot)
        ids = ks.lookup(batch_keys)
        keyed = [(p, i) for p, i in zip(todo, ids) if i is not None]
        general = [p for p, i in zip(todo, ids) if i is None]
        return [p for p, _ in keyed], [i for _, i in keyed], general

    def _use_epoch(self):
        """The verified-use counts' clock: one tick per 2^18 requests this
        authenticator has verified in batches or alone; a key's count halves
        per tick (so only keys in sustained use earn a slot, and a long tail of
        signers seen now and then does not churn the store)."""
        st = self._g.stats
        return (st["batch_items"] + st["single_verifies"]) >> 18

    def _count_verified(self, items, oks):
        """A general-path key earns a slot after hot_key_uses requests that
        VERIFIED (bad signatures cannot push keys into the store), counted
        with decay (_use_epoch)."""
        counts = {}
        for p, ok in zip(items, oks):
            if ok:
                counts[p.key] = counts.get(p.key, 0) + 1
        self._count_verified_keys(list(counts), list(counts.values()))

    def _count_verified_keys(self, keys, counts):
        """_count_verified for c[j] verified requests of key j at once."""
        g = self._g
        if g.max_keys <= 0:
            return
        for key in g.key_uses.add(keys, counts, self._use_epoch(), g.hot_key_uses):
            g.hot[key] = None

    def _verify_keyed(self, items, ids):
        """crypto_sign_open(sig || ser) against registered keys: the split at
        byte 64 done on the host (nacl_wrappers.py:108), len < 64 rejects."""
        eng = self._engine()
        if len(items) == 1 and len(items[0].sig) == 64 and hasattr(eng, "verify_one_keyed"):
            self._g.stats["keyed_items"] += 1  # one authenticate() the verify-ahead missed
            return [eng.verify_one_keyed(items[0].sig, ids[0], items[0].ser)]
        import numpy as np
        sig64, msgs, off, short = _pack_split64([p.sig for p in items], [p.ser for p in items])
        ok = self._engine().verify_batch_keyed(np.frombuffer(sig64, np.uint8).reshape(-1, 64),
                                               np.asarray(ids, np.uint32), np.frombuffer(msgs, np.uint8),
                                               np.frombuffer(off, np.uint64))
        ok = np.asarray(ok, bool) & (np.frombuffer(short, np.uint8) == 0)
        self._g.stats["keyed_items"] += len(items)
        return ok

    # -- verify-ahead cache ------------------------------------------------
    @staticmethod
    def _vkey(p):
        """Verdict-cache key: the verkey's bytes and crypto_sign_open's input
        sm = sig || ser (nacl_wrappers.py:108) -- exact content, so a hit is
        the verdict of exactly these bytes under exactly this key."""
        return (p.key, p.sig + p.ser)

    def _remember(self, p, ok, vkey=None):
        g = self._g
        k = vkey if vkey is not None else self._vkey(p)
        verdicts = g.verdicts
        if k in verdicts:
            verdicts[k] = ok
            return
        verdicts[k] = ok
        g.verdict_bytes += len(k[0]) + len(k[1]) + _VERDICT_ENTRY_BYTES
        now = monotonic()
        epochs = g.verdict_epochs
        if not epochs or now - epochs[-1][0] >= 1.0:
            epochs.append([now, 0])
        epochs[-1][1] += 1
        while len(verdicts) > g.verdict_cache_size or g.verdict_bytes > g.verdict_cache_bytes:
            self._forget_oldest_verdict()
        while epochs and now - epochs[0][0] > g.verdict_max_age and verdicts:
            self._forget_oldest_verdict()

    def _forget_oldest_verdict(self):
        g = self._g
        k, _ = g.verdicts.popitem(last=False)
        g.verdict_bytes -= len(k[0]) + len(k[1]) + _VERDICT_ENTRY_BYTES
        epochs = g.verdict_epochs
        if epochs:
            epochs[0][1] -= 1
            if epochs[0][1] <= 0:
                epochs.popleft()

    def _verify_miss(self, identifier, key, sm, vk):
        """_verify_prepared for authenticate()'s miss of the verdict cache (the
        cache key vk = (key, sm) already looked up): the steady state's
        registered, built key straight to the one-request launch with sm's two
        halves as views (no copies, no second lookup), else _verify_prepared."""
        g = self._g
        eng = g.engine
        if (len(sm) >= 64 and not g.hot and not g.pending and eng is not None
                and hasattr(eng, "verify_one_keyed") and g.max_keys > 0):
            with _engine_lock(eng):
                ks = self._key_store()
                kid = ks.lookup_one(key) if ks is not None else None
                if kid is not None:
                    g.stats["single_verifies"] += 1
                    mv = memoryview(sm)
                    ok = bool(eng.verify_one_keyed(mv[:64], kid, mv[64:]))
                    st = g.stats
                    st["batches"] += 1
                    st["batch_items"] += 1
                    st["keyed_items"] += 1
                    self._remember(None, ok, vk)
                    return ok
        return self._verify_prepared(_Prepared(identifier, sm[:64], sm[64:], key))

    def _verify_prepared(self, p):
        if not p.key:  # nacl_wrappers.py:237-238: no key -> False
            return False
        g = self._g
        vk = self._vkey(p)
        hit = g.verdicts.get(vk)
        if hit is not None:
            g.stats["cache_hits"] += 1
            return hit
        g.stats["single_verifies"] += 1
        eng = self._engine()
        with _engine_lock(eng):
            ok = None
            if len(p.sig) == 64 and not g.hot and not g.pending and hasattr(eng, "verify_one_keyed"):
                # the steady state's miss: a registered, built key -- straight to the one-request launch
                ks = self._key_store()
                kid = ks.lookup_one(p.key) if ks is not None else None
                if kid is not None:
                    ok = bool(eng.verify_one_keyed(p.sig, kid, p.ser))
                    g.stats["batches"] += 1
                    g.stats["batch_items"] += 1
                    g.stats["keyed_items"] += 1
            if ok is None:
                ok = self._verify_many_locked([p])[0]
            self._remember(p, ok, vk)
        return ok

    def _verify_many(self, prepared):
        """GPU launches over prepared items (crypto_sign_open semantics): items
        whose key is registered take the key-table path, the rest one general
        launch; items without a usable key are False without touching the GPU."""
        with _engine_lock(self._engine()):
            return self._verify_many_locked(prepared)

    def _verify_many_locked(self, prepared):
        g = self._g
        todo = [p for p in prepared if p.key]
        out = {}
        keyed, ids, general = self._route(todo)
        if keyed:
            for p, v in zip(keyed, self._verify_keyed(keyed, ids)):
                out[id(p)] = bool(v)
            g.stats["batches"] += 1
            g.stats["batch_items"] += len(keyed)
        if general:
            import numpy as np
            sm, off, pk = _pack_sm([p.sig for p in general], [p.ser for p in general], [p.key for p in general])
            ok = self._engine().sign_open_batch(np.frombuffer(sm, np.uint8), np.frombuffer(off, np.uint64),
                                                np.frombuffer(pk, np.uint8).reshape(-1, 32))
            g.stats["batches"] += 1
            g.stats["batch_items"] += len(general)
            for p, v in zip(general, ok):
                out[id(p)] = bool(v)
            self._count_verified(general, ok)
        return [out.get(id(p), False) for p in prepared]

    # -- batch API ----------------------------------------------------------
    def authenticate_batch(self, msgs, identifiers=None, signatures=None):
        """Per message: the identifier authenticate() would return, or the
        exception instance it would raise (same class, args and __cause__)."""
        # (_gc_paused's work inline: entering a context manager allocates, and that allocation could
        # set off the very collection -- over the caller's fresh batch list -- the pause is for)
        was = gc.isenabled()
        gc.disable()
        try:
            if _scan_batch is not None and not identifiers and not signatures and self._native_host_steps():
                return self._authenticate_batch_scanned(msgs)
            return self._authenticate_batch_each(msgs, identifiers, signatures)
        finally:
            if was:
                gc.enable()

    def _native_host_steps(self):
        """The native scan restates GpuAuthMixin._prepare / serializeForSig;
        a subclass that overrides either keeps its own (per-message) path, so
        authenticate() and authenticate_batch() always agree."""
        cls = type(self)
        return cls.serializeForSig is GpuAuthMixin.serializeForSig and cls._prepare is GpuAuthMixin._prepare

    def _key_for(self, identifier):
        """getVerkey + DidVerifier for one identifier (authenticate()'s
        :93-99): the key bytes (None = no key: the verify fails), or the
        exception authenticate() would raise."""
        try:
            verkey = self.getVerkey(identifier)
            if verkey is None:
                raise CouldNotAuthenticate('Can not find verkey for DID {}'.format(identifier))
            return self._key_of(identifier, verkey)
        except SigningException as e:
            return e
        except Exception as ex:
            e = CouldNotAuthenticate()
            e.__cause__ = ex
            return e

    def _keys_for(self, uniq):
        """[_key_for(i) for i in uniq] (getVerkey once per identifier, reference
        order of checks and exceptions), with the per-identifier key fast path
        inlined: a batch's ~1,000 identifiers in well under a millisecond."""
        fk = self._g.fast_keys
        if (_keys_known is not None and type(getattr(self, "clients", None)) is dict and type(fk) is dict
                and uniq.__class__ is list and _known_getverkey(type(self))):
            # getVerkey is SimpleAuthNr's (a clients lookup, the state only for a miss, no side
            # effects): the identifiers whose clients entry is the verkey fast_keys remembers need
            # no Python; the rest (state lookups, exceptions, changed verkeys) take _keys_for_py
            out, holes = _keys_known(self.clients, fk, uniq, VERKEY)
            if holes:
                for j, k in zip(holes, self._keys_for_py([uniq[j] for j in holes])):
                    out[j] = k
            return out
        return self._keys_for_py(uniq)

    def _keys_for_flat(self, uniq):
        """_keys_for(uniq) plus the keys as one buffer of 32 bytes each (zeros
        where a key is not 32 bytes), the positions of those (`odd`), and
        whether every identifier resolved to a key (bytes, non-empty): the
        per-identifier resolution on the scan's worker pool (keys_known_flat),
        the holes (state lookups, exceptions, changed verkeys) in Python."""
        fk = self._g.fast_keys
        if (_keys_known_flat is not None and type(getattr(self, "clients", None)) is dict and type(fk) is dict
                and uniq.__class__ is list and _known_getverkey(type(self))):
            out, holes, flat = _keys_known_flat(self.clients, fk, uniq, VERKEY)
            odd = []
            if holes:
                flat = bytearray(flat)
                for j, k in zip(holes, self._keys_for_py([uniq[j] for j in holes])):
                    out[j] = k
                    if k.__class__ is bytes and len(k) == 32:
                        flat[32 * j:32 * j + 32] = k
                    else:
                        odd.append(j)
            all_keys = not odd or all(out[j].__class__ is bytes and out[j] for j in odd)
            return out, bytes(flat), odd, all_keys
        out = self._keys_for(uniq)
        odd = [j for j, k in enumerate(out) if k.__class__ is not bytes or len(k) != 32]
        flat = b"".join(k if k.__class__ is bytes and len(k) == 32 else bytes(32) for k in out)
        return out, flat, odd, all(out[j].__class__ is bytes and out[j] for j in odd)

    def _keys_for_py(self, uniq):
        """_keys_for in Python: any getVerkey, in the identifiers' order."""
        fk = self._g.fast_keys
        get_verkey = self.getVerkey
        out = []
        append = out.append
        for idr in uniq:
            try:
                verkey = get_verkey(idr)
                e = fk.get(idr)
                if e is not None and e[0] is verkey:
                    append(e[1])
                    continue
                if verkey is None:
                    raise CouldNotAuthenticate('Can not find verkey for DID {}'.format(idr))
                append(self._key_of(idr, verkey))
            except SigningException as ex:
                append(ex)
            except Exception as ex:
                c = CouldNotAuthenticate()
                c.__cause__ = ex
                append(c)
        return out

    @staticmethod
    def _fresh(e):
        """A per-message copy of an exception (same class, args, __cause__)."""
        c = copy.copy(e)
        c.__cause__ = e.__cause__
        return c

    def _authenticate_batch_scanned(self, msgs):
        """authenticate_batch with the host steps in native code: one
        _hostpack.scan_batch_u over the dicts (signature / identifier checks,
        b58decode, serialization, crypto_sign_open's split at byte 64, on
        scan_threads host threads), the verkey resolved once per distinct
        identifier of the batch (getVerkey is called once per identifier, not
        once per message), one GPU launch per path, the result list built
        natively.  Messages the scan leaves to Python (odd types, missing
        fields, bad base58 ...) go through _prepare, which raises the
        reference's exception."""
        from time import perf_counter
        self._g.t_enter = perf_counter()  # (the breakdown's before_scan: buffers, staging reserve)
        eng = self._engine()
        with _engine_lock(eng):
            slot = _SIG_SLOT if getattr(eng, "supports_sig_slots", False) else 64
            bufs = self._scan_buffers(eng, len(msgs), slot)
            part = self._g.pipeline_part
            if part and len(msgs) >= 2 * part and hasattr(eng, "verify_submit") and bufs is not self._g.scan_out:
                return self._authenticate_pipelined(msgs, eng, slot, bufs, part)
            if (self._g.stage and _repack_spans is not None and len(msgs) >= _STAGE_MIN_BATCH
                    and getattr(eng, "supports_staging", False) and slot == _SIG_SLOT and bufs is not self._g.scan_out):
                res = self._authenticate_staged(msgs, eng, slot, bufs)
                if res is _BUSY:  # set 0's pinned buffers may still be feeding that batch's copies
                    return self._authenticate_batch_scanned_into(msgs, self._g.scan_out, slot)
                if res is not None:
                    return res
                bufs = self._scan_buffers(eng, len(msgs), slot)  # regrown from the new size estimate
            if (self._g.stream and _pack_range is not None and len(msgs) >= 2 * _STREAM_CHUNK
                    and hasattr(eng, "verify_submit") and bufs is not self._g.scan_out):
                return self._authenticate_streamed(msgs, eng, slot, bufs)
            return self._authenticate_batch_scanned_into(msgs, bufs, slot)

    def _authenticate_staged(self, msgs, eng, slot, bufs, staging_set=0, defer=False):
        """A large batch whose PCIe copy runs under its scan: the native scan's
        workers place each 4k-request chunk's messages at a bump cursor in the
        engine's pinned memory and queue that chunk's messages and signature
        slots to the device (edv_stage_put) as soon as they are written, so
        by the time the scan returns most of the batch is already in HBM;
        edv_verify_staged then waits for the rest and runs the kernels over
        the item spans.  Batches speculate: the scan
        also writes each request's key id from kid_map (the ids of the batches
        before) and its copier queues the kernels of every 2^16 staged
        requests (edv_verify_staged_part), so the kernels run under the scan
        too; after it, the ids of the batch's distinct identifiers (getVerkey,
        the key store) must equal the ones used and the store must not have
        moved a key (KeyStore.version), else the verify runs again the
        ordinary way -- the verdicts are the ordinary path's either way.  In
        the node's steady state (every item scanned, every identifier
        resolved to a built key); a batch with other items repacks its
        messages contiguously and takes the ordinary path (same verdicts).
        None when the scan could not stage (the pinned buffer was too small
        for this batch, or items needed the interpreter): the caller scans
        again the ordinary way.  staging_set / defer: the pipeline of
        authenticate_batches -- staged into that set of the engine's (and this
        authenticator's) buffers, and in the steady state a callable returning
        the results once the kernels are collected."""
        import numpy as np
        from time import perf_counter
        g = self._g
        n = len(msgs)
        msg_cap = len(bufs[1])
        slot_base = (msg_cap + 255) // 256 * 256
        try:
            if hasattr(eng, "stage_select"):
                eng.stage_select(staging_set)
            eng.stage_reserve(slot_base + n * slot)
        except Exception as ex:
            # the set is busy (EDV_EBUSY: an unfinished authenticate_batches iteration holds its batch
            # in flight there): nothing was scanned or staged, the caller takes the unstaged path.
            # Any other failure (allocation, HIP) is a fault and is raised, not read as busy.
            if defer or getattr(ex, "code", None) != _EDV_EBUSY:
                raise
            return _BUSY
        sfx = "" if staging_set == 0 else str(staging_set)
        spans_buf = self._pinned(eng, "pinned_spans" + sfx, 16 * n)  # the scan writes the item spans here
        kid_buf = self._pinned(eng, "pinned_kid" + sfx, 4 * n)  # key ids straight into pinned memory: no copy
        ks = self._key_store()
        spec, parts = None, None
        if (g.speculate and g.kid_map is not None and ks is not None and _kid_map is not None
                and os.environ.get("EDV_SPECULATE", "1") != "0"
                and spans_buf is not None and kid_buf is not None and getattr(eng, "supports_staged_parts", False)):
            # kid_map's ids are usable only while no slot has been reused since it was made: an
            # eviction, a retired slot or a reset (by anyone sharing the engine: _sync sees it)
            # bumps ks.version, and a slot rebuilt for another key may still be building, so the
            # kernels would read its old or half-written tables.  New keys in free slots do not
            # touch kid_map's slots.
            ks._sync()
            if g.kid_map_version == ks.version:
                ks_version = ks.version
                try:
                    parts = eng.verify_staged_begin(True, n)
                except Exception as ex:  # no speculation for this batch; the ordinary verify follows
                    parts = None
                    g.stats["part_failures"] = g.stats.get("part_failures", 0) + 1
                    g.last_part_error = str(ex)
                if parts is not None:
                    spec = (g.kid_map, kid_buf, eng.parter(), int(os.environ.get("EDV_PART_ITEMS", _PART_ITEMS)))
        t0 = perf_counter()
        try:
            scan = _scan_batch(msgs, [SIG], g.scan_threads, [bufs[0], bufs[1], spans_buf], slot, 2, eng.stager(),
                               slot_base, spec)
        except BaseException:
            if parts is not None:  # free the set the parts held
                for f in (eng.verify_staged_end, lambda: eng.verify_staged_collect(parts)):
                    try:
                        f()
                    except Exception:
                        pass
            raise
        fast_b, uidx_b, uniq, sig_o, msg_o, spans_b, short, staged_ok, spec_u, parts_ok, staged_bytes = scan
        if parts is not None:  # the parts' verdict copy queued after the last part
            try:
                eng.verify_staged_end()
            except Exception as ex:
                parts_ok = False  # a part failed: the verdicts come from the ordinary verify
                g.stats["part_failures"] = g.stats.get("part_failures", 0) + 1
                g.last_part_error = str(ex)  # (the library's message names the part's own failure)
        t1 = perf_counter()

        def drop_parts():  # the speculative verdicts are not used: free the set
            nonlocal parts
            if parts is not None:
                eng.verify_staged_collect(parts)
                parts = None
        try:  # (anything raised before the parts are collected or dropped frees their set)
            if spans_b is spans_buf:
                spans_b = memoryview(spans_b).cast("B")[:16 * n]
            spans = np.frombuffer(spans_b, np.uint64, count=2 * n)
            ms, me = spans[:n], spans[n:]
            if not staged_ok:
                drop_parts()
                g.msg_bytes_per_item *= 1.5  # the next buffers are sized larger
                return None
            # (the chunks' reservations are contiguous from 0: their total is the largest span end)
            g.msg_bytes_per_item = max(g.msg_bytes_per_item * 0.5, float(staged_bytes) / n if n else 0.0)
            # authenticate():93-99, once per identifier (on the worker pool; the keys also as one buffer)
            ukeys, uflat, uodd, all_keys = self._keys_for_flat(uniq)
            tk = g.t_ids_of = perf_counter()
            ids = None
            general_u = None  # distinct identifiers whose key has no built table: the general path
            tr = tk
            if ks is not None and fast_b.count(0) == 0 and all_keys:
                pre = None
                if g.hot or g.pending:  # (the batch's keys pinned by id: one native lookup)
                    pre = ks.ids_of(uflat, uodd, ukeys) if g.hot else None
                    g.t_ids_of = perf_counter()
                    v0 = ks.version
                    got = self._register_waiting(ks, ukeys, pre)
                    if got or ks.version != v0:
                        pre = None  # (a key of this batch may have been registered: look up again)
                tr = perf_counter()
                ids = ks.lookup_array(ukeys, uflat, uodd, pre)
                if (ids < 0).any():
                    general_u = np.flatnonzero(ids < 0)
                    ids[general_u] = 0xffffffff  # (an id the kernels reject)
                ids = ids.astype(np.uint32)
            if ids is None:  # not the steady state: contiguous messages, the ordinary path
                drop_parts()
                del spans, ms, me
                msg_c, off_c = _repack_spans(msg_o, spans_b)
                return self._finish_scanned(msgs, (fast_b, uidx_b, uniq, sig_o, msg_c, off_c, short), slot, ukeys)
            if general_u is not None:  # a mixed batch (key churn): the keyed verify, then the rest
                drop_parts()
                return self._staged_mixed(msgs, eng, slot, slot_base, ks, ukeys, ids, general_u, scan, spans_buf,
                                          kid_buf, t0, t1, None if uodd else uflat, (tk, tr))
            ids_b = np.asarray(ids, np.uint32).tobytes()
            spec_hit = parts is not None and parts_ok and spec_u == ids_b and ks.version == ks_version
            if g.speculate and _kid_map is not None and (spec_u != ids_b or g.kid_map is None or
                                                         g.kid_map_version != ks.version):
                # remember this batch's ids for the next batch's scan (a fresh map when the store moved keys)
                fresh = g.kid_map is None or g.kid_map_version != ks.version or _kid_map_size(g.kid_map) > g.kid_map_max
                g.kid_map = _kid_map(None if fresh else g.kid_map, uniq, ids_b)
                g.kid_map_version = ks.version
            t2 = perf_counter()
            g.stats["batches"] += 1
            g.stats["batch_items"] += n
            g.stats["keyed_items"] += n
            g.stats["speculated"] = g.stats.get("speculated", 0) + (n if spec_hit else 0)

            def verdicts(ok, t3):
                results, failed = _results_failing(ok, short, uidx_b, uniq)
                t4 = perf_counter()
                g.last_breakdown = {"before_scan": (t0 - getattr(g, "t_enter", t0)) * 1e3,
                                    "scan_and_copies": (t1 - t0) * 1e3, "keys_and_ids": (t2 - t1) * 1e3,
                                    "verify_wait": (t3 - t2) * 1e3, "verdicts": (t4 - t3) * 1e3,
                                    "speculated": bool(spec_hit)}
                return results
            if spec_hit:  # the kernels ran under the scan with exactly these ids
                ticket, parts = parts, None
                del spans, ms, me, spans_b
                if defer:  # (they may still run: collected when the caller asks for the results)
                    def finish_spec():
                        with _engine_lock(eng):
                            ok = np.asarray(eng.verify_staged_collect(ticket), bool)
                        return verdicts(ok, perf_counter())
                    return finish_spec
                ok = np.asarray(eng.verify_staged_collect(ticket), bool)
                return verdicts(ok, perf_counter())
        except BaseException:
            if parts is not None:
                try:
                    eng.verify_staged_collect(parts)
                except Exception:
                    pass
            raise
        drop_parts()
        kid = np.frombuffer(_gather_u32(ids_b, uidx_b, kid_buf if kid_buf is not None else g.kid_out), np.uint32,
                            count=n)
        if defer:  # the kernels run while the caller goes on (its next batch's scan)
            handle = eng.verify_staged_submit(True, kid, slot_base, 0, ms, me)
            t2 = perf_counter()
            del kid, spans, ms, me, spans_b

            def finish():
                with _engine_lock(eng):
                    ok = np.asarray(eng.verify_staged_collect(handle), bool)
                return verdicts(ok, perf_counter())
            return finish
        ok = np.asarray(eng.verify_staged(True, kid, slot_base, 0, ms, me), bool)
        del kid, spans, ms, me, spans_b
        return verdicts(ok, perf_counter())

    def _staged_mixed(self, msgs, eng, slot, slot_base, ks, ukeys, ids, general_u, scan, spans_buf, kid_buf, t0, t1,
                      uflat=None, t_keys=None):
        """A staged batch whose identifiers' keys are partly without a built
        table (a signer population larger than the key store): one keyed
        verify of the whole staged batch over the store's ids (the others get
        an id the kernels reject), then the general path (the key bytes) for
        the items of the other identifiers only -- on the engine's copy of the
        staged batch (edv_verify_staged_subset: indices and keys cross PCIe),
        or gathered from the pinned buffers -- the same verdicts as per
        message."""
        import numpy as np
        from time import perf_counter
        g = self._g
        fast_b, uidx_b, uniq, sig_o, msg_o, spans_b, short = scan[:7]
        n = len(msgs)
        if spans_b is spans_buf:
            spans_b = memoryview(spans_b).cast("B")[:16 * n]
        spans = np.frombuffer(spans_b, np.uint64, count=2 * n)
        kid = np.frombuffer(_gather_u32(np.asarray(ids, np.uint32).tobytes(), uidx_b,
                                        kid_buf if kid_buf is not None else g.kid_out), np.uint32, count=n)
        t2 = perf_counter()
        # the keyed verify queued first; the general items' indices and keys are gathered while it runs
        handle = eng.verify_staged_submit(True, kid, slot_base, 0, spans[:n], spans[n:]) \
            if hasattr(eng, "verify_staged_submit") else None
        ok = None if handle is not None else np.array(eng.verify_staged(True, kid, slot_base, 0, spans[:n],
                                                                        spans[n:]), bool)
        try:
            uidx = np.frombuffer(uidx_b, np.uint32, count=n)
            is_gen = np.zeros(len(ukeys), np.uint8)
            is_gen[general_u] = 1
            if uflat is not None and len(uflat) == 32 * len(ukeys):
                ukey_flat = uflat  # (the general keys are 32 B)
            else:
                ukey_arr = np.zeros((len(ukeys), 32), np.uint8)
                ukey_arr[general_u] = np.frombuffer(b"".join(ukeys[u] for u in general_u), np.uint8).reshape(-1, 32)
                ukey_flat = ukey_arr.tobytes()
            if _general_items is not None:  # (positions and their keys in one parallel pass)
                gen_b, keys_b = _general_items(uidx, is_gen, ukey_flat)
                gen = np.frombuffer(gen_b, np.uint32)
                gen_keys = np.frombuffer(keys_b, np.uint8).reshape(-1, 32)
            else:
                gen = np.flatnonzero(is_gen[uidx]).astype(np.uint32)
                gen_keys = np.frombuffer(ukey_flat, np.uint64).reshape(-1, 4).take(uidx[gen], axis=0).view(
                    np.uint8).reshape(-1, 32)
        except BaseException:
            if handle is not None:  # (the set is freed before the error propagates)
                eng.verify_staged_collect(handle)
            raise
        tg = perf_counter()
        if handle is not None:
            ok = np.array(eng.verify_staged_collect(handle), bool)
        tw = perf_counter()
        if len(gen):
            if getattr(eng, "supports_staged_subset", False):
                # the staged batch is still in HBM: only the items' indices and key bytes go over
                okg = np.asarray(eng.verify_staged_subset(gen, gen_keys), bool)
            else:
                s_sig, s_msg, s_off = _gather_spans(memoryview(sig_o).cast("B")[:slot * n], msg_o, spans_b,
                                                    gen.astype(np.uint32).tobytes(), slot)
                okg = np.asarray(eng.verify_batch(np.frombuffer(s_sig, np.uint8).reshape(-1, slot),
                                                  gen_keys, np.frombuffer(s_msg, np.uint8),
                                                  np.frombuffer(s_off, np.uint64),
                                                  **({"sig_slot": slot} if slot != 64 else {})), bool)
            ok[gen] = okg
            tv = perf_counter()
            # general-path keys earn a slot by verified requests (short items never verify)
            good = gen[okg & (np.frombuffer(short, np.uint8)[gen] == 0)]
            per_u = np.bincount(uidx[good], minlength=len(ukeys))
            # (keys with fewer verified requests in this batch than 1/HOT_COUNT_FLOOR of the threshold
            # cannot reach it through the decay: not counted -- the long tail of a churning batch)
            floor = max(1, g.hot_key_uses // HOT_COUNT_FLOOR)
            if uflat is not None and len(uflat) == 32 * len(ukeys) and g.key_uses.native:
                if g.max_keys > 0:  # the batch's flat key buffer counted natively: no per-key Python
                    for j in g.key_uses.add_flat(uflat, per_u, self._use_epoch(), g.hot_key_uses, floor).tolist():
                        g.hot[ukeys[j]] = None
            else:
                hot_u = np.flatnonzero(per_u >= floor).tolist()
                self._count_verified_keys([ukeys[u] for u in hot_u], per_u[hot_u])
        else:
            tv = tw
        t3 = perf_counter()
        g.stats["batches"] += 1
        g.stats["batch_items"] += n
        g.stats["keyed_items"] += n - len(gen)
        results, failed = _results_failing(ok, short, uidx_b, uniq)
        g.last_breakdown = {"before_scan": (t0 - getattr(g, "t_enter", t0)) * 1e3,
                            "scan_and_copies": (t1 - t0) * 1e3, "keys_and_ids": (t2 - t1) * 1e3,
                            "verify_wait": (t3 - t2) * 1e3, "verdicts": (perf_counter() - t3) * 1e3,
                            "speculated": False, "general_items": int(len(gen)),
                            # keys_and_ids' parts: the batch's keys resolved, slots registered, ids
                            # looked up (and the kid gather); verify_wait's: the general items'
                            # keys gathered under the keyed verify, its wait, the general
                            # verify, the verified-use counts
                            "parts_ms": {k: round(v * 1e3, 3) for k, v in (
                                (("keys", t_keys[0] - t1), ("register", t_keys[1] - t_keys[0]),
                                 ("ids_of", max(0.0, getattr(g, "t_ids_of", t_keys[0]) - t_keys[0])),
                                 ("ids", t2 - t_keys[1])) if t_keys else ()) + (
                                ("gather", tg - t2), ("keyed_wait", tw - tg), ("general", tv - tw),
                                ("count", t3 - tv))}}
        return results

    def _speculation_ready(self):
        """The next staged batch would speculate: a key-id map from the batches before that no key
        store change has invalidated (_authenticate_staged's condition)."""
        g = self._g
        if not (g.speculate and g.kid_map is not None and _kid_map is not None
                and os.environ.get("EDV_SPECULATE", "1") != "0"
                and getattr(self._engine(), "supports_staged_parts", False)):
            return False
        ks = self._key_store()
        if ks is None:
            return False
        ks._sync()
        return g.kid_map_version == ks.version

    def authenticate_batches(self, batches):
        """authenticate_batch over an iterable of batches, yielding each batch's
        result list in order, with two batches in flight: batch k + 1's host
        scan (and its PCIe copy, staged under it) runs while batch k's kernels
        run on the GPU -- the engine's two staging sets (edv_stage_select,
        edv_verify_staged_submit / _collect) and two sets of this
        authenticator's pinned buffers alternate.  A node verifying drain after
        drain ahead of handling them gets the same.  Batches outside the
        staged steady state (small, or items the scan leaves to Python, or
        keys not yet built) are finished synchronously, after the batch in
        flight; every outcome equals authenticate_batch's.  Other calls on
        this authenticator must not interleave with an unfinished iteration."""
        eng = self._engine()
        slot = _SIG_SLOT if getattr(eng, "supports_sig_slots", False) else 64
        can = (self._g.stage and _scan_batch is not None and _repack_spans is not None and slot == _SIG_SLOT and
               getattr(eng, "supports_staging", False) and hasattr(eng, "verify_staged_submit") and
               self._native_host_steps())
        pending = None
        k = 0
        try:
            for msgs in batches:
                res = None
                if can and len(msgs) >= _STAGE_MIN_BATCH and pending is None and self._speculation_ready():
                    # the steady state: this batch's kernels run under its own scan (speculation), so
                    # there is no GPU work left to overlap with the next batch -- one staging set, the
                    # synchronous batch (two sets in flight measured slower there: profiles/r10f, r10h)
                    yield self.authenticate_batch(msgs)
                    continue
                if can and len(msgs) >= _STAGE_MIN_BATCH:
                    with _engine_lock(eng), _gc_paused():
                        self._g.t_enter = _perf_counter()
                        s = k % 2
                        bufs = self._scan_buffers(eng, len(msgs), slot, s)
                        if bufs is not self._g.scan_out:
                            res = self._authenticate_staged(msgs, eng, slot, bufs, staging_set=s, defer=True)
                if callable(res):
                    prev, pending = pending, res  # (held first: a close() at the yield collects it)
                    k += 1
                    if prev is not None:
                        with _gc_paused():
                            out = prev()
                        yield out
                    continue
                if pending is not None:  # the batch in flight first (its staging set is free after)
                    done, pending = pending, None
                    with _gc_paused():
                        out = done()
                    yield out
                yield res if res is not None else self.authenticate_batch(msgs)
            if pending is not None:
                done, pending = pending, None
                with _gc_paused():
                    out = done()
                yield out
        finally:
            if pending is not None:  # an iteration abandoned with a batch in flight: free its staging set
                pending()

    def _authenticate_streamed(self, msgs, eng, slot, bufs):
        """A large batch whose pack overlaps its DMA: one scan of the whole
        batch with the pack deferred (scan_batch_u defer=1), then per
        library chunk of 2^18 requests the pack of its messages into pinned
        memory (pack_range) and edv_verify_submit, so chunk c's copy engine
        and kernels run while chunk c + 1 packs; one collect per chunk.  In
        the node's steady state (every item scanned, every identifier
        resolved to a built key); any other batch packs whole and takes the
        ordinary path (same verdicts)."""
        import numpy as np
        from time import perf_counter
        g = self._g
        n = len(msgs)
        t0 = perf_counter()
        scan = _scan_batch(msgs, [SIG], g.scan_threads, bufs, slot, 1)
        t1 = perf_counter()
        fast_b, uidx_b, uniq, sig_o, msg_o, off, short, handle = scan
        off_a = np.frombuffer(off, np.uint64)
        mlen = int(off_a[-1])
        g.msg_bytes_per_item = max(g.msg_bytes_per_item * 0.5, mlen / n)
        ukeys = self._keys_for(uniq)  # authenticate():93-99, once per identifier
        ids = None
        ks = self._key_store()
        if ks is not None and fast_b.count(0) == 0 and all(k.__class__ is bytes for k in ukeys):
            if g.hot or g.pending:
                self._register_waiting(ks, list(dict.fromkeys(ukeys)))
            ids = ks.lookup(ukeys)
            if any(i is None for i in ids):
                ids = None
        if ids is None:  # not the steady state: the whole batch packed, the ordinary path
            _pack_range(handle, 0, n)
            return self._finish_scanned(msgs, scan[:7], slot, ukeys)
        kid = np.frombuffer(_gather_u32(np.asarray(ids, np.uint32).tobytes(), uidx_b, g.kid_out), np.uint32, count=n)
        sig_a = np.frombuffer(sig_o, np.uint8, count=slot * n).reshape(-1, slot)
        msg_a = np.frombuffer(msg_o, np.uint8, count=mlen)
        t2 = perf_counter()
        handles, oks = [], []
        try:
            for c0 in range(0, n, _STREAM_CHUNK):
                c1 = min(n, c0 + _STREAM_CHUNK)
                _pack_range(handle, c0, c1)
                if len(handles) - len(oks) >= _STREAM_WINDOW:  # bounded in flight (the library holds 64 tickets)
                    oks.append(np.asarray(eng.verify_collect(handles[len(oks)]), bool))
                handles.append(eng.verify_submit(sig_a[c0:c1], kid[c0:c1], msg_a, off_a[c0:c1 + 1], True, slot))
            t3 = perf_counter()
            while len(oks) < len(handles):
                oks.append(np.asarray(eng.verify_collect(handles[len(oks)]), bool))
        finally:
            _collect_quietly(eng, handles[len(oks):])  # an exception between submit and collect: free the tickets
        ok = np.concatenate(oks) if oks else np.zeros(0, bool)
        t4 = perf_counter()
        del handles, oks, sig_a, msg_a, kid
        g.stats["batches"] += 1
        g.stats["batch_items"] += n
        g.stats["keyed_items"] += n
        results, failed = _results_failing(ok, short, uidx_b, uniq)
        t5 = perf_counter()
        # where this batch's time went (bench.py end_to_end.in_batch_ms)
        g.last_breakdown = {"scan": (t1 - t0) * 1e3, "keys_and_ids": (t2 - t1) * 1e3,
                            "pack_and_submit": (t3 - t2) * 1e3, "collect_wait": (t4 - t3) * 1e3,
                            "verdicts": (t5 - t4) * 1e3}
        return results

    def _authenticate_pipelined(self, msgs, eng, slot, bufs, part):
        """A large batch in parts of `part` requests: the scan of part k + 1
        (host threads) runs while part k's copies and kernels run on the GPU
        (edv_verify_submit / edv_verify_collect).  Each part's scan writes into
        its own stretch of the pinned buffers.  A part in the node's steady
        state (every item scanned, every identifier resolved to a registered
        key) is submitted asynchronously; any other part takes the ordinary
        path synchronously (same verdicts either way).  getVerkey is called
        once per distinct identifier of the whole batch.  At most
        _STREAM_WINDOW parts are in flight (the library holds kMaxPending
        tickets); a part that raises leaves no ticket behind."""
        import numpy as np
        g = self._g
        n = len(msgs)
        ks = self._key_store()
        memo = {}
        sig_mv = memoryview(bufs[0]).cast("B")
        msg_mv = memoryview(bufs[1]).cast("B")
        mpos, mtotal = 0, 0
        parts = []
        inflight = []  # indices into parts of the submitted, uncollected parts (oldest first)

        def collect(j):
            handle, uidx_b, uniq, short = parts[j][1]
            ok = np.asarray(eng.verify_collect(handle), bool) & (np.frombuffer(short, np.uint8) == 0)
            res = _results_from(ok.view(np.uint8).tobytes(), uidx_b, uniq)
            for i in np.flatnonzero(~ok).tolist():
                res[i] = InvalidSignature()
            parts[j] = ("done", res)
        try:
            for lo in range(0, n, part):
                hi = min(n, lo + part)
                chunk = msgs[lo:hi]
                out = [sig_mv[lo * slot:hi * slot], msg_mv[mpos:]]
                scan = _scan_batch(chunk, [SIG], g.scan_threads, out, slot)
                fast_b, uidx_b, uniq, sig_o, msg_o, off, short = scan
                mlen = int(np.frombuffer(off, np.uint64)[-1])
                mtotal += mlen
                if msg_o is out[1]:
                    mpos += mlen
                ukeys = []
                for idr in uniq:
                    k = memo.get(idr, _MISSING)
                    if k is _MISSING:
                        k = memo[idr] = self._key_for(idr)  # authenticate():93-99, once per identifier
                    ukeys.append(k)
                ids = None
                if ks is not None and fast_b.count(0) == 0 and all(k.__class__ is bytes for k in ukeys):
                    ids = ks.lookup(ukeys)
                    if any(i is None for i in ids):
                        ids = None
                if ids is None:  # not the steady state: this part the ordinary way
                    parts.append(("done", self._finish_scanned(chunk, scan, slot, ukeys)))
                    continue
                if len(inflight) >= _STREAM_WINDOW:  # bounded in flight
                    collect(inflight.pop(0))
                kid = np.asarray(ids, np.uint32)[np.frombuffer(uidx_b, np.uint32)]
                handle = eng.verify_submit(np.frombuffer(sig_o, np.uint8, count=slot * (hi - lo)).reshape(-1, slot),
                                           kid, np.frombuffer(msg_o, np.uint8, count=mlen),
                                           np.frombuffer(off, np.uint64), True, slot)
                parts.append(("async", (handle, uidx_b, uniq, short)))
                inflight.append(len(parts) - 1)
                g.stats["batches"] += 1
                g.stats["batch_items"] += hi - lo
                g.stats["keyed_items"] += hi - lo
            while inflight:
                collect(inflight[0])
                inflight.pop(0)
        finally:
            _collect_quietly(eng, [parts[j][1][0] for j in inflight])
        if n:
            g.msg_bytes_per_item = max(g.msg_bytes_per_item * 0.5, mtotal / n)
        results = []
        for _, payload in parts:
            results += payload
        return results

    def _pinned(self, eng, name, nbytes):
        """A pinned host buffer of at least nbytes kept on the state under `name`
        (engine.host_alloc; grown by half again when short, never shrunk), or
        None without pinned memory."""
        g = self._g
        buf = g.__dict__.get(name)
        if buf is not None and len(buf) >= nbytes:
            return buf
        alloc = getattr(eng, "host_alloc", None)
        if alloc is None:
            return None
        try:
            buf = alloc(max(int(nbytes * 1.25) + 4096, int(len(buf) * 1.5) if buf is not None else 0))
        except Exception:
            return None
        g.__dict__[name] = buf
        return buf

    def _scan_buffers(self, eng, n, slot, staging_set=0):
        """The scan's output buffers for an n-request batch: the engine's pinned
        host memory (host_alloc) when it has some -- the GPU call then copies
        from them with no staging copy -- grown ahead of need (never shrunk),
        else the reused bytearrays.  staging_set 1: the second set of the
        pipeline (authenticate_batches)."""
        g = self._g
        alloc = getattr(eng, "host_alloc", None)
        if alloc is None or n < _PINNED_MIN_BATCH:
            return g.scan_out
        need = (n * slot, int(n * g.msg_bytes_per_item * 1.25) + (64 << 10))
        if staging_set:
            bufs = g.__dict__.get("pinned_out1")
            if bufs is None or any(len(b) < k for b, k in zip(bufs, need)):
                old = [len(b) for b in bufs] if bufs else [0, 0]
                try:
                    bufs = [alloc(max(k, int(o * 1.5))) for k, o in zip(need, old)]
                except Exception:
                    return g.scan_out
                g.__dict__["pinned_out1"] = bufs
            return bufs
        bufs = g.pinned_out
        if bufs is None or any(len(b) < k for b, k in zip(bufs, need)):
            old = [len(b) for b in bufs] if bufs else [0, 0]
            try:
                bufs = [alloc(max(k, int(o * 1.5))) for k, o in zip(need, old)]
            except Exception:
                return g.scan_out  # no pinned memory: the library stages (correct, slower)
            g.pinned_out = bufs
        return bufs

    def _authenticate_batch_scanned_into(self, msgs, out, slot=64):
        import numpy as np
        n = len(msgs)
        g = self._g
        scan = _scan_batch(msgs, [SIG], g.scan_threads, out, slot)
        mlen = int(np.frombuffer(scan[5], np.uint64)[-1])
        if n:
            g.msg_bytes_per_item = max(g.msg_bytes_per_item * 0.5, mlen / n)  # sizes the next batch's buffer
        return self._finish_scanned(msgs, scan, slot)

    def _finish_scanned(self, msgs, scan, slot, ukeys=None):
        """Everything after the native scan of msgs: key resolution, the
        verify launches, the result list."""
        import numpy as np
        n = len(msgs)
        fast_b, uidx_b, uniq, sig_o, msg_o, off, short = scan
        # views of exactly this batch's bytes (released when the batch returns, so the next
        # batch may grow the buffers again)
        mlen = int(np.frombuffer(off, np.uint64)[-1])
        sig64 = memoryview(sig_o)[:slot * n]
        mbuf = memoryview(msg_o)[:mlen]
        fast = np.frombuffer(fast_b, np.uint8).view(bool)
        uidx = np.frombuffer(uidx_b, np.uint32)
        if ukeys is None:
            ukeys = self._keys_for(uniq)  # authenticate():93-99, once per identifier
        # per distinct identifier: 0 = key bytes, 1 = no key (the verify fails), 2 = exception
        ucls = np.fromiter((0 if k.__class__ is bytes else 1 if k is None else 2 for k in ukeys), np.uint8,
                           len(ukeys))
        if n and fast_b.count(0) == 0 and not (ucls == 2).any():
            # every item scanned and every identifier resolved (the node's steady state): no index
            # arrays over the batch
            ok = self._verify_scanned(None, uidx, ukeys, ucls, sig64, mbuf, off, short, slot)
            results = _results_from(ok.view(np.uint8).tobytes(), uidx_b, uniq)
            for i in np.flatnonzero(~ok).tolist():
                results[i] = InvalidSignature()
            return results
        fidx = np.nonzero(fast)[0]
        icls = ucls[uidx[fidx]] if len(fidx) else np.zeros(0, np.uint8)
        vidx = fidx[icls != 2]  # the items that reach the verify
        codes = np.zeros(n, np.uint8)
        ok = self._verify_scanned(vidx, uidx, ukeys, ucls, sig64, mbuf, off, short, slot) if len(vidx) else \
            np.zeros(0, bool)
        codes[vidx[ok]] = 1
        results = _results_from(codes.tobytes(), uidx_b, uniq)  # the identifier where verified
        for i in vidx[~ok].tolist():
            results[i] = InvalidSignature()
        for i in fidx[icls == 2].tolist():
            results[i] = self._fresh(ukeys[uidx[i]])
        slow = np.nonzero(~fast)[0].tolist()
        if slow:
            for i, r in zip(slow, self._authenticate_batch_each([msgs[i] for i in slow])):
                results[i] = r
        return results

    def _verify_scanned(self, vidx, uidx, ukeys, ucls, sig64, mbuf, off, short, slot=64):
        """Verdicts of the scanned items vidx (None: every item; split sig64 /
        messages of the whole batch; item i's key = ukeys[uidx[i]]): registered
        keys on the key-table path, the rest one general launch, no key -> False.
        slot = 96: sig64 holds the scan's signature slots (base58 text decoded
        on the GPU, edverify.h EDV_SIG_SLOT96)."""
        import numpy as np
        g = self._g
        everything = vidx is None
        m = len(uidx) if everything else len(vidx)
        item_u = uidx if everything else uidx[vidx]
        short_a = np.frombuffer(short, np.uint8).view(bool)
        if not everything:
            short_a = short_a[vidx]
        ok = np.zeros(m, bool)
        has_key = np.nonzero(ucls == 0)[0]
        ukey_list = [ukeys[u] for u in has_key.tolist()]
        uniq_keys = list(dict.fromkeys(ukey_list))
        kid_u = np.full(len(ukeys), -2, np.int64)  # -2: no key, -1: general path, >= 0: key-store id
        kid_u[has_key] = -1
        ks = self._key_store()
        if ks is not None and uniq_keys:
            self._register_waiting(ks, uniq_keys)
            id_of = {k: i for k, i in zip(uniq_keys, ks.lookup(uniq_keys)) if i is not None}
            kid_u[has_key] = [id_of.get(k, -1) for k in ukey_list]
        # the items of each path: a whole-batch slice when one path takes them all
        if (kid_u >= 0).all():
            groups, general = [(slice(None), True)], np.zeros(0, np.int64)
        elif (kid_u == -1).all():
            groups, general = [(slice(None), False)], np.arange(m)
        else:
            kid = kid_u[item_u]
            general = np.nonzero(kid == -1)[0]
            groups = [(np.nonzero(kid >= 0)[0], True), (general, False)]
        eng = self._engine()
        whole = m == len(uidx)
        for sel, is_keyed in groups:
            cnt = m if isinstance(sel, slice) else len(sel)
            if not cnt:
                continue
            if whole and cnt == m:
                s_sig, s_msg, s_off = sig64, mbuf, off
            else:
                s_sig, s_msg, s_off = _gather_items(sig64, mbuf, off,
                                                    (np.arange(m) if everything else vidx)[sel].astype(np.uint32)
                                                    .tobytes(), slot)
            s_sig = np.frombuffer(s_sig, np.uint8).reshape(-1, slot)
            s_msg, s_off = np.frombuffer(s_msg, np.uint8), np.frombuffer(s_off, np.uint64)
            kw = {"sig_slot": slot} if slot != 64 else {}
            if is_keyed:
                v = eng.verify_batch_keyed(s_sig, kid_u.astype(np.uint32)[item_u[sel]], s_msg, s_off, **kw)
                g.stats["keyed_items"] += cnt
            else:
                ukey_arr = np.zeros((len(ukeys), 32), np.uint8)
                ukey_arr[has_key] = np.frombuffer(b"".join(ukey_list), np.uint8).reshape(-1, 32)
                v = eng.verify_batch(s_sig, ukey_arr[item_u[sel]], s_msg, s_off, **kw)
            ok[sel] = np.asarray(v, bool)
            g.stats["batches"] += 1
            g.stats["batch_items"] += cnt
        ok &= ~short_a
        if len(general):  # general-path keys earn a slot by verified requests
            verified_u = np.bincount(item_u[general[ok[general]]], minlength=len(ukeys))
            per_key = {}
            for u in np.nonzero(verified_u)[0].tolist():
                per_key[ukeys[u]] = per_key.get(ukeys[u], 0) + int(verified_u[u])
            self._count_verified_keys(list(per_key), list(per_key.values()))
        return ok

    def _authenticate_batch_each(self, msgs, identifiers=None, signatures=None):
        n = len(msgs)
        identifiers = identifiers or [None] * n
        signatures = signatures or [None] * n
        results = [None] * n
        prepared, where = [], []
        for i, msg in enumerate(msgs):
            try:
                prepared.append(self._prepare(msg, identifiers[i], signatures[i]))
                where.append(i)
            except SigningException as e:
                results[i] = e
            except Exception as ex:
                e = CouldNotAuthenticate()
                e.__cause__ = ex
                results[i] = e
        for i, p, ok in zip(where, prepared, self._verify_many(prepared)):
            results[i] = p.identifier if ok else InvalidSignature()
        return results

    def prefetch(self, msgs):
        """Verify-ahead: batch-verify every message that gets as far as the
        verify step, and cache the verdicts for authenticate().  Returns the
        number of distinct signatures verified.  The host steps run in the
        native scan (as in authenticate_batch), the drain's copies of a
        request are verified once (distinct (identifier, sig || ser)), and
        the verdict cache is written under the engine lock."""
        if _scan_batch is not None and _distinct_sm is not None and self._native_host_steps():
            return self._prefetch_scanned(msgs)
        prepared = []
        for msg in msgs:
            try:
                prepared.append(self._prepare(msg))
            except Exception:
                continue  # authenticate() will raise it again
        return self._prefetch_prepared(prepared)

    def _prefetch_prepared(self, prepared):
        verdicts = self._g.verdicts
        uniq = OrderedDict()
        for p in prepared:
            k = self._vkey(p)
            if k not in verdicts and k not in uniq:
                uniq[k] = p
        items = list(uniq.items())
        with _engine_lock(self._engine()):
            oks = self._verify_many_locked([p for _, p in items])
            for (k, p), ok in zip(items, oks):
                self._remember(p, ok, k)
        self._g.stats["prefetched"] += len(items)
        return len(items)

    def _prefetch_scanned(self, msgs):
        import numpy as np
        g = self._g
        eng = self._engine()
        with _engine_lock(eng):
            # slot 64: sig64 holds sm[:64], the message buffer sm[64:] (the split at byte 64)
            fast_b, uidx_b, uniq, sig_o, msg_o, off, short = _scan_batch(msgs, [SIG], g.scan_threads, g.scan_out, 64)
            n = len(msgs)
            picks, sms = _distinct_sm(memoryview(sig_o)[:64 * n], msg_o, off, short, uidx_b, fast_b)
        ukeys = {}
        uidx = np.frombuffer(uidx_b, np.uint32)
        verdicts = g.verdicts
        prepared, seen = [], set()
        for i, sm in zip(picks, sms):
            u = int(uidx[i])
            key = ukeys.get(u, _MISSING)
            if key is _MISSING:
                key = ukeys[u] = self._key_for(uniq[u])  # getVerkey + DidVerifier, once per identifier
            if key.__class__ is not bytes or not key:
                continue  # no key (False without a verify) or an exception: authenticate() raises it
            vk = (key, sm)
            if vk in verdicts or vk in seen:
                continue
            seen.add(vk)
            prepared.append(_Prepared(uniq[u], sm[:64], sm[64:], key))
        slow = [msgs[i] for i in np.flatnonzero(np.frombuffer(fast_b, np.uint8) == 0).tolist()]
        for msg in slow:  # items the scan left to Python (odd types, non-ASCII, bad base58 ...)
            try:
                prepared.append(self._prepare(msg))
            except Exception:
                continue  # authenticate() will raise it again
        return self._prefetch_prepared(prepared)

    def clear_verdicts(self):
        self._g.verdicts.clear()
        self._g.verdict_bytes = 0
        self._g.verdict_epochs.clear()

    # -- multi-signature extension (parity unpinned) --------------------------
    def _prepare_multi(self, msg, signatures, threshold):
        """Host half of authenticate_multi; returns (threshold, steps) where a
        step is an exception to raise or a prepared item, in dict order."""
        num_sigs = len(signatures)
        if threshold is not None:
            if num_sigs < threshold:
                raise InsufficientSignatures(num_sigs, threshold)
        else:
            threshold = num_sigs
        ser = None
        steps = []
        for idr, signature in signatures.items():
            try:
                try:
                    sig = b58decode(signature)
                except Exception as ex:
                    raise InvalidSignatureFormat from ex
                if ser is None:
                    ser = self.serializeForSig(msg, topLevelKeysToIgnore=[SIG, SIGS])
                verkey = self.getVerkey(idr)
                if verkey is None:
                    raise CouldNotAuthenticate('Can not find verkey for {}'.format(idr))
                steps.append(_Prepared(idr, sig, ser, self._resolve_key(verkey, idr)))
            except Exception as ex:
                steps.append(ex)
        return threshold, steps

    @staticmethod
    def _finish_multi(threshold, steps, verdict):
        correct = []
        for st in steps:
            if isinstance(st, Exception):
                raise st
            if verdict(st):
                correct.append(st.identifier)
                if len(correct) == threshold:
                    return correct
        raise InsufficientCorrectSignatures(len(correct), threshold)

    def authenticate_multi(self, msg, signatures, threshold=None):
        """Identifiers whose signatures over msg (minus top-level 'signature'
        and 'signatures') verify, in dict order, stopping at `threshold`
        (default: all).  Raises InsufficientSignatures if fewer signatures
        than the threshold are given, InsufficientCorrectSignatures if too
        few verify, or the first per-signature error reached in order."""
        threshold, steps = self._prepare_multi(msg, signatures, threshold)
        items = [s for s in steps if not isinstance(s, Exception)]
        verdicts = dict(zip(map(id, items), self._verify_many(items)))
        return self._finish_multi(threshold, steps, lambda p: verdicts[id(p)])

    def authenticate_multi_batch(self, reqs):
        """reqs: iterable of (msg, signatures, threshold).  One GPU launch for
        every signature of every request; per request the result list or the
        exception authenticate_multi would raise."""
        staged, items = [], []
        for msg, sigs, thr in reqs:
            try:
                threshold, steps = self._prepare_multi(msg, sigs, thr)
                staged.append((threshold, steps))
                items.extend(s for s in steps if not isinstance(s, Exception))
            except Exception as ex:
                staged.append(ex)
        verdicts = dict(zip(map(id, items), self._verify_many(items)))
        out = []
        for st in staged:
            if isinstance(st, Exception):
                out.append(st)
                continue
            try:
                out.append(self._finish_multi(st[0], st[1], lambda p: verdicts[id(p)]))
            except Exception as ex:
                out.append(ex)
        return out


class ClientAuthNr:
    """Interface for client authenticators (client_authn.py:22-63)."""

    @abstractmethod
    def authenticate(self, msg: Dict, identifier: str = None, signature: str = None) -> str:
        """Return the identifier or raise a SigningException subclass."""

    @abstractmethod
    def addIdr(self, identifier, verkey, role=None):
        """Register an identifier's verification key."""

    @abstractmethod
    def getVerkey(self, identifier):
        """Verification key of an identifier."""


class NaclAuthNr(GpuAuthMixin, ClientAuthNr):
    """client_authn.py:66-119 with the Ed25519 check on the GPU engine.
    Subclasses provide addIdr / getVerkey."""

    @abstractmethod
    def addIdr(self, identifier, verkey, role=None):
        pass

    @abstractmethod
    def getVerkey(self, identifier):
        pass


class SimpleAuthNr(NaclAuthNr):
    """client_authn.py:122-154.  `state` lookups for identifiers not added with
    addIdr go through `nym_lookup(state, identifier)` (the reference calls
    DomainRequestHandler.getNymDetails(state, identifier, isCommitted=False),
    domain_req_handler.py:146-155); with no lookup the state is empty."""

    def __init__(self, state=None, nym_lookup=None):
        self.clients = {}  # type: Dict[str, Dict]
        self.state = state
        self.nym_lookup = nym_lookup

    def addIdr(self, identifier, verkey, role=None):
        self.clients[identifier] = {VERKEY: verkey, ROLE: role}
        self._queue_key(identifier, verkey)

    def getVerkey(self, identifier):
        nym = self.clients.get(identifier)
        if not nym:
            nym = self.nym_lookup(self.state, identifier) if self.nym_lookup else {}
            if not nym:
                raise UnknownIdentifier(identifier)
        return nym.get(VERKEY)


class GpuAuthNr(SimpleAuthNr):
    """Drop-in SimpleAuthNr whose Ed25519 checks run on the MI355X."""

    def __init__(self, state=None, nym_lookup=None, engine=None, device=0, **options):
        SimpleAuthNr.__init__(self, state=state, nym_lookup=nym_lookup)
        self._gpu_init(engine=engine, device=device, **options)


CoreAuthNr = GpuAuthNr


class NoAuthenticatorFound(SigningException):
    code = 160
    reason = 'no authenticator found'


class ReqAuthenticator:
    """Aggregates client authenticators (north-star name; absent from the
    reference snapshot).  authenticate(req) returns the set of identifiers
    every registered authenticator vouches for; each sees its own deepcopy."""

    def __init__(self):
        self._authenticators = []

    def register_authenticator(self, authnr):
        self._authenticators.append(authnr)

    @property
    def core_authenticator(self):
        for a in self._authenticators:
            if isinstance(a, GpuAuthMixin):
                return a
        raise NoAuthenticatorFound

    def authenticate(self, req_data):
        identifiers = set()
        for a in self._authenticators:
            rv = a.authenticate(deepcopy(req_data))
            if rv:
                identifiers.update([rv] if isinstance(rv, str) else rv)
        if not identifiers:
            raise NoAuthenticatorFound
        return identifiers

    def prefetch(self, reqs):
        for a in self._authenticators:
            if hasattr(a, "prefetch"):
                a.prefetch(reqs)
