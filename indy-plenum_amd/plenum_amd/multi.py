"""MultiEngine: every GPU of the box behind one engine object, inside one
process.

A Plenum node is one asyncio process (stp_core/loop/looper.py:141-151), so the
drop-in authenticator cannot use the one-process-per-GPU torch.distributed
layout bench.py uses.  MultiEngine holds one EdVerifyEngine (one HIP context
and stream) per device and splits each batch by contiguous request index,
shard bounds multiples of 64 (dist.shard_bounds -- the same partition the
RCCL path uses).  The shards run concurrently: one host
thread per device, and the ctypes calls release the GIL while the device
works.  Verdicts are concatenated in request order, so the result is the
single-engine result exactly.

The key store is replicated: keys_add / keys_set register the same keys on
every device (the same ids everywhere), so a keyed shard can run on any GPU.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .engine import _u8


def shard_bounds(n, world, rank):
    """[lo, hi) request range of `rank`; lo is a multiple of 64 (dist.py)."""
    words = (n + 63) // 64
    per = (words + world - 1) // world
    return min(n, rank * per * 64), min(n, (rank + 1) * per * 64)


class MultiEngine:
    def __init__(self, devices=None, engines=None, min_shard=4096):
        """devices: device indices ("all" / None = every visible device);
        engines: ready engines (e.g. test doubles) instead.  Batches smaller
        than min_shard per device use fewer devices."""
        if engines is None:
            from . import _lib
            from .engine import EdVerifyEngine
            if devices in (None, "all"):
                devices = range(_lib.load().edv_device_count())
            engines = [EdVerifyEngine(d) for d in devices]
        if not engines:
            raise ValueError("no engines")
        self.engines = list(engines)
        self.min_shard = min_shard
        self._pool = ThreadPoolExecutor(max_workers=len(self.engines)) if len(self.engines) > 1 else None
        self.keys_generation = 0

    def __len__(self):
        return len(self.engines)

    def close(self):
        if self._pool:
            self._pool.shutdown()
        for e in self.engines:
            if hasattr(e, "close"):
                e.close()

    # ------------------------------------------------------------ sharding
    def _shards(self, n):
        world = max(1, min(len(self.engines), -(-n // self.min_shard)))
        return [shard_bounds(n, world, r) for r in range(world)]

    def _run(self, n, call):
        """call(engine, lo, hi) -> bool array for [lo, hi); results concatenated."""
        shards = [(e, lo, hi) for e, (lo, hi) in zip(self.engines, self._shards(n)) if hi > lo]
        if len(shards) <= 1 or self._pool is None:
            parts = [call(e, lo, hi) for e, lo, hi in shards]
        else:
            futs = [self._pool.submit(call, e, lo, hi) for e, lo, hi in shards]
            parts = [f.result() for f in futs]
        if not parts:
            return np.zeros(0, bool)
        return np.concatenate([np.asarray(p, bool) for p in parts])

    # -------------------------------------------------------------- verify
    @property
    def supports_sig_slots(self):
        return all(getattr(e, "supports_sig_slots", False) for e in self.engines)

    def host_alloc(self, nbytes):
        """Pinned host memory (portable: every device's copy engine reads it)."""
        return self.engines[0].host_alloc(nbytes)

    def verify_batch(self, sig64, pk32, msgs, msg_off, sig_slot=64):
        sig64, pk32, msgs = _u8(sig64, sig_slot), _u8(pk32, 32), _u8(msgs)
        off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        kw = {"sig_slot": sig_slot} if sig_slot != 64 else {}
        return self._run(sig64.shape[0], lambda e, lo, hi: e.verify_batch(sig64[lo:hi], pk32[lo:hi], msgs,
                                                                          off[lo:hi + 1], **kw))

    def sign_open_batch(self, sm, sm_off, pk32):
        sm, pk32 = _u8(sm), _u8(pk32, 32)
        off = np.ascontiguousarray(sm_off, dtype=np.uint64)
        return self._run(pk32.shape[0], lambda e, lo, hi: e.sign_open_batch(sm, off[lo:hi + 1], pk32[lo:hi]))

    def verify_batch_keyed(self, sig64, key_idx, msgs, msg_off, sig_slot=64):
        sig64, msgs = _u8(sig64, sig_slot), _u8(msgs)
        kidx = np.ascontiguousarray(key_idx, dtype=np.uint32)
        off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        kw = {"sig_slot": sig_slot} if sig_slot != 64 else {}
        return self._run(sig64.shape[0], lambda e, lo, hi: e.verify_batch_keyed(sig64[lo:hi], kidx[lo:hi], msgs,
                                                                                off[lo:hi + 1], **kw))

    def verify_submit(self, sig, keys, msgs, msg_off, keyed, sig_slot=64):
        """Each device's shard queued (edv_verify_submit); verify_collect
        concatenates the shards' verdicts in request order."""
        sig, msgs = _u8(sig, sig_slot), _u8(msgs)
        keys = np.ascontiguousarray(keys, dtype=np.uint32) if keyed else _u8(keys, 32)
        off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        shards = [(e, lo, hi) for e, (lo, hi) in zip(self.engines, self._shards(sig.shape[0])) if hi > lo]
        return [(e, e.verify_submit(sig[lo:hi], keys[lo:hi], msgs, off[lo:hi + 1], keyed, sig_slot))
                for e, lo, hi in shards]

    def verify_collect(self, handle):
        parts = [e.verify_collect(h) for e, h in handle]
        return np.concatenate(parts) if parts else np.zeros(0, bool)

    # ---------------------------------------------------- replicated key store
    def keys_reset(self):
        for e in self.engines:
            e.keys_reset()
        self.keys_generation += 1

    def keys_set_window(self, w):
        for e in self.engines:
            e.keys_set_window(w)

    def _each(self, fn):
        """fn(engine) on every device at once (a host thread per device; the
        ctypes calls release the GIL, so the table builds run concurrently)."""
        if self._pool is None:
            return [fn(e) for e in self.engines]
        futs = [self._pool.submit(fn, e) for e in self.engines]
        return [f.result() for f in futs]

    def keys_add(self, pk32):
        pk32 = _u8(pk32, 32)
        firsts = set(self._each(lambda e: e.keys_add(pk32)))
        if len(firsts) != 1:
            raise RuntimeError("key stores of the devices diverged (first ids %s)" % sorted(firsts))
        return firsts.pop()

    def keys_set(self, first_id, pk32):
        pk32 = _u8(pk32, 32)
        self._each(lambda e: e.keys_set(first_id, pk32))

    @property
    def supports_async_keys(self):
        return all(hasattr(e, "keys_add_async") for e in self.engines)

    def keys_add_async(self, pk32):
        """Queued on every device at once; the ticket is the tuple of the
        devices' tickets (ready when every device's build is)."""
        pk32 = _u8(pk32, 32)
        res = self._each(lambda e: e.keys_add_async(pk32))
        firsts = {f for f, _ in res}
        if len(firsts) != 1:
            raise RuntimeError("key stores of the devices diverged (first ids %s)" % sorted(firsts))
        return firsts.pop(), tuple(t for _, t in res)

    def keys_set_many_async(self, ids, pk32):
        pk32 = _u8(pk32, 32)
        return tuple(self._each(lambda e: e.keys_set_many_async(ids, pk32)))

    def keys_set_async(self, first_id, pk32):
        pk32 = _u8(pk32, 32)
        return tuple(self._each(lambda e: e.keys_set_async(first_id, pk32)))

    def keys_ready(self, ticket):
        return all(e.keys_ready(t) for e, t in zip(self.engines, ticket))

    def keys_sync(self):
        self._each(lambda e: e.keys_sync())

    def keys_count(self):
        return self.engines[0].keys_count()

    # ----------------------------------------------------- one-device helpers
    def tally(self, *a, **k):
        return self.engines[0].tally(*a, **k)

    def seed_keypair_batch(self, seeds32):
        return self.engines[0].seed_keypair_batch(seeds32)

    def sign_batch(self, sk64, key_idx, msgs, msg_off):
        return self.engines[0].sign_batch(sk64, key_idx, msgs, msg_off)
