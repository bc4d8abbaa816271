"""The registered-key store of one engine, shared by every authenticator that
uses the engine.

The key-table path (edv_keys_add / edv_verify_batch_keyed) verifies a request
against a key id; the id -> key binding lives in the engine's HBM.  One
KeyStore object per engine owns that binding, so two authenticators sharing an
engine (e.g. under ReqAuthenticator) can never see each other's ids point at
different keys.  The engine's keys_generation (bumped by every keys_reset)
is checked on each use: a reset by anyone else empties the map instead of
leaving stale ids.

Capacity is bounded (max_keys tables at the chosen comb window); once full,
least-recently-used keys are evicted in place (edv_keys_set rebuilds a slot),
never a key the current batch is using.  Recency is a per-slot tick (the
lookup call that last returned the slot's id; registration counts as a use),
so a batch's lookups mark its keys with one vectorized store and an eviction
picks the slots with the oldest ticks (ties: lowest slot).  Which keys get in is the caller's
policy (client_authn.GpuAuthMixin): keys given to addIdr while there is free
room, and keys that verified successfully hot_key_uses times.  A key whose
registration fails (allocation, HIP error) is remembered as unregistrable and
its requests keep taking the general path, which gives the same verdicts.

Registrations made on the request path are asynchronous when the engine has
edv_keys_add_async (register(..., asynchronous=True)): the ids are assigned at
once, the tables build on the engine's build stream while batches go on, and
lookup() answers None for an id whose build ticket has not completed, so its
requests take the general path until then (same verdicts, no stall).
"""
from collections import OrderedDict

import numpy as np

try:  # the native mirror of the key -> id map (csrc/hostpack.cpp KeyIndex)
    from ._hostpack import key_index as _key_index, key_index_set as _ki_set, key_index_del as _ki_del, \
        key_index_clear as _ki_clear, key_index_get as _ki_get
except ImportError:  # pragma: no cover
    _key_index = None
try:  # the promotion policy's use counts for 32-byte keys (csrc/hostpack.cpp UseTable)
    from ._hostpack import use_table as _use_table, use_table_add as _ut_add, use_table_pop as _ut_pop, \
        use_table_has as _ut_has, use_table_len as _ut_len
except ImportError:  # pragma: no cover
    _use_table = None

# comb windows the library builds (edverify.h edv_keys_set_window)
WINDOWS = (4, 6, 8, 10, 12, 13, 14, 16)


def key_rows(w):
    return (254 + w - 1) // w


def key_table_bytes(w):
    """HBM per registered key at window w: rows x 2^(w-1) entries x 128 B."""
    return key_rows(w) * (1 << (w - 1)) * 128


def auto_window(max_keys, budget_bytes):
    """Widest window whose max_keys tables fit in budget_bytes (>= 4)."""
    best = WINDOWS[0]
    for w in WINDOWS:
        if key_table_bytes(w) * max_keys <= budget_bytes:
            best = w
    return best


class KeyStore:
    def __init__(self, engine, window, capacity):
        self.engine = engine
        self.window = window
        self.capacity = capacity
        self._ids = {}                # key bytes -> id
        # the same map for 32-byte keys, natively (lookup_array over a batch's flat key buffer)
        self._index = _key_index() if _key_index is not None else None
        self._slot_key = []           # id -> key bytes (None: a retired slot)
        self._retired = np.zeros(max(int(capacity), 1), bool)  # id -> retired (the eviction candidates' mask)
        self._used = np.zeros(max(int(capacity), 1), np.int64)  # id -> tick of its last use
        self._tick = 1
        self._failed = OrderedDict()  # keys that could not be registered
        self._generation = None
        self._building = {}           # id -> ticket of its latest build (asynchronous registrations)
        self._tickets = OrderedDict()  # ticket -> ids, ascending (tickets complete in order)
        # bumped whenever an id may stop meaning the key it meant (a reset, an eviction, a retired
        # slot): what a speculative batch (key ids from earlier batches) checks it ran against
        self.version = 0

    @classmethod
    def attach(cls, engine, window, capacity):
        """The engine's store (created by the first caller, whose window and
        capacity it keeps); None if the engine has no key-table path."""
        if not hasattr(engine, "keys_add"):
            return None
        ks = getattr(engine, "_edv_key_store", None)
        if ks is None:
            ks = cls(engine, window, capacity)
            engine._edv_key_store = ks
        return ks

    def _sync(self):
        gen = getattr(self.engine, "keys_generation", 0)
        if self._generation == gen:
            return
        # first use, or someone reset the engine's store: start from empty
        self.engine.keys_reset()
        if hasattr(self.engine, "keys_set_window"):
            self.engine.keys_set_window(self.window)
        self._ids.clear()
        if self._index is not None:
            _ki_clear(self._index)
        self._slot_key = []
        self._retired[:] = False
        self._used[:] = 0
        self._building.clear()
        self._tickets.clear()
        self._generation = getattr(self.engine, "keys_generation", 0)
        self.version += 1

    def _id_set(self, key, i):
        self._ids[key] = i
        if self._index is not None and len(key) == 32:
            _ki_set(self._index, key, int(i).to_bytes(8, "little", signed=True))

    def _id_pop(self, key):
        i = self._ids.pop(key)
        if self._index is not None and len(key) == 32:
            _ki_del(self._index, key)
        return i

    def _refresh(self):
        """Drop the ids whose builds have completed from the building set
        (one edv_keys_ready query per completed ticket, oldest first)."""
        while self._tickets:
            t = next(iter(self._tickets))
            if not self.engine.keys_ready(t):
                return
            for i in self._tickets.pop(t):
                if self._building.get(i) == t:
                    del self._building[i]

    def building(self):
        """Ids whose tables are still being built."""
        self._refresh()
        return len(self._building)

    def settle(self):
        """Wait for every queued build (e.g. before a timed run)."""
        if self._tickets and hasattr(self.engine, "keys_sync"):
            self.engine.keys_sync()
        self._building.clear()
        self._tickets.clear()

    def _mark_building(self, ids, ticket):
        for i in ids:
            self._building[i] = ticket
        self._tickets.setdefault(ticket, []).extend(ids)

    def __len__(self):
        return len(self._ids)

    def __contains__(self, key):
        return key in self._ids and self._generation == getattr(self.engine, "keys_generation", 0)

    def free_slots(self):
        self._sync()
        return self.capacity - len(self._ids)

    def lookup(self, keys):
        """Ids of keys (None for unregistered keys and for keys whose tables
        are still building), marking them recently used."""
        self._sync()
        if self._building:
            self._refresh()
        building = self._building
        get = self._ids.get
        out = [get(k) for k in keys]
        hit = [i for i in out if i is not None]
        if hit:
            self._used[hit] = self._tick  # (one tick per call: its keys are equally recent)
            self._tick += 1
        if building:
            out = [None if i is not None and i in building else i for i in out]
        return out

    def lookup_one(self, key):
        """lookup([key])[0] without the list and array operations: the id of
        one key (None if unregistered or still building), marked recently used
        (the per-message authenticate() path)."""
        self._sync()
        if self._building:
            self._refresh()
        i = self._ids.get(key)
        if i is None:
            return None
        self._used[i] = self._tick
        self._tick += 1
        return None if i in self._building else i

    def lookup_array(self, keys, flat=None, odd=(), ids=None):
        """lookup() as an int64 array, -1 where lookup() answers None (one
        pass over the keys; the hits' ticks and the building filter vectorized).
        flat: the same keys as one buffer of 32 bytes each (keys_known_flat),
        looked up in the native index in one call; odd: the positions of keys
        that are not 32 bytes (zeros in flat), looked up in the dict; ids: the
        same keys' ids_of() answer when nothing was registered since.""" 
        self._sync()
        if self._building:
            self._refresh()
        if ids is not None and len(ids) == len(keys):  # (ids_of's answer, no registration since)
            ids = np.array(ids, np.int64)
        elif flat is not None and self._index is not None and len(flat) == 32 * len(keys):
            ids = np.frombuffer(_ki_get(self._index, flat), np.int64).copy()
            for j in odd:  # (keys that are not 32 bytes: zeros in flat)
                ids[j] = self._ids.get(keys[j], -1) if keys[j].__class__ is bytes else -1
        else:
            get = self._ids.get
            ids = np.fromiter((get(k, -1) for k in keys), np.int64, len(keys))
        hit = ids[ids >= 0]
        if len(hit):
            self._used[hit] = self._tick
            self._tick += 1
        if self._building:  # (a mask over the slots: np.isin sorted the batch's ~30k ids)
            building = np.zeros(max(len(self._slot_key), self.capacity, 1), bool)
            building[np.fromiter(self._building, np.int64, len(self._building))] = True
            live = ids >= 0
            ids[live & building[np.where(live, ids, 0)]] = -1
        return ids

    def _touch(self, ids):
        if len(ids):
            self._used[np.asarray(ids, np.int64)] = self._tick
            self._tick += 1

    def ids_of(self, flat, odd=(), keys=None):
        """The ids of 32-byte keys given as one buffer (-1: not registered), from the native index,
        without marking them used; odd: positions of keys not 32 bytes (looked up in `keys`)."""
        self._sync()
        if self._index is not None:
            ids = np.frombuffer(_ki_get(self._index, flat), np.int64).copy()
        else:
            get = self._ids.get
            ids = np.fromiter((get(bytes(flat[32 * j:32 * j + 32]), -1) for j in range(len(flat) // 32)), np.int64)
        for j in odd:
            ids[j] = self._ids.get(keys[j], -1) if keys is not None and keys[j].__class__ is bytes else -1
        return ids

    def _victims(self, count, pinned, pinned_ids=None):
        """Up to count least-recently-used keys outside `pinned` (or the ids pinned_ids) (oldest
        tick first, then lowest slot)."""
        n = len(self._slot_key)
        if count <= 0 or n == 0:
            return []
        live = ~self._retired[:n]
        if pinned_ids is None:
            get = self._ids.get
            pinned_ids = np.fromiter((get(k, -1) for k in pinned), np.int64)
        pid = np.asarray(pinned_ids, np.int64)
        live[pid[(pid >= 0) & (pid < n)]] = False
        cand = np.flatnonzero(live)
        if len(cand) > count:
            used = self._used[cand]
            sel = np.argpartition(used, count - 1)[:count]
            cand = cand[sel]
        cand = cand[np.lexsort((cand, self._used[cand]))]
        return [self._slot_key[i] for i in cand[:count]]

    def register(self, keys, pinned=(), evict=True, asynchronous=False, pinned_ids=None):
        """Register keys not yet in the store: into free slots, then (evict)
        over least-recently-used keys outside `pinned`.  Returns the keys
        registered.  asynchronous: queue the table builds and return at once
        (engines with keys_add_async; lookup() hides the ids until built)."""
        self._sync()
        use_async = asynchronous and getattr(self.engine, "supports_async_keys",
                                             hasattr(self.engine, "keys_add_async"))
        fresh = [k for k in OrderedDict.fromkeys(keys) if k not in self._ids and k not in self._failed]
        if not fresh:
            return []
        room = max(self.capacity - len(self._ids), 0)
        new, over = fresh[:room], fresh[room:]
        done = []
        if new:
            pk = np.frombuffer(b"".join(new), np.uint8).reshape(-1, 32)
            ticket = None
            try:
                if use_async:
                    first, ticket = self.engine.keys_add_async(pk)
                else:
                    first = self.engine.keys_add(pk)
            except Exception:
                self._fail(new)
                new = []
            for j, k in enumerate(new):
                self._id_set(k, first + j)
                self._slot_key.append(k)
            if new:
                self._touch(range(first, first + len(new)))
            if ticket is not None and new:
                self._mark_building(range(first, first + len(new)), ticket)
            done += new
        if over and evict and hasattr(self.engine, "keys_set"):
            victims = self._victims(len(over), pinned, pinned_ids)
            if use_async and hasattr(self.engine, "keys_set_many_async") and victims:
                # every eviction of this call in one upload and one build launch
                pairs = list(zip(over, victims))
                slots = [self._id_pop(k_old) for _, k_old in pairs]
                self.version += 1
                pk = np.frombuffer(b"".join(k for k, _ in pairs), np.uint8).reshape(-1, 32)
                try:
                    ticket = self.engine.keys_set_many_async(np.asarray(slots, np.uint32), pk)
                except Exception:
                    for sl in slots:  # the slots' old tables may be half rewritten: retire them
                        self._slot_key[sl] = None
                        self._retired[sl] = True
                    self._fail([k for k, _ in pairs])
                    return done
                self._mark_building(slots, ticket)
                for (k_new, _), sl in zip(pairs, slots):
                    self._slot_key[sl] = k_new
                    self._id_set(k_new, sl)
                    done.append(k_new)
                self._touch(slots)
                return done
            for k_new, k_old in zip(over, victims):
                slot = self._id_pop(k_old)
                self.version += 1
                try:
                    pk = np.frombuffer(k_new, np.uint8).reshape(1, 32)
                    if use_async and hasattr(self.engine, "keys_set_async"):
                        self._mark_building([slot], self.engine.keys_set_async(slot, pk))
                    else:
                        self.engine.keys_set(slot, pk)
                except Exception:
                    # the slot's old table may be half rewritten: retire the slot
                    self._slot_key[slot] = None
                    self._retired[slot] = True
                    self._fail([k_new])
                    continue
                self._slot_key[slot] = k_new
                self._id_set(k_new, slot)
                self._touch([slot])
                done.append(k_new)
        return done

    def _fail(self, keys):
        for k in keys:
            self._failed[k] = None
        while len(self._failed) > 65536:
            self._failed.popitem(last=False)


class UseCounts:
    """Decayed verified-use counts of general-path keys, the state of the
    promotion policy (client_authn.GpuAuthMixin._count_verified_keys): a
    key's count halves per epoch since it was last counted; add() reports the
    keys whose count reached hot_at (and drops them: they earned a slot);
    bounded at cap keys, past which the least recently counted are dropped
    (down to 7/8 of cap).  32-byte keys -- every key a verify can count --
    live in the native table (csrc/hostpack.cpp UseTable: a batch's ~4k keys
    counted in one pass over its flat key buffer, add_flat), any other key
    in the array form (_ArrayUseCounts, the same policy).  pop / len / in
    behave as on a dict of (count, epoch)."""

    def __init__(self, cap):
        import threading
        self.cap = cap
        self._nat = _use_table(cap) if _use_table is not None else None
        self._py = _ArrayUseCounts(cap)
        self._lock = threading.Lock()

    @property
    def native(self):
        return self._nat is not None

    def _is_nat(self, key):
        return self._nat is not None and key.__class__ is bytes and len(key) == 32

    def __len__(self):
        return (_ut_len(self._nat) if self._nat is not None else 0) + len(self._py)

    def __contains__(self, key):
        if self._is_nat(key):
            return _ut_has(self._nat, key)
        return key in self._py

    def pop(self, key, default=None):
        if self._is_nat(key):
            with self._lock:
                r = _ut_pop(self._nat, key)
            return default if r is None else r
        return self._py.pop(key, default)

    def add_flat(self, flat, counts, now, hot_at, floor=1):
        """add() over 32-byte keys given as one buffer (flat[32 j:32 j + 32]
        = key j), counts[j] below floor not counted: the positions j of the
        keys that reached hot_at, in input order (int64 array)."""
        c = np.ascontiguousarray(counts, np.int64)
        with self._lock:
            return np.frombuffer(_ut_add(self._nat, flat, c, int(floor), int(now), int(hot_at)), np.int64)

    def add(self, keys, counts, now, hot_at):
        """Counts counts[j] verified requests of keys[j] at epoch now.  Returns,
        in input order, the keys whose count reached hot_at; their counts are
        dropped (they earned a slot; a later count starts from zero).  A key may
        appear more than once (two identifiers sharing a verkey): its counts
        are summed."""
        if self._nat is None:
            return self._py.add(keys, counts, now, hot_at)
        keys = list(keys)
        counts = np.asarray(counts, np.int64).reshape(-1)
        nat = [j for j, k in enumerate(keys) if self._is_nat(k)]
        if len(nat) == len(keys):
            return [keys[j] for j in self.add_flat(b"".join(keys), counts, now, hot_at).tolist()]
        # the other keys first: an unhashable one raises before anything of this call is counted
        oth = [j for j, k in enumerate(keys) if not self._is_nat(k)]
        hot_o = self._py.add([keys[j] for j in oth], counts[oth], now, hot_at)
        first = {}
        for j in oth:
            first.setdefault(keys[j], j)
        out = [(first[k], k) for k in hot_o]
        if nat:
            pos = self.add_flat(b"".join(keys[j] for j in nat), counts[nat], now, hot_at).tolist()
            out += [(nat[p], keys[nat[p]]) for p in pos]
        return [k for _, k in sorted(out, key=lambda x: x[0])]


class _ArrayUseCounts:
    """UseCounts' policy for keys the native table does not take (and its
    whole form without the native module): key ->
    a row of three arrays (count, the epoch it was last counted at, the call
    that last counted it).  Rows are dense (0 .. len-1; a released row is
    filled from the end), so add() maps a batch's keys to rows with one
    dict.setdefault per key and does the rest -- decay (a count halves per
    epoch since it was last counted), summing, promotion -- as array
    operations.  Bounded at cap keys: past it, the least recently counted are
    dropped (down to 7/8 of cap, so a churning batch stream trims every few
    batches, not every batch).  pop / len / in behave as on a dict of
    (count, epoch)."""

    def __init__(self, cap):
        import threading
        self.cap = cap
        self._row = {}                        # key -> row
        self._keys = np.empty(1024, object)   # row -> key
        self._u = np.zeros(1024, np.int64)
        self._e = np.zeros(1024, np.int64)
        self._t = np.zeros(1024, np.int64)    # the add() call that last counted the row
        self._tick = 0
        self._lock = threading.Lock()         # add() is several steps, not one dict op

    def __len__(self):
        return len(self._row)

    def __contains__(self, key):
        return key in self._row

    def pop(self, key, default=None):
        with self._lock:
            r = self._row.pop(key, None)
            if r is None:
                return default
            out = (int(self._u[r]), int(self._e[r]))
            self._compact(np.array([r]), len(self._row) + 1)
            return out

    def _compact(self, gone, n):
        """Rows `gone` (sorted, already out of the dict) of the n in use are
        freed: the rows past the new end that stay move into the holes."""
        m = n - len(gone)
        keep = np.ones(n - m, bool)
        keep[gone[gone >= m] - m] = False
        movers = m + np.flatnonzero(keep)
        holes = gone[gone < m]
        if len(holes):
            for a in (self._keys, self._u, self._e, self._t):
                a[holes] = a[movers]
            self._row.update(zip(self._keys[holes].tolist(), holes.tolist()))
        self._keys[m:n] = None

    def add(self, keys, counts, now, hot_at):
        """Counts counts[j] verified requests of keys[j] at epoch now.  Returns,
        in input order, the keys whose count reached hot_at; their rows are
        dropped (they earned a slot; a later count starts from zero).  A key may
        appear more than once (two identifiers sharing a verkey): its counts
        are summed."""
        c = np.asarray(counts, np.int64).reshape(-1)
        if not c.all():
            j = np.flatnonzero(c)
            keys, c = [keys[i] for i in j.tolist()], c[j]
        if not len(c):
            return []
        with self._lock:
            row = self._row
            n0 = len(row)
            if n0 + len(c) > len(self._u):
                grow = max(n0 + len(c), 2 * len(self._u)) - len(self._u)
                self._keys = np.concatenate([self._keys, np.empty(grow, object)])
                self._u = np.concatenate([self._u, np.zeros(grow, np.int64)])
                self._e = np.concatenate([self._e, np.zeros(grow, np.int64)])
                self._t = np.concatenate([self._t, np.zeros(grow, np.int64)])
            sd, ln = row.setdefault, row.__len__
            try:
                R = np.fromiter([sd(k, ln()) for k in keys], np.int64, len(c))
            except BaseException:  # (an unhashable key): drop the rows this call began
                for k in [k for k, r in row.items() if r >= n0]:
                    del row[k]
                raise
            n = len(row)
            if n > n0:  # new keys: rows n0 .. n-1, first occurrences in input order
                new = np.flatnonzero(R >= n0)
                if len(new) != n - n0:
                    _, fi = np.unique(R[new], return_index=True)
                    new = new[fi]
                karr = np.empty(len(c), object)
                karr[:] = keys
                self._keys[R[new]] = karr[new]
                self._u[n0:n] = 0
                self._e[n0:n] = now
            cu = np.bincount(R, weights=c, minlength=n).astype(np.int64)
            ur = np.flatnonzero(cu)
            shift = np.clip(now - self._e[ur], 0, 62)
            u = (self._u[ur] >> shift) + cu[ur]
            self._u[ur] = u
            self._e[ur] = now
            self._t[ur] = self._tick
            self._tick += 1
            hot = u >= hot_at
            out = []
            if hot.any():
                hot_rows = ur[hot]
                is_hot = np.zeros(n, bool)
                is_hot[hot_rows] = True
                pos = np.flatnonzero(is_hot[R])
                if len(pos) != len(hot_rows):
                    _, fi = np.unique(R[pos], return_index=True)
                    pos = np.sort(pos[fi])
                out = self._keys[R[pos]].tolist()
                for k in out:
                    del row[k]
                self._compact(hot_rows, n)
                n -= len(hot_rows)
            if n > self.cap:
                drop = n - self.cap + self.cap // 8
                # (ties: the lower row first -- the native table drops the same rows)
                v = np.sort(np.argsort(self._t[:n], kind="stable")[:drop]) if drop < n else np.arange(n)
                for k in self._keys[v].tolist():
                    del row[k]
                self._compact(v, n)
            return out
