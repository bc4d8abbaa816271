"""The N > 1 path on CPU: world_size-2 gloo process group, request-index
shards with 64-aligned bounds, bitmask all-gather and ballot all-reduce(MAX)
must reproduce the single-process result exactly (oracle verdicts)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, items_of, load_npz


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _words(bits):
    b = np.packbits(np.asarray(bits, dtype=np.uint8), bitorder="little")
    b = np.concatenate([b, np.zeros((-len(b)) % 8, np.uint8)])
    return torch.from_numpy(b.view(np.int64).copy())


def _worker(rank, world, port, q):
    import ctypes
    import sys
    sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from plenum_amd.dist import gather_bitmask, shard_bounds, union_ballots
    from tally_oracle import ballots_from_votes
    import tally_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libed25519_oracle.so"))
    items = items_of(load_npz("ed25519_edge.npz")) * 2  # 432 items: ragged last word
    n = len(items)
    lo, hi = shard_bounds(n, world, rank)
    local = [lib.oracle_verify_detached(s, m, ctypes.c_uint64(len(m)), p) == 0 for s, p, m, _ in items[lo:hi]]
    full = gather_bitmask(_words(local), n)
    bits = np.unpackbits(full.numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    rng = np.random.default_rng(42)
    nk, nv, nvotes = 40, 25, 3000
    k, v, ph = rng.integers(0, nk, nvotes), rng.integers(0, nv, nvotes), rng.integers(0, 2, nvotes)
    ok = rng.random(nvotes) < 0.95
    sl = slice(rank * nvotes // world, (rank + 1) * nvotes // world)
    ballot = torch.from_numpy(ballots_from_votes(k[sl], v[sl], ph[sl], ok[sl], nk, nv))
    union_ballots(ballot)
    counts, _, _ = tally_oracle.tally(k, v, ph, ok, nk, nv)
    q.put((rank, bits.tolist(), bool((ballot.numpy().sum(axis=2) == counts).all()), (lo, hi)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_process(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    items = items_of(load_npz("ed25519_edge.npz")) * 2
    want = [e for *_, e in items]
    bounds = sorted(r[3] for r in res)
    assert bounds[0][0] == 0 and bounds[-1][1] == len(items) and bounds[0][1] == bounds[1][0]
    assert bounds[0][1] % 64 == 0
    for rank, bits, ballots_ok, _ in res:
        assert bits == want
        assert ballots_ok


def test_shard_bounds_cover_and_align():
    from plenum_amd.dist import shard_bounds
    for n in (0, 1, 63, 64, 65, 1000, 16_000_000, 16_000_001):
        for world in (1, 2, 3, 4, 8):
            b = [shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            for (l0, h0), (l1, h1) in zip(b, b[1:]):
                assert h0 == l1
            assert all(lo % 64 == 0 or lo == hi == n for lo, hi in b)
