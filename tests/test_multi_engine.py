"""Single-process multi-GPU (MultiEngine): a batch split over N engines by
64-aligned request index gives exactly the N = 1 verdicts, for the general,
crypto_sign_open and keyed paths and through the drop-in authenticator.
Engines here are the oracle-backed doubles; tests/test_gpu_authn.py runs the
same code with N = 1 on the device (multi-GPU unmeasured until SCALE runs)."""
import numpy as np

from conftest import items_of, load_npz
from engine_double import OracleEngine
from plenum_amd.client_authn import GpuAuthNr
from plenum_amd.multi import MultiEngine, shard_bounds
import test_client_authn as T


def test_shard_bounds_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1000, 4097, 100_000):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all((lo % 64 == 0 or lo == n) and lo <= hi for lo, hi in b)
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))


def _batch():
    items = items_of(load_npz("ed25519_edge.npz")) + items_of(load_npz("ed25519_valid.npz"))[:300]
    sig = np.frombuffer(b"".join(s for s, _, _, _ in items), np.uint8).reshape(-1, 64)
    pk = np.frombuffer(b"".join(p for _, p, _, _ in items), np.uint8).reshape(-1, 32)
    msgs = [m for _, _, m, _ in items]
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return sig, pk, np.frombuffer(b"".join(msgs), np.uint8), off, np.array([e for *_, e in items])


def test_sharded_paths_equal_single(oracle):
    sig, pk, msgs, off, expect = _batch()
    one = OracleEngine(oracle)
    for n_dev in (2, 3, 5):
        me = MultiEngine(engines=[OracleEngine(oracle) for _ in range(n_dev)], min_shard=64)
        assert len(me._shards(len(sig))) == n_dev
        got = me.verify_batch(sig, pk, msgs, off)
        assert (got == one.verify_batch(sig, pk, msgs, off)).all() and (got == expect).all()
        sm = np.concatenate([np.concatenate([sig[i], msgs[int(off[i]):int(off[i + 1])]]) for i in range(len(sig))])
        sm_off = off + 64 * np.arange(len(off), dtype=np.uint64)
        assert (me.sign_open_batch(sm, sm_off, pk) == expect).all()
        uniq, inv = np.unique(pk, axis=0, return_inverse=True)
        me.keys_reset()
        assert me.keys_add(uniq) == 0 and me.keys_count() == len(uniq)
        assert (me.verify_batch_keyed(sig, inv.reshape(-1).astype(np.uint32), msgs, off) == expect).all()
        assert all(e.calls >= 1 for e in me.engines)
        me.close()


def test_authenticator_over_multi_engine(oracle):
    idrs, vks, msgs = T._signed(3, 300)
    forged = [dict(m, reqId=m["reqId"] + 7) if i % 5 == 0 else m for i, m in enumerate(msgs)]
    want = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    me = MultiEngine(engines=[OracleEngine(oracle) for _ in range(3)], min_shard=64)
    a = GpuAuthNr(engine=me)
    for idr, vk in zip(idrs, vks):
        want.addIdr(idr, vk)
        a.addIdr(idr, vk)
    exp = [r if isinstance(r, str) else type(r).__name__ for r in want.authenticate_batch(forged)]
    got = [r if isinstance(r, str) else type(r).__name__ for r in a.authenticate_batch(forged)]
    assert got == exp and a.stats["keyed_items"] == 300
    assert all(e.keys == me.engines[0].keys for e in me.engines)  # replicated store


def test_bench_devices_leg_reports_a_failing_device(oracle, monkeypatch):
    """bench.time_e2e_devices (end_to_end.by_devices): a device count whose engines cannot be
    created is reported in its entry; the counts before it are measured, the run goes on."""
    import bench
    idrs, vks, msgs = T._signed(3, 300)

    def no_device(d):
        raise RuntimeError("no HIP device %d" % d)
    monkeypatch.setattr(bench, "EdVerifyEngine", no_device)
    out = bench.time_e2e_devices(OracleEngine(oracle), [dict(m) for m in msgs], idrs, vks, [1, 2])
    assert out["1"]["accepted"] == 300 and out["1"]["engines"] == 1
    assert out["2"] == {"engines": 2, "error": "RuntimeError: no HIP device 1"}
