"""The drop-in authenticator on the real GPU engine: the reference KAT table
(tests/golden/authn_kat.json from the reference's own NaclAuthNr) and batch
== single, with no CPU verification anywhere on the path."""
import pytest

import test_client_authn as T
from plenum_amd.client_authn import GpuAuthNr

pytestmark = pytest.mark.gpu


def test_reference_kats_on_gpu(gpu_engine):
    for c in T.kat()["cases"]:
        T.check_result(c, T.run_single(T.make(gpu_engine, c), c))


def test_batch_on_gpu(gpu_engine):
    good = next(c for c in T.kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    a = T.make(gpu_engine, good)
    msgs = [dict(good["msg"]) for _ in range(1000)]
    for i in range(0, 1000, 3):
        msgs[i]["reqId"] += 1
    res = a.authenticate_batch(msgs)
    for i, r in enumerate(res):
        if i % 3 == 0:
            assert type(r).__name__ == "InvalidSignature"
        else:
            assert r == good["msg"]["identifier"]
    assert a.stats["batches"] == 1


def test_multi_on_gpu(gpu_engine):
    a, msg, sigs = T._multi_fixture(gpu_engine)
    assert a.authenticate_multi(msg, sigs) == list(sigs)


def test_default_engine_is_gpu():
    from plenum_amd.engine import EdVerifyEngine
    a = GpuAuthNr()
    assert isinstance(a._engine(), EdVerifyEngine)


def test_keyed_and_general_paths_agree_on_gpu(gpu_engine):
    with_keys, n_keyed = T._outcomes(gpu_engine, 16)
    without, n_general = T._outcomes(gpu_engine, 0)
    assert with_keys == without
    assert n_keyed > 0 and n_general == 0
    for c, r in zip(T.kat()["cases"], with_keys):
        if "result" in c:
            assert r == c["result"], c["name"]
        else:
            assert r[0] == c["raises"], c["name"]
