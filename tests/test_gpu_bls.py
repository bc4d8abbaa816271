"""BLS multi-signatures on the GPU (csrc/bls.hip over bn254.h) against the
oracle's committed vectors (tests/golden/bls_vectors.json), and the drop-in
classes (plenum_amd/bls.py) on the reference's own test scenarios
(crypto/test/bls/indy_crypto/test_bls_crypto_indy_crypto.py)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
V = json.load(open(os.path.join(GOLDEN, "bls_vectors.json")))


@pytest.fixture(params=["wave", "quad", "pair", "one"])
def bls_mode(request, gpu_engine):
    """Every verify form: one wave per check (the straight-line program), four lanes per check
    (batches up to half the pair limit), two, one.  Returns set(n): selects that form for an
    n-check batch."""
    def set_for(n):
        gpu_engine.bls_set_wave_checks(n if request.param == "wave" else 0)
        gpu_engine.bls_set_pair_lanes({"wave": 0, "quad": 2 * n, "pair": n, "one": 0}[request.param])
    yield set_for
    gpu_engine.bls_set_wave_checks(8192)
    gpu_engine.bls_set_pair_lanes(32768)


def _u8(hexes):
    return np.frombuffer(b"".join(bytes.fromhex(h) for h in hexes), np.uint8).reshape(-1, 128)


def test_bls_vectors_on_gpu(gpu_engine, bls_mode):
    from plenum_amd import pack_messages
    gen = np.frombuffer(bytes.fromhex(V["generator"]), np.uint8)
    msgs = [bytes.fromhex(m) for m in V["messages"]]
    # keys and signatures
    sks = np.frombuffer(b"".join(bytes.fromhex(k["sk"]) for k in V["keys"]), np.uint8).reshape(-1, 32)
    assert (gpu_engine.bls_keygen_batch(sks, gen) == _u8([k["vk"] for k in V["keys"]])).all()
    sig_items = V["signatures"]
    buf, off = pack_messages([msgs[s["msg"]] for s in sig_items])
    sk_rows = sks[[s["key"] for s in sig_items]]
    got = gpu_engine.bls_sign_batch(sk_rows, buf, off)
    assert (got == _u8([s["sig"] for s in sig_items])).all()
    # every verdict, single and multi in one launch
    cases = V["cases"]
    bls_mode(len(cases))
    buf, off = pack_messages([msgs[c["msg"]] for c in cases])
    vks, vk_off = [], [0]
    for c in cases:
        vks += c["vks"]
        vk_off.append(len(vks))
    ok = gpu_engine.bls_verify_batch(_u8([c["sig"] for c in cases]), buf, off, _u8(vks), gen,
                                     vk_off=np.asarray(vk_off, np.uint64))
    want = np.array([c["expect"] for c in cases])
    assert (ok == want).all(), [c["name"] for c, g, w in zip(cases, ok, want) if g != w]
    # create_multi_sig
    ag = V["aggregates"]
    sig_off = np.cumsum([0] + [len(a["sigs"]) for a in ag]).astype(np.uint64)
    out = gpu_engine.bls_aggregate(_u8([s for a in ag for s in a["sigs"]]), sig_off)
    assert (out == _u8([a["out"] for a in ag])).all()


def test_bls_random_batch_self_consistent(gpu_engine, bls_mode):
    """A larger batch: GPU keys and signatures verify, corrupted ones do not,
    across wave boundaries (n = 200: 4 waves of 64 checks, 7 of 32 pairs, or 13 of 16 quads)."""
    from plenum_amd import pack_messages
    rng = np.random.default_rng(5)
    gen = np.frombuffer(bytes.fromhex(V["generator"]), np.uint8)
    n = 200
    r = 36 * (-0x4080000000000001) ** 4 + 36 * (-0x4080000000000001) ** 3 + 18 * (-0x4080000000000001) ** 2 \
        + 6 * (-0x4080000000000001) + 1
    sks = np.frombuffer(b"".join((int.from_bytes(rng.bytes(32), "big") % r).to_bytes(32, "big")
                                 for _ in range(n)), np.uint8).reshape(n, 32)
    vks = gpu_engine.bls_keygen_batch(sks, gen)
    msgs = [rng.bytes(int(rng.integers(0, 300))) for _ in range(n)]
    buf, off = pack_messages(msgs)
    sigs = gpu_engine.bls_sign_batch(sks, buf, off)
    sigs[::7, 50] ^= 1  # off the curve
    vks[3::11] = vks[(np.arange(3, n, 11) + 1) % n]  # someone else's key
    bls_mode(n)
    ok = gpu_engine.bls_verify_batch(sigs, buf, off, vks, gen)
    want = np.ones(n, bool)
    want[::7] = False
    want[3::11] = False
    assert (ok == want).all(), np.nonzero(ok != want)


def test_dropin_reference_scenarios(gpu_engine):
    """The reference's test_bls_crypto_indy_crypto.py scenarios through the
    drop-in classes: sign / verify, long message, multi-signature, invalid and
    short / long base58 values."""
    from plenum_amd.bls import BlsCryptoSignerGpu, BlsCryptoVerifierGpu, BlsGroupParamsLoaderGpu, GpuBlsUtils
    from plenum_amd.base58 import b58encode
    params = BlsGroupParamsLoaderGpu().load_group_params()
    sk1, pk1 = BlsCryptoSignerGpu.generate_keys(params, "Node1", engine=gpu_engine)
    sk2, pk2 = BlsCryptoSignerGpu.generate_keys(params, "Node2", engine=gpu_engine)
    assert (sk1, pk1) != (sk2, pk2)
    assert BlsCryptoSignerGpu.generate_keys(params, "Node1", engine=gpu_engine) == (sk1, pk1)
    s1 = BlsCryptoSignerGpu(sk1, pk1, params, engine=gpu_engine)
    s2 = BlsCryptoSignerGpu(sk2, pk2, params, engine=gpu_engine)
    ver = BlsCryptoVerifierGpu(params, engine=gpu_engine)
    msg = b"Hello!"
    sig1, sig2 = s1.sign(msg), s2.sign(msg)
    assert ver.verify_sig(sig1, msg, pk1) and ver.verify_sig(sig2, msg, pk2)
    assert not ver.verify_sig(sig1, msg, pk2) and not ver.verify_sig(sig2, msg, pk1)
    long_msg = b"1" * 1000000
    assert ver.verify_sig(s1.sign(long_msg), long_msg, pk1)
    multi = ver.create_multi_sig([sig1, sig2])
    assert ver.verify_multi_sig(multi, msg, [pk1, pk2])
    assert not ver.verify_multi_sig(multi, msg, [pk1])
    assert not ver.verify_multi_sig(multi, b"Hello!!", [pk1, pk2])
    assert not ver.verify_multi_sig(ver.create_multi_sig([sig1]), msg, [pk1, pk2])
    # invalid / short / long values (reference :186-275): False, no exception
    for bad in (sig1 + b58encode(b"0"), sig1 + b58encode(b"somefake"), b58encode(b"1" * 10),
                b58encode(b"1" * 2), b58encode(b"1" * 500), "0OIl"):
        assert not ver.verify_sig(bad, msg, pk1)
        assert not ver.verify_multi_sig(bad, msg, [pk1, pk2])
        assert not ver.verify_sig(sig1, msg, bad)
        assert not ver.verify_multi_sig(multi, msg, [pk1, bad])
    # the batch form equals the one-by-one answers
    items = [(sig1, msg, pk1), (sig2, msg, pk1), (sig2, msg, pk2), (sig1 + "x", msg, pk1)]
    assert ver.verify_sig_batch(items) == [True, False, True, False]
    assert ver.verify_multi_sig_batch([(multi, msg, [pk1, pk2]), (multi, msg, [pk2])]) == [True, False]
    assert GpuBlsUtils.bls_from_str(multi) is not None


REDO_MSG = b"wave-form redo 11075"  # H(m) needs more than 16 candidates (tests/test_bls_program.py)


@pytest.mark.parametrize("tries", ["16", "61"])
def test_wave_form_hands_over_what_it_cannot_decide(gpu_engine, monkeypatch, tries):
    """The wave form tries H(m)'s candidates side by side (61 by default; EDV_BLS_HASH_TRIES=16
    here to force the hand-over): for REDO_MSG the first point is candidate 17 or later, so with
    16 tries those checks -- and only they, compacted -- go to the four-lane kernel (verdict 2 ->
    redo); with 61 the wave form decides them.  Either way, in a batch with ordinary checks,
    every verdict is the four-lane form's."""
    monkeypatch.setenv("EDV_BLS_HASH_TRIES", tries)
    from plenum_amd import pack_messages
    gen = np.frombuffer(bytes.fromhex(V["generator"]), np.uint8)
    sks = np.frombuffer(b"".join(bytes.fromhex(k["sk"]) for k in V["keys"][:2]), np.uint8).reshape(-1, 32)
    vks = gpu_engine.bls_keygen_batch(sks, gen)
    msgs = [REDO_MSG, b"ordinary", REDO_MSG, REDO_MSG + b"!"]
    buf, off = pack_messages(msgs)
    rows = sks[[0, 1, 1, 0]]
    sigs = gpu_engine.bls_sign_batch(rows, buf, off)
    sigs[3] = sigs[0]  # REDO_MSG's signature on another message
    vk_rows = vks[[0, 1, 0, 0]]  # check 2: signed by key 1, checked against key 0
    want = np.array([True, True, False, False])
    try:
        for wave in (16, 0):
            gpu_engine.bls_set_wave_checks(wave)
            gpu_engine.bls_set_pair_lanes(32768)
            assert (gpu_engine.bls_verify_batch(sigs, buf, off, vk_rows, gen) == want).all(), wave
    finally:
        gpu_engine.bls_set_wave_checks(8192)
