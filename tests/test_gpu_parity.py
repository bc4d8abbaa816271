"""Parity of the HIP path (libplenum_edverify.so on the MI355X) with libsodium
1.0.18 (golden vectors) and with the oracle (fresh random/adversarial
batches).  Bit-exact: every accept bit must equal libsodium's verdict."""
import hashlib

import numpy as np
import pytest

from conftest import items_of, load_npz
from plenum_amd import pack_messages
from plenum_amd.engine import lengths_mixed

pytestmark = pytest.mark.gpu
L = 2**252 + 27742317777372353535851937790883648493


@pytest.mark.parametrize("name", ["ed25519_valid.npz", "ed25519_edge.npz"])
def test_golden(gpu_engine, name):
    d = load_npz(name)
    got = gpu_engine.verify_batch(d["sig"], d["pk"], d["msgs"], d["off"])
    assert (got == d["expect"].astype(bool)).all(), np.nonzero(got != d["expect"].astype(bool))


def test_signer_matches_libsodium(gpu_engine):
    k = load_npz("sign_kat.npz")
    pk, sk = gpu_engine.seed_keypair_batch(k["seed"])
    assert (pk == k["pk"]).all()
    sig = gpu_engine.sign_batch(sk, np.arange(len(pk), dtype=np.uint32), k["msgs"], k["off"])
    assert (sig == k["sig"]).all()


def _random_batch(eng, n, seed, mlen_max=600):
    rng = np.random.default_rng(seed)
    pk, sk = eng.seed_keypair_batch(rng.integers(0, 256, (97, 32), dtype=np.uint8))
    kidx = rng.integers(0, 97, n).astype(np.uint32)
    msgs = [bytes(rng.integers(0, 256, int(rng.integers(0, mlen_max)), dtype=np.uint8)) for _ in range(n)]
    buf, off = pack_messages(msgs)
    sig = eng.sign_batch(sk, kidx, buf, off)
    pks = pk[kidx].copy()
    # corruptions, ~40%: R / S / pk bit flips, S + L, S high bit, random pk
    for i in range(n):
        r = rng.random()
        if r < 0.08:
            sig[i, rng.integers(0, 32)] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.16:
            sig[i, 32 + rng.integers(0, 32)] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.24:
            pks[i, rng.integers(0, 32)] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.30:
            s = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
            if s < 2**256:
                sig[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif r < 0.34:
            sig[i, 63] |= 0x80
        elif r < 0.40:
            pks[i] = rng.integers(0, 256, 32, dtype=np.uint8)
    return sig, pks, msgs, buf, off


def test_random_batch_vs_oracle(gpu_engine, oracle):
    n = 3001  # not a multiple of 64: ragged last ballot word
    sig, pks, msgs, buf, off = _random_batch(gpu_engine, n, 1)
    got = gpu_engine.verify_batch(sig, pks, buf, off)
    want = np.array([oracle.oracle_verify_detached(sig[i].tobytes(), msgs[i], len(msgs[i]), pks[i].tobytes()) == 0
                     for i in range(n)])
    assert (got == want).all(), np.nonzero(got != want)
    assert 0.5 < want.mean() < 0.75


def test_general_key_dedupe(gpu_engine, oracle):
    """General path, distinct-key dedupe (edv_dedup_*): requests share keys;
    keys that differ only in words the slot hash ignores (bytes 16..19 and
    24..27) collide in the hash table and must still get their own tables;
    a non-decodable key repeated across requests rejects all of them."""
    rng = np.random.default_rng(11)
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (5, 32), dtype=np.uint8))
    n = 2500
    kidx = rng.integers(0, 5, n).astype(np.uint32)
    msgs = [bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)) for _ in range(n)]
    buf, off = pack_messages(msgs)
    sig = gpu_engine.sign_batch(sk, kidx, buf, off)
    pks = pk[kidx].copy()
    variant = rng.integers(0, 4, n)
    pks[variant == 1, 16] ^= 0x01  # same slot hash as the true key
    pks[variant == 2, 25] ^= 0x40  # ditto
    pks[variant == 3] = pk[kidx[variant == 3]]
    pks[variant == 3, 31] = 0x7F  # y >= p for many keys: usually fails to decode
    pks[variant == 3, :31] = 0xFF
    got = gpu_engine.verify_batch(sig, pks, buf, off)
    want = np.array([oracle.oracle_verify_detached(sig[i].tobytes(), msgs[i], len(msgs[i]), pks[i].tobytes()) == 0
                     for i in range(n)])
    assert (got == want).all(), np.nonzero(got != want)
    assert want[variant == 0].all() and not want[variant != 0].any()


def test_general_distinct_keys(gpu_engine, oracle):
    """Every request its own key (the dedupe's worst case), 4 sub-batches."""
    rng = np.random.default_rng(12)
    n = 5000
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (n, 32), dtype=np.uint8))
    msgs = [bytes(rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8)) for _ in range(n)]
    buf, off = pack_messages(msgs)
    sig = gpu_engine.sign_batch(sk, np.arange(n, dtype=np.uint32), buf, off)
    bad = rng.choice(n, 250, replace=False)
    sig[bad, 5] ^= 0x20
    with gpu_engine.options(pipeline=4):  # (the previous options come back however the block ends)
        got = gpu_engine.verify_batch(sig, pk, buf, off)
    assert gpu_engine.get_options()["pipeline"] == 1
    want = np.ones(n, bool)
    want[bad] = False
    assert (got == want).all(), np.nonzero(got != want)


def test_message_offsets_and_alignment(gpu_engine, oracle):
    # msg_off[0] != 0, odd offsets, empty messages, zero-length batch
    sig, pks, msgs, buf, off = _random_batch(gpu_engine, 257, 2, mlen_max=50)
    pad = np.concatenate([np.full(3, 0xAB, np.uint8), buf])
    got = gpu_engine.verify_batch(sig, pks, pad, off + 3)
    ref = gpu_engine.verify_batch(sig, pks, buf, off)
    assert (got == ref).all()
    assert gpu_engine.verify_batch(np.zeros((0, 64), np.uint8), np.zeros((0, 32), np.uint8),
                                   np.zeros(0, np.uint8), np.zeros(1, np.uint64)).shape == (0,)
    e = load_npz("ed25519_edge.npz")
    got = gpu_engine.verify_batch(e["sig"][:1], e["pk"][:1], e["msgs"], e["off"][:2])
    assert got.tolist() == [bool(e["expect"][0])]


def test_sign_open_any_signature_length(gpu_engine, oracle):
    d = items_of(load_npz("ed25519_valid.npz"))[:40]
    sms, pks = [], []
    for j, (sig, pk, msg, _) in enumerate(d):
        cut = [64, 63, 65, 0, 10, 64][j % 6]
        s = (sig + b"\x01")[:cut] if cut <= 65 else sig
        sms.append(s + msg)
        pks.append(pk)
    buf, off = pack_messages(sms)
    got = gpu_engine.sign_open_batch(buf, off, np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32))
    want = [oracle.oracle_sign_open(sm, len(sm), pk) == 0 for sm, pk in zip(sms, pks)]
    assert got.tolist() == want
    assert sum(want) == len([j for j in range(40) if j % 6 in (0, 5)])


@pytest.fixture(scope="module")
def nym_1m(gpu_engine):
    """BASELINE configs[1] on the device: 1M NYM requests (~200 B signed
    payload, synth.nym_messages), 1,000 signers, signed on the GPU."""
    import torch
    from plenum_amd import synth
    n = 1_000_000
    pks, sks = gpu_engine.seed_keypair_batch(synth.signer_seeds(1000))
    msgs, kidx, _ = synth.nym_messages(n, pks, alias_len=43)
    buf, off = pack_messages(msgs)
    dev = torch.device("cuda", 0)
    d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    gpu_engine.sign_batch_device(torch.from_numpy(sks).to(dev), torch.from_numpy(kidx.astype(np.int32)).to(dev),
                                 d_msgs, d_off, n, d_sig)
    torch.cuda.synchronize()
    return dict(n=n, pks=pks, kidx=kidx, buf=buf, off=off, sig=d_sig.cpu().numpy(), msgs=msgs)


def _bits(words, n):
    return np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)


def _oracle_sample(oracle, sig, pk, buf, off, idx):
    return np.array([oracle.oracle_verify_detached(sig[i].tobytes(), buf[int(off[i]):int(off[i + 1])].tobytes(),
                                                   int(off[i + 1] - off[i]), pk[i].tobytes()) == 0 for i in idx])


def test_large_batch_properties(gpu_engine, nym_1m):
    """1M requests (BASELINE configs[1] size), general path: every honest
    signature accepted, every corrupted one rejected, bitmask popcount exact;
    plus a checksum of the accept mask stable across two launches."""
    import torch
    n, dev = nym_1m["n"], torch.device("cuda", 0)
    sig = nym_1m["sig"].copy()
    rng = np.random.default_rng(5)
    bad = rng.choice(n, n // 20, replace=False)
    sig[bad, 40] ^= 0x10
    d_sig = torch.from_numpy(sig).to(dev)
    d_pk = torch.from_numpy(nym_1m["pks"][nym_1m["kidx"]]).to(dev)
    d_msgs = torch.from_numpy(np.concatenate([nym_1m["buf"], np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(nym_1m["off"].view(np.int64)).to(dev)
    words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    digests = []
    for _ in range(2):
        gpu_engine.verify_batch_device(d_sig, d_pk, d_msgs, d_off, n, words)
        torch.cuda.synchronize()
        digests.append(hashlib.sha256(words.cpu().numpy().tobytes()).hexdigest())
    bits = _bits(words, n)
    want = np.ones(n, bool)
    want[bad] = False
    wrong = np.nonzero(bits != want)[0]
    assert len(wrong) == 0, (len(wrong), wrong[:8], wrong[-8:], bits[wrong[:8]])
    assert digests[0] == digests[1]


@pytest.mark.parametrize("config,w,sort", [("c1", 14, "auto"), ("c2", 14, "auto"), ("c2", 16, "auto"),
                                           ("c2", 16, "off")])
def test_keyed_headline_1m(gpu_engine, oracle, sodium_verdicts, nym_1m, config, w, sort):
    """The headline configuration as bench.py times it: key-table path at key
    window 14 / 16, 1M requests, message spans, 4 sub-batches, the comb in
    key-sorted order (edv_set_key_sort auto) or request order.  c1: all valid ->
    every bit set.  c2: the configs[2] 10% corruption mix (synth.corrupt_configs2:
    R/S/M bit flips, S+L, S|2^255, small-order and non-canonical A, R = identity,
    R+T8; corrupted keys registered as keys of their own) -> the construction's
    verdicts exactly.  Both: ALL 1M verdicts == libsodium 1.0.18's
    crypto_sign_verify_detached on the same bytes (every host CPU), plus a
    small C-oracle sample."""
    import torch
    from plenum_amd import synth
    n, dev = nym_1m["n"], torch.device("cuda", 0)
    sig, buf, off = nym_1m["sig"].copy(), nym_1m["buf"].copy(), nym_1m["off"]
    pk = nym_1m["pks"][nym_1m["kidx"]].copy()
    expect = np.ones(n, bool)
    if config == "c2":
        expect = synth.corrupt_configs2(sig, pk, buf, off, np.random.default_rng(2))
    uniq, inv = np.unique(pk, axis=0, return_inverse=True)
    try:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(w)
        gpu_engine.set_key_sort(sort)
        assert gpu_engine.keys_add(uniq) == 0
        d_sig = torch.from_numpy(sig).to(dev)
        d_k = torch.from_numpy(inv.reshape(-1).astype(np.int32)).to(dev)
        d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
        d_ms = torch.from_numpy(off[:-1].astype(np.int64)).to(dev)
        d_me = torch.from_numpy(off[1:].astype(np.int64)).to(dev)
        words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        gpu_engine.set_pipeline(4)
        gpu_engine.verify_spans_device(d_sig, d_k, True, d_msgs, d_ms, d_me, n, words)
        torch.cuda.synchronize()
        got = _bits(words, n)
    finally:
        gpu_engine.set_key_sort("auto")
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(10)
    wrong = np.nonzero(got != expect)[0]
    assert len(wrong) == 0, (config, len(wrong), wrong[:8])
    lib = sodium_verdicts(sig, pk, buf, off[:-1], off[1:])  # every item, libsodium itself
    wrong = np.nonzero(got != lib)[0]
    assert len(wrong) == 0, (config, "vs libsodium", len(wrong), wrong[:8])
    rng = np.random.default_rng(77)
    bad = np.nonzero(~expect)[0]
    idx = np.concatenate([rng.choice(n, 300, replace=False),
                          bad[:300] if len(bad) else np.zeros(0, np.int64), [0, n - 1]]).astype(np.int64)
    assert (_oracle_sample(oracle, sig, pk, buf, off, idx) == got[idx]).all()


# ---- key-table path -------------------------------------------------------
def test_keyed_golden_and_edge(gpu_engine):
    """Every golden item through the key-table path (each item's pk registered
    as its own key): same verdicts as libsodium, including small-order,
    non-canonical and off-curve keys, and mixed-order keys."""
    for name in ("ed25519_edge.npz", "ed25519_valid.npz"):
        d = load_npz(name)
        gpu_engine.keys_reset()
        first = gpu_engine.keys_add(d["pk"])
        kidx = np.arange(first, first + len(d["pk"]), dtype=np.uint32)
        got = gpu_engine.verify_batch_keyed(d["sig"], kidx, d["msgs"], d["off"])
        assert (got == d["expect"].astype(bool)).all(), np.nonzero(got != d["expect"].astype(bool))


def test_keyed_random_vs_oracle_and_out_of_range(gpu_engine, oracle):
    n = 2049
    sig, pks, msgs, buf, off = _random_batch(gpu_engine, n, 9)
    gpu_engine.keys_reset()
    uniq, inv = np.unique(pks, axis=0, return_inverse=True)
    first = gpu_engine.keys_add(uniq)
    kidx = (inv.reshape(-1) + first).astype(np.uint32)
    got = gpu_engine.verify_batch_keyed(sig, kidx, buf, off)
    want = gpu_engine.verify_batch(sig, pks, buf, off)
    assert (got == want).all()
    kidx[::5] = gpu_engine.keys_count() + 7  # unregistered ids reject
    got = gpu_engine.verify_batch_keyed(sig, kidx, buf, off)
    assert not got[::5].any() and (got[1::5] == want[1::5]).all()


@pytest.mark.parametrize("pipeline", [1, 3])
def test_key_sorted_comb_matches_request_order(gpu_engine, oracle, pipeline):
    """edv_set_key_sort: the comb in key-sorted lane order (counting sort of
    the key ids; the encode reads the permutation back and packs verdict
    bytes) gives the request-order verdicts bit for bit: 20,011 requests
    (not a multiple of 64), 1,500 keys in random order, 5% of the ids
    unregistered, 10% of the signatures corrupted, 1 or 3 sub-batches (each
    sorts with its own scratch); == the general path with the same keys."""
    n = 20011
    rng = np.random.default_rng(31)
    seeds = rng.integers(0, 256, size=(1500, 32), dtype=np.uint8)
    pks, sks = gpu_engine.seed_keypair_batch(seeds)
    msgs = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 400)), dtype=np.uint8)) for _ in range(n)]
    buf, off = pack_messages(msgs)
    kid = rng.integers(0, 1500, size=n).astype(np.uint32)
    sig = gpu_engine.sign_batch(sks, kid, buf, off)
    bad = rng.random(n) < 0.10
    sig[bad, rng.integers(0, 64, size=int(bad.sum()))] ^= 1
    want = gpu_engine.verify_batch(sig, pks[kid], buf, off)
    try:
        gpu_engine.keys_reset()
        first = gpu_engine.keys_add(pks)
        ids = kid + np.uint32(first)
        drop = rng.random(n) < 0.05
        ids[drop] = gpu_engine.keys_count() + 3
        gpu_engine.set_pipeline(pipeline)
        got = {}
        for mode in ("off", "on", "auto"):
            gpu_engine.set_key_sort(mode)
            got[mode] = gpu_engine.verify_batch_keyed(sig, ids, buf, off)
    finally:
        gpu_engine.set_key_sort("auto")
        gpu_engine.set_pipeline(1)
        gpu_engine.keys_reset()
    exp = want & ~drop
    for mode, g in got.items():
        assert (g == exp).all(), (mode, np.nonzero(g != exp)[0][:8])
    idx = np.nonzero(~drop)[0][:300]
    assert (_oracle_sample(oracle, sig, pks[kid], buf, off, idx) == got["on"][idx]).all()


@pytest.mark.parametrize("w", [4, 6, 8, 12, 13, 14, 16])
def test_keyed_every_window(gpu_engine, w):
    """The key store at every window edv_keys_set_window accepts (the default
    10 is covered above): golden edge + valid items, each key its own table."""
    e, v = load_npz("ed25519_edge.npz"), load_npz("ed25519_valid.npz")
    try:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(w)
        assert gpu_engine.keys_window == w
        for d, step in ((e, 2), (v, 9)):
            gpu_engine.keys_reset()
            sel = np.arange(0, len(d["pk"]), step)
            first = gpu_engine.keys_add(d["pk"][sel])
            kidx = np.full(len(d["pk"]), 0xFFFFFFFF, np.uint32)
            kidx[sel] = np.arange(first, first + len(sel), dtype=np.uint32)
            got = gpu_engine.verify_batch_keyed(d["sig"], kidx, d["msgs"], d["off"])
            want = d["expect"].astype(bool).copy()
            want[np.setdiff1d(np.arange(len(want)), sel)] = False  # unregistered ids reject
            assert (got == want).all(), (w, np.nonzero(got != want))
    finally:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(10)


@pytest.mark.parametrize("w", [10, 13])
def test_keyed_store_growth(gpu_engine, w):
    """Keys registered in slices across key-store growth (64 -> 128 -> 256
    tables): the row-major store is re-laid out on every growth, and earlier
    keys keep their verdicts."""
    d = load_npz("ed25519_edge.npz")
    try:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(w)
        ids = []
        for a in range(0, len(d["pk"]), 40):
            first = gpu_engine.keys_add(d["pk"][a:a + 40])
            ids.extend(range(first, first + len(d["pk"][a:a + 40])))
        kidx = np.asarray(ids, np.uint32)
        got = gpu_engine.verify_batch_keyed(d["sig"], kidx, d["msgs"], d["off"])
        assert (got == d["expect"].astype(bool)).all(), np.nonzero(got != d["expect"].astype(bool))
    finally:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(10)


@pytest.mark.parametrize("n", [1023, 1024, 1025, 4096, 4097, 6143])
def test_sub_batch_boundaries(gpu_engine, oracle, n):
    """The pipelined launcher cuts a chunk into up to 4 sub-batches aligned to
    1024 requests on two streams: sizes around those boundaries give the same
    bits as one un-pipelined launch, and both match the oracle (sampled)."""
    sig, pks, msgs, buf, off = _random_batch(gpu_engine, n, 100 + n, mlen_max=120)
    gpu_engine.set_pipeline(4)
    gpu_engine.set_length_buckets(False)
    got4 = gpu_engine.verify_batch(sig, pks, buf, off)
    per = -(-(-(-n // 4)) // 1024) * 1024  # ceil(ceil(n / 4) / 1024) * 1024
    assert gpu_engine.last_launch_count() == -(-n // per)
    gpu_engine.set_length_buckets(True)  # sorted hash lanes: at most 2 sub-batches
    got2 = gpu_engine.verify_batch(sig, pks, buf, off)
    per = -(-(-(-n // 2)) // 1024) * 1024
    assert gpu_engine.last_launch_count() == -(-n // per)
    gpu_engine.set_length_buckets("auto")
    gpu_engine.set_pipeline(1)
    got1 = gpu_engine.verify_batch(sig, pks, buf, off)
    assert gpu_engine.last_launch_count() == 1
    gpu_engine.set_pipeline(4)
    assert (got4 == got1).all(), np.nonzero(got4 != got1)
    assert (got2 == got1).all(), np.nonzero(got2 != got1)
    for i in list(range(0, n, 97)) + [n - 1]:
        want = oracle.oracle_verify_detached(sig[i].tobytes(), msgs[i], len(msgs[i]), pks[i].tobytes()) == 0
        assert got4[i] == want, i
    # keyed path: the same requests against registered keys
    gpu_engine.keys_reset()
    uniq, inv = np.unique(pks, axis=0, return_inverse=True)
    gpu_engine.keys_add(uniq)
    gotk = gpu_engine.verify_batch_keyed(sig, inv.reshape(-1).astype(np.uint32), buf, off)
    assert (gotk == got1).all(), np.nonzero(gotk != got1)


def test_length_buckets_mixed_lengths(gpu_engine, oracle):
    """configs[3]-style lengths (log-uniform 0 B .. 4 KiB): the hash lanes run in
    SHA-512 block-count order; verdicts equal the unsorted run and the oracle."""
    rng = np.random.default_rng(33)
    n = 2500
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (31, 32), dtype=np.uint8))
    kidx = rng.integers(0, 31, n).astype(np.uint32)
    lens = np.exp(rng.uniform(0, np.log(4096), n)).astype(int)
    lens[::17] = 0
    msgs = [bytes(rng.integers(0, 256, int(m), dtype=np.uint8)) for m in lens]
    buf, off = pack_messages(msgs)
    sig = gpu_engine.sign_batch(sk, kidx, buf, off)
    sig[::5, 33] ^= 4
    pks = pk[kidx]
    assert lengths_mixed(off[:-1], off[1:])
    gpu_engine.set_length_buckets(True)
    got = gpu_engine.verify_batch(sig, pks, buf, off)
    gpu_engine.set_length_buckets(False)
    plain = gpu_engine.verify_batch(sig, pks, buf, off)
    gpu_engine.set_length_buckets("auto")
    auto = gpu_engine.verify_batch(sig, pks, buf, off)
    assert (got == plain).all(), np.nonzero(got != plain)
    assert (auto == plain).all(), np.nonzero(auto != plain)
    gpu_engine.keys_reset()
    gpu_engine.keys_add(pk)
    gpu_engine.set_length_buckets(True)
    keyed = gpu_engine.verify_batch_keyed(sig, kidx, buf, off)
    gpu_engine.set_length_buckets("auto")
    assert (keyed == plain).all(), np.nonzero(keyed != plain)
    want = np.ones(n, bool)
    want[::5] = False
    assert (got == want).all(), np.nonzero(got != want)
    for i in range(0, n, 83):
        assert got[i] == (oracle.oracle_verify_detached(sig[i].tobytes(), msgs[i], len(msgs[i]),
                                                       pks[i].tobytes()) == 0), i


@pytest.mark.parametrize("arena", [None, 300 * 1024])
def test_packed_units_mixed_lengths(gpu_engine, oracle, arena):
    """Length-bucketed SoA packing (mode "packed", north_star (1)): messages of
    every SHA-512 block count 0 B .. 4 KiB (plus exact block boundaries) at
    every byte alignment, packed into lane-interleaved units and hashed from
    them; the bits equal the in-place (AoS) run and the oracle, on both paths.
    A 300 KiB arena holds only the first groups: the rest are read in place."""
    rng = np.random.default_rng(35)
    n = 3000
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (23, 32), dtype=np.uint8))
    kidx = rng.integers(0, 23, n).astype(np.uint32)
    lens = np.exp(rng.uniform(0, np.log(4096), n)).astype(int)
    lens[::13] = 0
    edges = [128 * b + d for b in range(33) for d in (-81, -80, -79, -65, -64, -63) if 0 <= 128 * b + d <= 4096]
    lens[2::11][:len(edges)] = edges
    msgs = [bytes(rng.integers(0, 256, int(m), dtype=np.uint8)) for m in lens]
    buf, off = pack_messages(msgs)
    sig = gpu_engine.sign_batch(sk, kidx, buf, off)
    sig[::6, 12] ^= 2
    sig[3::11, 50] ^= 8
    pks = pk[kidx]
    gpu_engine.set_length_buckets(False)
    plain = gpu_engine.verify_batch(sig, pks, buf, off)
    try:
        if arena is not None:
            gpu_engine.set_unit_arena(arena)
        gpu_engine.set_length_buckets("packed")
        got = gpu_engine.verify_batch(sig, pks, buf, off)
        assert (got == plain).all(), np.nonzero(got != plain)
        gpu_engine.keys_reset()
        gpu_engine.keys_add(pk)
        keyed = gpu_engine.verify_batch_keyed(sig, kidx, buf, off)
        assert (keyed == plain).all(), np.nonzero(keyed != plain)
    finally:
        gpu_engine.set_length_buckets("auto")
        gpu_engine.set_unit_arena(1280 << 20)
        gpu_engine.keys_reset()
    want = np.ones(n, bool)
    want[::6] = False
    want[3::11] = False
    assert (plain == want).all(), np.nonzero(plain != want)
    for i in range(0, n, 71):
        assert got[i] == (oracle.oracle_verify_detached(sig[i].tobytes(), msgs[i], len(msgs[i]),
                                                       pks[i].tobytes()) == 0), i


def test_spans_share_messages(gpu_engine):
    """edv_verify_spans_device: k signatures over one message copy (multi-sig
    requests) give the same bits as the contiguous layout with duplicated
    messages, on both paths."""
    import torch
    rng = np.random.default_rng(34)
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (9, 32), dtype=np.uint8))
    reqs = [bytes(rng.integers(0, 256, int(rng.integers(64, 900)), dtype=np.uint8)) for _ in range(300)]
    rbuf, roff = pack_messages(reqs)
    item_req, item_key = [], []
    for r in range(len(reqs)):
        k = int(rng.integers(1, 6))
        item_req += [r] * k
        item_key += list(rng.choice(9, k, replace=False))
    item_req = np.array(item_req)
    item_key = np.array(item_key, np.uint32)
    n = len(item_req)
    dup = [reqs[r] for r in item_req]
    dbuf, doff = pack_messages(dup)
    sig = gpu_engine.sign_batch(sk, item_key, dbuf, doff)
    sig[::7, 5] ^= 1
    want = gpu_engine.verify_batch(sig, pk[item_key], dbuf, doff)
    assert want.sum() == n - len(range(0, n, 7))
    dev = torch.device("cuda", 0)
    d_sig = torch.from_numpy(sig).to(dev)
    d_msgs = torch.from_numpy(np.concatenate([rbuf, np.zeros(16, np.uint8)])).to(dev)
    d_ms = torch.from_numpy(roff[:-1][item_req].astype(np.int64)).to(dev)
    d_me = torch.from_numpy(roff[1:][item_req].astype(np.int64)).to(dev)
    words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    d_pk = torch.from_numpy(pk[item_key]).to(dev)
    gpu_engine.verify_spans_device(d_sig, d_pk, False, d_msgs, d_ms, d_me, n, words)
    torch.cuda.synchronize()
    got = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert (got == want).all()
    gpu_engine.keys_reset()
    gpu_engine.keys_add(pk)
    words.zero_()
    d_k = torch.from_numpy(item_key.astype(np.int32)).to(dev)
    gpu_engine.verify_spans_device(d_sig, d_k, True, d_msgs, d_ms, d_me, n, words)
    torch.cuda.synchronize()
    got = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert (got == want).all()
    for keyed, keys, mode in ((True, d_k, True), (False, d_pk, True), (True, d_k, "packed"),
                              (False, d_pk, "packed")):  # sorted / packed hash lanes over spans
        gpu_engine.set_length_buckets(mode)
        words.zero_()
        gpu_engine.verify_spans_device(d_sig, keys, keyed, d_msgs, d_ms, d_me, n, words)
        torch.cuda.synchronize()
        gpu_engine.set_length_buckets("auto")
        got = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        assert (got == want).all(), (keyed, mode)


def test_sig_slots_match_sig64(gpu_engine, oracle):
    """EDV_SIG_SLOT96: the same batch as 64-byte signatures and as slots
    (base58 text where it decodes to 64 bytes, else raw) gives identical
    verdicts on both paths; texts with leading '1's (R with leading zero
    bytes), the all-'1' text (64 zero bytes), raw slots and corrupted texts
    included; a sample agrees with the oracle."""
    from plenum_amd import _hostpack, pack_messages
    rng = np.random.default_rng(31)
    n = 40000
    seeds = rng.integers(0, 256, size=(16, 32), dtype=np.uint8)
    pk, sk = gpu_engine.seed_keypair_batch(seeds)
    msgs = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 300)), dtype=np.uint8)) for _ in range(n)]
    buf, off = pack_messages(msgs)
    kidx = (np.arange(n) % 16).astype(np.uint32)
    sig = gpu_engine.sign_batch(sk, kidx, buf, off)
    sig[::7, 50] ^= 4                      # corrupted S
    sig[1] = 0                             # all zero: the text is 64 '1's
    sig[2, :3] = 0                         # leading zero bytes
    texts = _hostpack.b58encode_rows(sig.tobytes(), 64)
    slots = np.zeros((n, 96), np.uint8)
    raw = np.zeros(n, bool)
    raw[::13] = True                       # host-decoded slots
    for i, t in enumerate(texts):
        assert _hostpack.b58_len64(t) == 1
        if raw[i]:
            slots[i, :64] = sig[i]
        else:
            slots[i, :len(t)] = np.frombuffer(t.encode(), np.uint8)
            slots[i, 95] = len(t)
    assert (slots[:, 95] > 0).sum() > 30000 and texts[1] == "1" * 64 and texts[2].startswith("111")
    want = gpu_engine.verify_batch(sig, pk[kidx], buf, off)
    got = gpu_engine.verify_batch(slots, pk[kidx], buf, off, sig_slot=96)
    assert (got == want).all() and want.sum() > n * 0.8
    uniq_ids = gpu_engine.keys_add(pk)
    try:
        gotk = gpu_engine.verify_batch_keyed(slots, kidx + uniq_ids, buf, off, sig_slot=96)
        assert (gotk == want).all()
    finally:
        gpu_engine.keys_reset()
    idx = rng.choice(n, 500, replace=False)
    assert (_oracle_sample(oracle, sig, pk[kidx], buf, off, idx) == got[idx]).all()


@pytest.mark.parametrize("w", [4, 6, 10, 14, 16])
def test_small_batch_kernel_matches_batch_path(gpu_engine, oracle, w):
    """edv_verify_small_kernel (keyed host-pointer batches of <= 256 requests:
    rows on lanes summed as trees, R decoded instead of R' inverted) gives the
    batch kernels' verdicts bit for bit: every golden edge item (small-order
    and non-canonical R, A and S, R + T8, mixed-order keys) and valid item in
    chunks of 1 / 7 / 64 / 256 requests, unregistered ids, and random
    corrupted signatures, at every comb window shape (64 / 43 / 26 / 19 / 16
    key rows)."""
    e, v = load_npz("ed25519_edge.npz"), load_npz("ed25519_valid.npz")
    try:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(w)
        for d in (e, v):
            gpu_engine.keys_reset()
            first = gpu_engine.keys_add(d["pk"])
            kidx = np.arange(first, first + len(d["pk"]), dtype=np.uint32)
            kidx[5::11] = gpu_engine.keys_count() + 1  # unregistered
            want = d["expect"].astype(bool).copy()
            want[5::11] = False
            gpu_engine.set_small_batch(0)
            big = gpu_engine.verify_batch_keyed(d["sig"], kidx, d["msgs"], d["off"])
            assert (big == want).all(), (w, np.nonzero(big != want)[0][:8])
            gpu_engine.set_small_batch(256)
            for step in (1, 7, 64, 256):
                for a in range(0, len(kidx), step):
                    b = min(len(kidx), a + step)
                    off = d["off"][a:b + 1]
                    got = gpu_engine.verify_batch_keyed(d["sig"][a:b], kidx[a:b], d["msgs"], off)
                    assert (got == want[a:b]).all(), (w, step, a, np.nonzero(got != want[a:b])[0][:8])
                if step == 1 and len(kidx) > 300:
                    break  # one request per call over the edge set only (hundreds of launches)
        # random batch with corrupted S / R / M bits and shared keys
        n = 200
        sig, pks, msgs, buf, off = _random_batch(gpu_engine, n, 41)
        gpu_engine.keys_reset()
        uniq, inv = np.unique(pks, axis=0, return_inverse=True)
        first = gpu_engine.keys_add(uniq)
        kidx = (inv.reshape(-1) + first).astype(np.uint32)
        gpu_engine.set_small_batch(0)
        big = gpu_engine.verify_batch_keyed(sig, kidx, buf, off)
        gpu_engine.set_small_batch(256)
        small = gpu_engine.verify_batch_keyed(sig, kidx, buf, off)
        assert (small == big).all()
        idx = np.arange(0, n, 7)
        assert (_oracle_sample(oracle, sig, pks, buf, off, idx) == small[idx]).all()
    finally:
        gpu_engine.set_small_batch(256)
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(10)


def test_verify_one_keyed_matches_batch(gpu_engine):
    """EdVerifyEngine.verify_one_keyed (one authenticate() that missed the verify-ahead cache:
    bytes in, the small kernel, its verdict byte straight into pinned host memory) gives the
    batch path's verdict on every golden edge item and on unregistered ids."""
    e = load_npz("ed25519_edge.npz")
    try:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(14)
        first = gpu_engine.keys_add(e["pk"])
        kidx = np.arange(first, first + len(e["pk"]), dtype=np.uint32)
        kidx[5::11] = gpu_engine.keys_count() + 1  # unregistered
        want = e["expect"].astype(bool).copy()
        want[5::11] = False
        msgs, off = bytes(e["msgs"]), e["off"]
        for i in range(len(kidx)):
            got = gpu_engine.verify_one_keyed(bytes(e["sig"][i]), int(kidx[i]), msgs[int(off[i]):int(off[i + 1])])
            assert got == bool(want[i]), i
    finally:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(10)


def test_resident_single_request_path(gpu_engine, oracle):
    """edv_verify_one's resident kernel (one workgroup taking requests from a pinned mailbox):
    the same verdicts as the oracle through everything that makes it leave and come back --
    back-to-back requests, a batch call between two (the yield), an idle gap longer than its
    200 us timeout, a message over its 4 KiB mailbox (the launch path), a key window change
    (a kernel of the new window), and a key slot rebuilt for another key between two requests
    (the verdict follows the new key: no stale table lines read from the kernel's caches)."""
    import time
    rng = np.random.default_rng(41)
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (6, 32), dtype=np.uint8))
    lens = [0, 1, 63, 64, 200, 255, 1000, 4095, 4096, 4097, 6000] + [int(x) for x in rng.integers(0, 400, 60)]
    msgs = [bytes(rng.integers(0, 256, m, dtype=np.uint8)) for m in lens]
    kidx = (np.arange(len(msgs)) % 4).astype(np.uint32)
    buf, off = pack_messages(msgs)
    sig = gpu_engine.sign_batch(sk, kidx, buf, off)
    sig[3::7, 5] ^= 4  # forged R
    sig[4::9, 40] ^= 1  # forged S

    def want(i, key):
        return oracle.oracle_verify_detached(sig[i].tobytes(), msgs[i], len(msgs[i]), pk[key].tobytes()) == 0
    try:
        for w in (10, 14):
            gpu_engine.keys_reset()
            gpu_engine.keys_set_window(w)
            assert gpu_engine.keys_add(pk[:4]) == 0
            for i in range(len(msgs)):
                assert gpu_engine.verify_one_keyed(bytes(sig[i]), int(kidx[i]), msgs[i]) == want(i, kidx[i]), (w, i)
                if i % 10 == 3:  # a batch call between two single requests
                    got = gpu_engine.verify_batch_keyed(sig[:8], kidx[:8], buf, off[:9])
                    assert list(got) == [want(j, kidx[j]) for j in range(8)]
                if i % 10 == 6:
                    time.sleep(0.002)  # longer than the idle timeout: the kernel has left
            # an unregistered id rejects
            assert not gpu_engine.verify_one_keyed(bytes(sig[0]), 4 + 9, msgs[0])
        # slot 0 rebuilt for key 4 (an eviction): requests of key 0 now reject, key 4's accept
        i0 = int(np.flatnonzero((kidx == 0) & (np.array(lens) < 300))[0])
        assert gpu_engine.verify_one_keyed(bytes(sig[i0]), 0, msgs[i0]) == want(i0, 0)
        gpu_engine.keys_set(0, pk[4:5])
        assert gpu_engine.verify_one_keyed(bytes(sig[i0]), 0, msgs[i0]) == want(i0, 4)
        m4 = b"key four"
        b4, o4 = pack_messages([m4])
        s4 = gpu_engine.sign_batch(sk[4:5], np.zeros(1, np.uint32), b4, o4)
        assert gpu_engine.verify_one_keyed(bytes(s4[0]), 0, m4)
    finally:
        gpu_engine.keys_reset()
        gpu_engine.keys_set_window(10)


def test_resident_single_request_is_faster_than_a_launch(gpu_engine):
    """The reason for the resident kernel: one request's engine call (p50 of 300 back to back)
    is shorter than with a kernel launch per request (a context created with EDV_RESIDENT=0)."""
    import os
    import time
    from plenum_amd import EdVerifyEngine
    rng = np.random.default_rng(43)
    pk, sk = gpu_engine.seed_keypair_batch(rng.integers(0, 256, (2, 32), dtype=np.uint8))
    msg = bytes(rng.integers(0, 256, 200, dtype=np.uint8))
    b, o = pack_messages([msg])
    sig = bytes(gpu_engine.sign_batch(sk, np.zeros(1, np.uint32), b, o)[0])
    os.environ["EDV_RESIDENT"] = "0"
    try:
        launch_eng = EdVerifyEngine(0)
    finally:
        del os.environ["EDV_RESIDENT"]
    try:
        p50 = {}
        for name, eng in (("resident", gpu_engine), ("launch", launch_eng)):
            eng.keys_reset()
            eng.keys_set_window(10)
            eng.keys_add(pk)
            lat = []
            for _ in range(330):
                t = time.perf_counter()
                assert eng.verify_one_keyed(sig, 0, msg)
                lat.append(time.perf_counter() - t)
            p50[name] = float(np.median(lat[30:])) * 1e6
        print("engine call p50 us:", p50)
        assert p50["resident"] < p50["launch"], p50
    finally:
        launch_eng.close()
        gpu_engine.keys_reset()
