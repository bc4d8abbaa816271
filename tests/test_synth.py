"""The bench's synthetic NYM payloads are exactly what a Plenum client signs:
serialize_msg_for_signing(request, ['signature']) (signer_did.py:114-121)."""
import numpy as np

from plenum_amd import synth


def test_nym_messages_equal_serializer_output():
    pks = np.random.default_rng(0).integers(0, 256, (7, 32), dtype=np.uint8)
    for alias_len in (0, 43):
        msgs, kidx, spec = synth.nym_messages(300, pks, alias_len=alias_len, seed=3)
        for i in range(0, 300, 7):
            assert synth.check_nym_message(spec, i, 7, msgs[i])
        assert (kidx == np.arange(300) % 7).all()
    msgs, _, _ = synth.nym_messages(1000, pks, alias_len=43)
    assert abs(np.mean([len(m) for m in msgs]) - 200) < 2


def test_signer_seeds_match_config_c0():
    s = synth.signer_seeds(3)
    assert s[1].tobytes() == (1).to_bytes(2, "little") + b"\0" * 30


def test_add_torsion_changes_R():
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import edwards as E
    R = E.encode(E.mul(12345, E.B))
    Rt = synth.add_torsion(R)
    assert Rt != R and E.mul(8, E.decode(Rt)) == E.mul(8, E.decode(R))


def test_lengths_mixed_rule():
    """The auto length-bucket rule (edverify.hip lengths_mixed, mirrored by
    engine.lengths_mixed): configs[1] NYM payloads (one SHA-512 block count)
    stay unsorted; configs[3]'s log-uniform 64 B - 4 KiB payloads sort."""
    import numpy as np
    from plenum_amd.engine import lengths_mixed
    msgs, _, _ = synth.nym_messages(4096, [bytes(range(32))] * 4)
    lens = np.array([len(m) for m in msgs])
    off = np.concatenate([[0], np.cumsum(lens)])
    assert not lengths_mixed(off[:-1], off[1:])
    rng = np.random.default_rng(3)
    lens = np.exp(rng.uniform(np.log(64), np.log(4096), 4096)).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens)])
    assert lengths_mixed(off[:-1], off[1:])
    assert not lengths_mixed([], [])
    # exactly the 1.25x threshold: one 3-block message per wave of 2-block ones
    blk2, blk3 = 100, 300  # (len + 81 + 127) // 128 = 2 / 3 blocks
    lens = np.full(64, blk2)
    lens[0] = blk3
    off = np.concatenate([[0], np.cumsum(lens)])
    assert lengths_mixed(off[:-1], off[1:])  # 64*3 = 192 > 1.25 * 129


def test_churn_messages_are_the_serialized_dicts():
    """synth.churn_messages' signing bytes == serialize_msg_for_signing of the
    dict churn_request_dict rebuilds; Zipf signers: a long tail and a head."""
    from plenum_amd import synth
    from plenum_amd.serialization import serialize_msg_for_signing
    kidx = synth.zipf_signers(5000, 2000, 1.1, seed=3)
    counts = np.bincount(kidx, minlength=2000)
    assert counts.max() > 200 and (counts == 0).sum() > 500  # a few hot signers, many never seen
    idrs = ["Idr%05d" % k for k in range(2000)]
    msgs, spec = synth.churn_messages(kidx, idrs, alias_len=43)
    for i in range(0, 5000, 97):
        assert serialize_msg_for_signing(synth.churn_request_dict(spec, i), topLevelKeysToIgnore=["signature"]) == \
            msgs[i]
