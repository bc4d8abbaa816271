"""The wave form's BLS check program (tools/gen_bls_program.py -> bls_program.h,
run by edv_bls_verify_wave_kernel) on the CPU:

* the scheduled, slot-allocated program simulated step by step equals the
  oracle's reduced pairing product e(P1, Q1) e(-P2, Q2) -- Q2 Jacobian with
  Z != 1, as a verkey sum reaches it;
* the generated header's program run by the host build of the device code
  (bls_wave.h in libedv_hostcheck.so: Montgomery products, the binary-gcd
  inversion, read-before-write steps) gives bn254.h's verdict on every
  committed case, single and multi-signature, and the oracle's on random
  valid / forged signatures;
* the program's structure: <= 64 operations per step, no step reads a slot
  another operation of the step writes, every slot written before it is read."""
import ctypes
import json
import os
import random
import sys

from conftest import GOLDEN, ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bls_bn254_oracle as o  # noqa: E402
import gen_bls_program as gp  # noqa: E402

V = json.load(open(os.path.join(GOLDEN, "bls_vectors.json")))


def test_program_equals_oracle_pairing_product():
    prog = gp.compile_program()
    assert gp.check(prog, trials=2, seed=7)


def test_program_structure():
    g, ops, outs, steps, slot, nslots, pinned = gp.compile_program()
    written = {slot[x] for x in pinned}
    for st in steps:
        assert 0 < len(st) <= gp.LANES
        dsts = {slot[x] for x in st if ops[x].kind != gp.ZCHK}
        srcs = {slot[a] for x in st for a in ops[x].args()}
        assert not (dsts & srcs)
        assert srcs <= written
        written |= dsts
        for x in st:
            op = ops[x]
            assert len(op.A) + len(op.B) <= gp.MAX_TERMS
            assert op.kind != gp.MUL or (len(op.A) <= 2 and len(op.B) <= 2)
    assert all(slot[x] in written for x in outs)
    assert nslots * 32 <= 64 * 1024  # LDS per wave


def _verify_program(hc, sig, msg, vks, gen):
    f = hc.edv_host_bls_verify_program
    f.restype = ctypes.c_int
    return f(sig, msg, ctypes.c_uint64(len(msg)), b"".join(vks), ctypes.c_uint64(len(vks)), gen)


def test_host_program_matches_device_arithmetic_on_vectors(hostcheck):
    gen = bytes.fromhex(V["generator"])
    msgs = [bytes.fromhex(m) for m in V["messages"]]
    hostcheck.edv_host_bls_verify.restype = ctypes.c_int
    n = 0
    for c in V["cases"]:
        m = msgs[c["msg"]]
        vks = [bytes.fromhex(v) for v in c["vks"]]
        got = _verify_program(hostcheck, bytes.fromhex(c["sig"]), m, vks, gen)
        want = int(c["expect"])
        assert (1 if got == 1 else 0) == want, c["name"]
        assert got != 2, c["name"]
        if len(vks) == 1:
            assert hostcheck.edv_host_bls_verify(bytes.fromhex(c["sig"]), m, ctypes.c_uint64(len(m)), vks[0],
                                                 gen) == want
        n += 1
    assert n >= 10


def test_host_program_random_checks(hostcheck):
    rng = random.Random(3)
    g = o.generator()
    gen = o.g2_to_bytes(g)
    for t in range(3):
        sks = [rng.randrange(1, o.R) for _ in range(1 + t)]
        msg = b"commit %d" % t
        sig = o.aggregate([o.sign(msg, k) for k in sks])
        vks = [o.g2_to_bytes(o.keygen(k)) for k in sks]
        assert _verify_program(hostcheck, o.g1_to_bytes(sig), msg, vks, gen) == 1
        assert _verify_program(hostcheck, o.g1_to_bytes(sig), msg + b"!", vks, gen) == 0
        if len(vks) > 1:
            assert _verify_program(hostcheck, o.g1_to_bytes(sig), msg, vks[:-1], gen) == 0


def test_redo_fixture_needs_more_than_16_hash_candidates():
    """tests/test_gpu_bls.py's REDO_MSG: the wave form's 16 side-by-side candidates of H(m)'s
    try-and-increment are all non-points, so the kernel must hand the check over."""
    import hashlib
    h = int.from_bytes(hashlib.sha256(b"wave-form redo 11075").digest(), "big")
    for k in range(16):
        x = (h + k) % o.P
        assert not o._is_square((x ** 3 + o.B1) % o.P)
    x, y = o.hash_to_g1(b"wave-form redo 11075")
    assert (x - h % o.P) % o.P >= 16
