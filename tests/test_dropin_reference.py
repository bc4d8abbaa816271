"""The drop-in against the REAL reference classes: tests/golden/check_dropin_ref.py
mixes GpuAuthMixin in front of /root/reference's own SimpleAuthNr (Python 3.9,
ref_standins.py) over the oracle-backed engine double and asserts the KAT
outcomes, engine-only verification (0 libsodium calls), the reference's
BaseExc / SuspiciousNode for a forged PROPAGATE (node.py:1313-1316), and 0
engine calls for authenticate() after prefetch().  Runs in the container that
holds the reference (CPU); the committed dropin_ref_check.json is the record."""
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

PY39 = "/opt/conda/bin/python3.9"


@pytest.mark.skipif(not (os.path.exists(PY39) and os.path.isdir("/root/reference/plenum")),
                    reason="needs the reference tree and Python 3.9 (container only)")
def test_mixin_over_reference_simpleauthnr():
    out = subprocess.run([PY39, os.path.join(GOLDEN, "check_dropin_ref.py")], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert got["ok"] and got["libsodium_crypto_sign_open_calls"] == 0 and got["engine_calls"] > 0
    assert got["raised"] == got["raised_reference_baseexc"] > 0
    assert got["authenticate_after_prefetch_engine_calls"] == 0
    assert got["batch_vs_single_matched"] == got["batch_vs_single_items"] > 0


def test_committed_record():
    rec = json.load(open(os.path.join(GOLDEN, "dropin_ref_check.json")))
    assert rec["ok"] and rec["matched"] == rec["cases"] == 64
    assert rec["libsodium_crypto_sign_open_calls"] == 0
    assert rec["forged_propagate"].startswith("SuspiciousNode")
    # authenticate_batch == authenticate() over 5 signers on the reference class, before and after
    # a verkey is replaced, with the batch's keys from the native lookup (the reference's getVerkey)
    assert rec["batch_vs_single_matched"] == rec["batch_vs_single_items"] == 600
    assert rec["known_getverkey"] and rec["keys_known_native_calls"] == 2


@pytest.mark.skipif(not (os.path.exists(PY39) and os.path.isdir("/root/reference/crypto")),
                    reason="needs the reference tree and Python 3.9 (container only)")
def test_bls_classes_over_reference_abcs():
    """plenum_amd.bls against the reference's crypto.bls.bls_crypto ABCs and
    the reference's own BLS test scenarios (tests/golden/check_bls_dropin_ref.py)."""
    out = subprocess.run([PY39, os.path.join(GOLDEN, "check_bls_dropin_ref.py")], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert got["ok"] and all(got["checks"].values()) and got["engine_calls"] > 0


def test_bls_committed_record():
    rec = json.load(open(os.path.join(GOLDEN, "bls_dropin_ref_check.json")))
    assert rec["ok"] and len(rec["checks"]) == 8
