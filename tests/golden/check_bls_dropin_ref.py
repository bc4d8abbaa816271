"""BLS drop-in check against the REAL reference interface (container-side only):

    /opt/conda/bin/python3.9 tests/golden/check_bls_dropin_ref.py [--write]

Imports /root/reference's crypto.bls.bls_crypto (the abstract BlsCryptoSigner /
BlsCryptoVerifier / BlsGroupParamsLoader every Plenum BLS caller types against:
plenum/bls/bls_bft_replica_plenum.py:157,170,205, plenum/client/client.py:541)
before plenum_amd.bls, and asserts:
  1. the GPU classes derive from the reference's ABCs and implement every
     abstract method (they instantiate);
  2. the group parameters are the reference's (the generator literal of
     crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:14-15);
  3. over the oracle-backed BLS engine double (tests/engine_double.py; the
     GPU runs the same scenarios in tests/test_gpu_bls.py): the reference test
     scenarios of crypto/test/bls/indy_crypto/test_bls_crypto_indy_crypto.py
     (sign / verify own and other's key, multi-signature of two nodes, the
     invalid / short / long base58 values) give the reference's booleans.
With --write the summary goes to bls_dropin_ref_check.json."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import ref_standins as R  # noqa: E402

R.install()
import crypto.bls.bls_crypto as ref_bls  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from plenum_amd import bls as B  # noqa: E402
from plenum_amd.base58 import b58encode  # noqa: E402
from engine_double import OracleBlsEngine  # noqa: E402


def main():
    eng = OracleBlsEngine()
    assert B.REFERENCE, "plenum_amd.bls did not pick up the reference's crypto.bls.bls_crypto"
    assert issubclass(B.BlsCryptoVerifierGpu, ref_bls.BlsCryptoVerifier)
    assert issubclass(B.BlsCryptoSignerGpu, ref_bls.BlsCryptoSigner)
    assert issubclass(B.BlsGroupParamsLoaderGpu, ref_bls.BlsGroupParamsLoader)
    params = B.BlsGroupParamsLoaderGpu().load_group_params()
    assert isinstance(params, ref_bls.GroupParams) and params.group_name == "generator"
    ref_src = open(os.path.join(R.REF, "crypto", "bls", "indy_crypto", "bls_crypto_indy_crypto.py")).read()
    assert params.g in ref_src.replace('"\n        "', "")
    sk1, pk1 = B.BlsCryptoSignerGpu.generate_keys(params, "Node1", engine=eng)
    sk2, pk2 = B.BlsCryptoSignerGpu.generate_keys(params, "Node2", engine=eng)
    s1 = B.BlsCryptoSignerGpu(sk1, pk1, params, engine=eng)
    s2 = B.BlsCryptoSignerGpu(sk2, pk2, params, engine=eng)
    ver = B.BlsCryptoVerifierGpu(params, engine=eng)
    assert isinstance(ver, ref_bls.BlsCryptoVerifier) and isinstance(s1, ref_bls.BlsCryptoSigner)
    msg = b"Hello!"
    sig1, sig2 = s1.sign(msg), s2.sign(msg)
    checks = {
        "verify own key": ver.verify_sig(sig1, msg, pk1),
        "verify other key": not ver.verify_sig(sig1, msg, pk2),
        "multi two nodes": ver.verify_multi_sig(ver.create_multi_sig([sig1, sig2]), msg, [pk1, pk2]),
        "multi one key missing": not ver.verify_multi_sig(ver.create_multi_sig([sig1, sig2]), msg, [pk1]),
        "sig + b58('0')": not ver.verify_sig(sig1 + b58encode(b"0"), msg, pk1),
        "short sig": not ver.verify_sig(b58encode(b"1" * 10), msg, pk1),
        "long sig": not ver.verify_sig(b58encode(b"1" * 500), msg, pk1),
        "non-base58 pk": not ver.verify_sig(sig1, msg, "0OIl"),
    }
    summary = {"ok": all(checks.values()), "checks": checks, "engine_calls": eng.calls,
               "reference_abcs": ["BlsCryptoVerifier", "BlsCryptoSigner", "BlsGroupParamsLoader", "GroupParams"],
               "note": "over the oracle-backed BLS engine double; tests/test_gpu_bls.py runs the same on the GPU"}
    print(json.dumps(summary))
    if "--write" in sys.argv:
        with open(os.path.join(HERE, "bls_dropin_ref_check.json"), "w") as f:
            json.dump(summary, f, indent=1)
    return 0 if summary["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
