"""Shared fixtures.  `-m gpu` tests need an MI355X (they run on the GPU box);
everything else runs on a CPU.  The oracle (oracle/_build) and the host-built
kernel arithmetic (libedv_hostcheck.so) are test infrastructure only."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "indy-plenum_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


def _ensure_built(path, make_dir):
    if not os.path.exists(path):
        subprocess.check_call(["make", "-j8"], cwd=make_dir)
    return path


@pytest.fixture(scope="session")
def oracle():
    lib = ctypes.CDLL(_ensure_built(os.path.join(ROOT, "oracle", "_build", "libed25519_oracle.so"),
                                    os.path.join(ROOT, "oracle")))
    lib.oracle_verify_detached.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.oracle_sign_open.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    return lib


@pytest.fixture(scope="session")
def hostcheck():
    path = os.path.join(PKG, "libedv_hostcheck.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "libedv_hostcheck.so"], cwd=PKG)
    return ctypes.CDLL(path)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name))


def items_of(d):
    """(sig, pk, msg, expect) tuples of a golden npz."""
    off = d["off"]
    return [(d["sig"][i].tobytes(), d["pk"][i].tobytes(), d["msgs"][int(off[i]):int(off[i + 1])].tobytes(),
             bool(d["expect"][i])) for i in range(len(d["expect"]))]


from engine_double import OracleEngine  # noqa: E402


@pytest.fixture
def oracle_engine(oracle):
    return OracleEngine(oracle)


@pytest.fixture(scope="session")
def gpu_engine():
    from plenum_amd import EdVerifyEngine
    eng = EdVerifyEngine(0)
    yield eng
    eng.close()


@pytest.fixture(autouse=True)
def _gpu_engine_options_restored(request):
    """Every test that uses the session's GPU engine leaves it with the default options
    (edv_options), however it ends: the next test starts from a fresh context's modes."""
    yield
    if "gpu_engine" in request.fixturenames:
        eng = request.getfixturevalue("gpu_engine")
        from plenum_amd import EdVerifyEngine
        eng.set_options(**EdVerifyEngine.default_options())


def sodium():
    """libsodium 1.0.18 via ctypes if present (this container and the GPU
    box image have it); None otherwise."""
    for cand in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23"):
        try:
            lib = ctypes.CDLL(cand)
        except OSError:
            continue
        lib.sodium_init()
        lib.sodium_version_string.restype = ctypes.c_char_p
        return lib
    return None


def host_threads():
    """CPUs this process may use: affinity capped by a cgroup v2 quota (the GPU
    box shows 256 CPUs and grants 16)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(float(q) / float(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


@pytest.fixture(scope="session")
def sodium_verdicts():
    """verdicts(sig64[n,64], pk32[n,32], msgs, start[n], end[n]) -> bool[n]:
    libsodium 1.0.18's crypto_sign_verify_detached on every item, on all of
    this host's CPUs (oracle/cpu_baseline.c; test infrastructure) -- the
    full-batch parity check (about 2 s per 1M items on 16 threads)."""
    lib = ctypes.CDLL(_ensure_built(os.path.join(ROOT, "oracle", "_build", "libcpu_baseline.so"),
                                    os.path.join(ROOT, "oracle")))
    lib.cpu_baseline_sodium_version.restype = ctypes.c_char_p
    P = ctypes.c_void_p

    def verdicts(sig, pk, msgs, start, end):
        sig = np.ascontiguousarray(sig, np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8)
        msgs = np.ascontiguousarray(msgs, np.uint8)
        start = np.ascontiguousarray(start, np.uint64)
        end = np.ascontiguousarray(end, np.uint64)
        n = len(start)
        assert sig.shape == (n, 64) and pk.shape == (n, 32) and len(end) == n
        assert n == 0 or int(end.max()) <= len(msgs)
        ok = np.zeros(n, np.uint8)
        r = lib.cpu_baseline_verdicts_spans(P(sig.ctypes.data), P(pk.ctypes.data), P(msgs.ctypes.data),
                                            P(start.ctypes.data), P(end.ctypes.data), ctypes.c_uint64(n),
                                            host_threads(), P(ok.ctypes.data))
        assert r == 1, "libsodium not loadable (cpu_baseline_verdicts_spans -> %d)" % r
        assert lib.cpu_baseline_sodium_version().decode() == "1.0.18"
        return ok.astype(bool)
    return verdicts
