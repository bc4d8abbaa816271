"""CPU test double with EdVerifyEngine's verify / key-store interface,
answering with the C oracle (oracle/_build/libed25519_oracle.so).  Used ONLY
to test host-side logic (check order, exception mapping, batching, key-store
ownership, sharding) without a GPU; the product has no CPU path.  Plain
numpy + ctypes, so the Python 3.9 reference checks (tests/golden/) use it too.
`calls` counts verify launches (one per batch call)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_oracle():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libed25519_oracle.so"))
    lib.oracle_verify_detached.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.oracle_sign_open.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    return lib


class OracleEngine:
    def __init__(self, lib=None):
        self.lib = lib or load_oracle()
        self.calls = 0
        self.keyed_calls = 0
        self.keys = []
        self.window = 10
        self.keys_generation = 0
        self.fail_keys_add = False

    def keys_reset(self):
        self.keys = []
        self.keys_generation += 1

    def keys_set_window(self, w):
        assert not self.keys
        self.window = w

    def keys_add(self, pk32):
        if self.fail_keys_add:
            raise RuntimeError("edverify error -3: key store allocation failed (test)")
        first = len(self.keys)
        self.keys.extend(bytes(r) for r in np.asarray(pk32, np.uint8).reshape(-1, 32))
        return first

    def keys_set(self, first_id, pk32):
        rows = [bytes(r) for r in np.asarray(pk32, np.uint8).reshape(-1, 32)]
        assert first_id + len(rows) <= len(self.keys)
        self.keys[first_id:first_id + len(rows)] = rows

    def keys_count(self):
        return len(self.keys)

    def verify_batch_keyed(self, sig64, key_idx, msgs, msg_off):
        self.keyed_calls += 1
        pk = np.frombuffer(b"".join(self.keys[int(k)] if int(k) < len(self.keys) else b"\0" * 32
                                    for k in key_idx), np.uint8).reshape(-1, 32)
        ok = self._verify(sig64, pk, msgs, msg_off)
        self.calls += 1
        return ok & np.array([int(k) < len(self.keys) for k in key_idx], bool)

    def sign_open_batch(self, sm, sm_off, pk32):
        self.calls += 1
        sm = bytes(sm) if not isinstance(sm, np.ndarray) else sm.tobytes()
        pk32 = np.asarray(pk32, dtype=np.uint8).reshape(-1, 32) if not isinstance(pk32, list) else \
            np.frombuffer(b"".join(pk32), np.uint8).reshape(-1, 32)
        off = [int(x) for x in sm_off]
        return np.array([self.lib.oracle_sign_open(sm[off[i]:off[i + 1]], off[i + 1] - off[i], pk32[i].tobytes()) == 0
                         for i in range(len(off) - 1)], dtype=bool)

    def verify_batch(self, sig64, pk32, msgs, msg_off):
        self.calls += 1
        return self._verify(sig64, pk32, msgs, msg_off)

    def _verify(self, sig64, pk32, msgs, msg_off):
        msgs = bytes(msgs) if not isinstance(msgs, np.ndarray) else msgs.tobytes()
        sig64 = np.asarray(sig64, np.uint8).reshape(-1, 64)
        pk32 = np.asarray(pk32, np.uint8).reshape(-1, 32)
        off = [int(x) for x in msg_off]
        return np.array([self.lib.oracle_verify_detached(sig64[i].tobytes(), msgs[off[i]:off[i + 1]],
                                                         off[i + 1] - off[i], pk32[i].tobytes()) == 0
                         for i in range(len(off) - 1)], dtype=bool)
