"""DID verkey resolution, restated from plenum/common/verifier.py:21-46
(DidVerifier) and the key half of stp_core/crypto/nacl_wrappers.py:62-79,
216-230 (Verifier/VerifyKey construction).

Instead of wrapping a libnacl key, DidVerifier resolves to the raw 32-byte
Ed25519 public key that the GPU batch verifies against; verification itself is
done in batches by the engine (client_authn.py).  Resolution is deterministic,
so resolved keys (or the exception resolution raises) are cached per
(verkey, identifier) -- SURVEY.md 7 'Host-side Python is the real bottleneck'.
"""
import binascii
import copy
from collections import OrderedDict

from .base58 import b58decode, b58encode
from .exceptions import InvalidKey

PUBLICKEYBYTES = 32


def raw_verify_key(key):
    """nacl_wrappers.Verifier(key) key handling: a falsy key -> None (every
    verify then fails, nacl_wrappers.py:237-238); a 32-byte key is raw;
    anything else is hex-decoded (HexEncoder, encoding.py:22-23) and must then
    be 32 bytes (VerifyKey, nacl_wrappers.py:75-79) -- else ValueError."""
    if not key:
        return None
    if len(key) != PUBLICKEYBYTES:
        key = binascii.unhexlify(key)
    if len(key) != PUBLICKEYBYTES:
        raise ValueError("The key must be exactly %s bytes long" % PUBLICKEYBYTES)
    return bytes(key)


class Verifier:
    def verify(self, sig, msg) -> bool:
        raise NotImplementedError


class DidVerifier(Verifier):
    """Same construction semantics as the reference DidVerifier:
    cryptonym fallback when the identifier is 32 bytes and no verkey is given,
    '~'-abbreviated verkey expansion, InvalidKey (from the cause) when the
    resolved verkey is not a usable key.  `.key` is the raw public key (or
    None); `.verify(sig, msg)` checks one signature through `engine` with
    crypto_sign_open semantics."""

    def __init__(self, verkey, identifier=None, engine=None):
        _verkey = verkey
        self._verkey = None
        self.key = None
        self._engine = engine
        if identifier:
            rawIdr = b58decode(identifier)
            if len(rawIdr) == 32 and not verkey:  # assume cryptonym
                verkey = identifier
            assert verkey, 'verkey must be provided'
            if verkey[0] == '~':  # abbreviated
                verkey = b58encode(b58decode(identifier) + b58decode(verkey[1:]))
        try:
            self.verkey = verkey
        except Exception as ex:
            raise InvalidKey("verkey {}".format(_verkey)) from ex

    @property
    def verkey(self):
        return self._verkey

    @verkey.setter
    def verkey(self, value):
        self._verkey = value
        self.key = raw_verify_key(b58decode(value))

    def verify(self, sig, msg) -> bool:
        if not self.key:
            return False
        if self._engine is None:
            raise RuntimeError("DidVerifier.verify needs an EdVerifyEngine")
        return bool(self._engine.sign_open_batch(bytes(sig) + bytes(msg), [0, len(sig) + len(msg)],
                                                 [self.key])[0])


class VerkeyCache:
    """LRU of (verkey, identifier) -> raw key bytes | None | the exception
    DidVerifier construction raised (re-raised verbatim on a hit)."""

    def __init__(self, maxsize=1 << 20):
        self.maxsize = maxsize
        self._d = OrderedDict()

    def resolve(self, verkey, identifier):
        k = (verkey, identifier)
        hit = self._d.get(k)
        if hit is not None:
            self._d.move_to_end(k)
            kind, val = hit
            if kind == "exc":
                ex = copy.copy(val)
                ex.__cause__ = val.__cause__
                raise ex
            return val
        try:
            key = DidVerifier(verkey, identifier=identifier).key
            self._d[k] = ("key", key)
        except Exception as ex:
            self._d[k] = ("exc", ex)
            if len(self._d) > self.maxsize:
                self._d.popitem(last=False)
            raise
        if len(self._d) > self.maxsize:
            self._d.popitem(last=False)
        return key

    def clear(self):
        self._d.clear()
