"""GPU BLS multi-signatures for Plenum's COMMIT / state-proof path (SURVEY
§8(f)4): the drop-in for crypto/bls/indy_crypto/bls_crypto_indy_crypto.py.

Same classes and methods as the reference module, over the HIP library
(edv_bls_*, csrc/bls.hip) instead of indy-crypto 0.1.6:
  BlsGroupParamsLoaderGpu.load_group_params      (:11-16, the same generator)
  BlsCryptoVerifierGpu.verify_sig                (:59-70)
  BlsCryptoVerifierGpu.verify_multi_sig          (:72-84)
  BlsCryptoVerifierGpu.create_multi_sig          (:86-90)
  BlsCryptoSignerGpu.generate_keys / sign        (:93-117)
plus batch forms (verify_sig_batch, verify_multi_sig_batch) for the callers
that hold many checks at once (the COMMITs of a 3PC batch,
plenum/bls/bls_bft_replica_plenum.py:150-170).  String handling follows
IndyCryptoBlsUtils (:19-55): base58, None for undecodable values or lengths
other than 32 / 128 (then the check is False).

Parity: the generator literal pins the curve, twist and G2 encoding; the G1
encoding, H(m) and the key derivation from a seed are restated from
indy-crypto/AMCL, which is absent here (parity unpinned; DESIGN.md,
oracle/bls_bn254_oracle.py).  A 128-byte value of the wrong group decodes to
the point at infinity as in AMCL (no exception).
When the reference package is importable the classes derive from its
crypto.bls.bls_crypto abstract bases."""
import hashlib
import logging
import os

import numpy as np

from .base58 import b58decode, b58encode
from .engine import EdVerifyEngine, pack_messages

try:
    from crypto.bls.bls_crypto import BlsCryptoSigner, BlsCryptoVerifier, BlsGroupParamsLoader, GroupParams
    REFERENCE = True
except Exception:
    from abc import ABCMeta
    from collections import namedtuple

    REFERENCE = False
    GroupParams = namedtuple("GroupParams", "group_name, g")

    class BlsGroupParamsLoader(metaclass=ABCMeta):
        pass

    class BlsCryptoSigner(metaclass=ABCMeta):
        def __init__(self, sk, pk, params):
            assert sk
            assert pk
            self._sk = sk
            self.pk = pk
            self._group_params = params

    class BlsCryptoVerifier(metaclass=ABCMeta):
        pass

logger = logging.getLogger(__name__)

# bls_crypto_indy_crypto.py:14-15
GENERATOR = ("3LHpUjiyFC2q2hD7MnwwNmVXiuaFbQx2XkAFJWzswCjgN1utjsCeLzHsKk1nJvFEaS4fcrUmVAkdhtPCYbrVyATZcmzwJReTcJqwqBCPTmT"
             "Q9uWPwz6rEncKb2pYYYFcdHa8N17HzVyTqKfgPi4X9pMetfT3A5xCHq54R2pDNYWVLDX")
# BN254 group order r (AMCL BN254: 36x^4 + 36x^3 + 18x^2 + 6x + 1, x = -0x4080000000000001)
_X = -0x4080000000000001
ORDER = 36 * _X**4 + 36 * _X**3 + 18 * _X**2 + 6 * _X + 1

_shared_engine = None


def _engine(engine):
    global _shared_engine
    if engine is not None:
        return engine
    if _shared_engine is None:
        _shared_engine = EdVerifyEngine(0)
    return _shared_engine


class BlsGroupParamsLoaderGpu(BlsGroupParamsLoader):
    def load_group_params(self):
        return GroupParams("generator", GENERATOR)


class GpuBlsUtils:
    """IndyCryptoBlsUtils (bls_crypto_indy_crypto.py:19-55) over raw bytes."""
    SEED_LEN = 48

    @staticmethod
    def bls_to_str(v):
        return b58encode(bytes(v))

    @staticmethod
    def bls_from_str(v):
        try:
            bts = b58decode(v)
        except ValueError:
            logger.error("BLS: value %s can not be decoded to base58", v)
            return None
        if len(bts) not in (32, 128):  # the reference's length guard
            return None
        return bts

    @staticmethod
    def prepare_seed(seed):
        seed_bytes = None
        if isinstance(seed, str):
            seed_bytes = seed.encode()
        if isinstance(seed, (bytes, bytearray)):
            seed_bytes = bytes(seed)
        if seed_bytes:
            if len(seed_bytes) < GpuBlsUtils.SEED_LEN:
                seed_bytes += b"0" * (GpuBlsUtils.SEED_LEN - len(seed_bytes))
            assert len(seed_bytes) == GpuBlsUtils.SEED_LEN
        return seed_bytes


def _point128(bts):
    """A decoded value used as a group element: 128 bytes, else None (a 32-byte
    value is a scalar, never a point)."""
    return bts if bts is not None and len(bts) == 128 else None


class BlsCryptoVerifierGpu(BlsCryptoVerifier):
    def __init__(self, params, engine=None):
        self._gen = _point128(GpuBlsUtils.bls_from_str(params.g))
        if self._gen is None:
            raise ValueError("BLS generator must be a 128-byte base58 G2 point")
        self._engine = engine

    @property
    def engine(self):
        self._engine = _engine(self._engine)
        return self._engine

    # ---- batch forms: one GPU launch for many checks
    def verify_sig_batch(self, items):
        """items: [(signature: str, message: bytes, pk: str)] -> [bool]."""
        return self._verify([(s, m, [pk]) for s, m, pk in items], multi=False)

    def verify_multi_sig_batch(self, items):
        """items: [(signature: str, message: bytes, pks: [str])] -> [bool]."""
        return self._verify(items, multi=True)

    def _verify(self, items, multi):
        out = [False] * len(items)
        sigs, msgs, vks, vk_off, idx = [], [], [], [0], []
        for i, (sig, msg, pks) in enumerate(items):
            s = _point128(GpuBlsUtils.bls_from_str(sig))
            keys = [_point128(GpuBlsUtils.bls_from_str(p)) for p in pks]
            if s is None or any(k is None for k in keys):
                continue  # bls_from_str returned None: False (:61-66, :73-80)
            if not keys:
                continue  # no verkeys: the sum is infinity, never verifies (bn254.h bls_check)
            sigs.append(s)
            msgs.append(bytes(message_bytes(msg)))
            vks.extend(keys)
            vk_off.append(len(vks))
            idx.append(i)
        if not idx:
            return out
        buf, off = pack_messages(msgs)
        ok = self.engine.bls_verify_batch(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 128), buf, off,
                                          np.frombuffer(b"".join(vks), np.uint8).reshape(-1, 128) if vks
                                          else np.zeros((0, 128), np.uint8),
                                          np.frombuffer(self._gen, np.uint8),
                                          vk_off=np.asarray(vk_off, np.uint64) if multi else None)
        for j, i in enumerate(idx):
            out[i] = bool(ok[j])
        return out

    # ---- the reference interface
    def verify_sig(self, signature, message, pk):
        return self.verify_sig_batch([(signature, message, pk)])[0]

    def verify_multi_sig(self, signature, message, pks):
        return self.verify_multi_sig_batch([(signature, message, list(pks))])[0]

    def create_multi_sig(self, signatures):
        sigs = [_point128(GpuBlsUtils.bls_from_str(s)) for s in signatures]
        if any(s is None for s in sigs):
            raise ValueError("BLS: a signature is not a 128-byte base58 G1 point")
        out = self.engine.bls_aggregate(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 128),
                                        np.asarray([0, len(sigs)], np.uint64))
        return GpuBlsUtils.bls_to_str(out[0].tobytes())


def message_bytes(m):
    return m.encode() if isinstance(m, str) else m


class BlsCryptoSignerGpu(BlsCryptoSigner):
    def __init__(self, sk, pk, params, engine=None):
        super().__init__(sk, pk, params)
        self._sk_bytes = GpuBlsUtils.bls_from_str(sk)
        self._engine = engine

    @staticmethod
    def generate_keys(params, seed=None, engine=None):
        """(sk, vk) as base58 strings.  sk = SHA-256(seed) mod r (indy-crypto's
        AMCL RAND derivation is not restated: keys from a seed differ from the
        reference's; parity unpinned) or random without a seed."""
        seed = GpuBlsUtils.prepare_seed(seed)
        raw = hashlib.sha256(seed).digest() if seed else os.urandom(32)
        sk = int.from_bytes(raw, "big") % ORDER or 1
        skb = sk.to_bytes(32, "big")
        gen = _point128(GpuBlsUtils.bls_from_str(params.g))
        vk = _engine(engine).bls_keygen_batch(np.frombuffer(skb, np.uint8).reshape(1, 32),
                                              np.frombuffer(gen, np.uint8))[0].tobytes()
        return GpuBlsUtils.bls_to_str(skb), GpuBlsUtils.bls_to_str(vk)

    def sign(self, message):
        msg = bytes(message_bytes(message))
        buf, off = pack_messages([msg])
        sig = _engine(self._engine).bls_sign_batch(np.frombuffer(self._sk_bytes, np.uint8).reshape(1, 32), buf, off)
        return GpuBlsUtils.bls_to_str(sig[0].tobytes())


try:
    from crypto.bls.bls_factory import BlsFactoryCrypto as _FactoryBase
except Exception:  # standalone: the same template methods, no base class
    _FactoryBase = object


class BlsFactoryGpu(_FactoryBase):
    """BlsFactoryIndyCrypto (plenum/bls/bls_crypto_factory.py:31-52) with the
    GPU classes: a node built with this factory (create_default_bls_crypto_factory's
    replacement) signs and verifies COMMIT BLS signatures here."""

    def __init__(self, basedir=None, node_name=None, engine=None):
        self._basedir = basedir
        self._node_name = node_name
        self._engine = engine

    def _create_group_params_loader(self):
        return BlsGroupParamsLoaderGpu()

    def _get_bls_crypto_signer_class(self):
        return BlsCryptoSignerGpu

    def _create_bls_crypto_signer(self, sk, pk, group_params):
        return BlsCryptoSignerGpu(sk=sk, pk=pk, params=group_params, engine=self._engine)

    def _create_bls_crypto_verifier(self, group_params):
        return BlsCryptoVerifierGpu(group_params, engine=self._engine)

    def _create_key_manager(self, group_params):
        from plenum.bls.bls_key_manager_file import BlsKeyManagerFile
        assert self._basedir
        assert self._node_name
        return BlsKeyManagerFile(self._basedir, self._node_name)

    def create_bls_crypto_verifier(self):
        return self._create_bls_crypto_verifier(self._create_group_params_loader().load_group_params())
