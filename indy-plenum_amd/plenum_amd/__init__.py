"""plenum_amd -- MI355X-native batched Ed25519 request authentication for
Hyperledger Plenum (drop-in for plenum/server/client_authn.py's authenticators)."""
from ._lib import EdVerifyError, EdVerifyUnavailable  # noqa: F401
from .engine import EdVerifyEngine, pack_messages, unpack_bits  # noqa: F401

__version__ = "0.1.0"
