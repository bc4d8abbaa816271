"""Base58 (Bitcoin alphabet) with the API and behaviour of the `base58`
package the reference pins (0.2.4, build-scripts/ubuntu-1604/build-3rd-parties.sh:43):
b58encode(bytes) -> str, b58decode(str | bytes) -> bytes, leading zero bytes
<-> leading '1's, ValueError on a character outside the alphabet.
Used by client_authn.py:89 (signature) and verifier.py:26-46 (identifier /
verkey expansion)."""

alphabet = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
_INDEX = {c: i for i, c in enumerate(alphabet)}


def b58encode(v):
    if not isinstance(v, (bytes, bytearray)):
        raise TypeError("a bytes-like object is required, not '%s'" % type(v).__name__)
    v = bytes(v)
    nz = len(v) - len(v.lstrip(b"\0"))
    acc = int.from_bytes(v, "big")
    out = []
    while acc > 0:
        acc, mod = divmod(acc, 58)
        out.append(alphabet[mod])
    return alphabet[0] * nz + "".join(reversed(out))


try:  # native fast path (csrc/hostpack.cpp): exact bytes, or None -> the code below
    from . import _hostpack
except ImportError:  # pragma: no cover
    _hostpack = None


def b58decode(v):
    if _hostpack is not None:
        r = _hostpack.b58decode(v)
        if r is not None:
            return r
    return b58decode_py(v)


def b58decode_py(v):
    if not isinstance(v, str):
        v = v.decode("ascii")
    nz = len(v) - len(v.lstrip(alphabet[0]))
    acc = 0
    for c in v[nz:]:
        try:
            acc = acc * 58 + _INDEX[c]
        except KeyError:
            raise ValueError("substring not found") from None
    body = acc.to_bytes((acc.bit_length() + 7) // 8, "big") if acc else b""
    return b"\0" * nz + body
