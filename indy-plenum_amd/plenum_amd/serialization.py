"""Canonical bytes-to-sign of a Plenum message.

Restates common/serializers/signing_serializer.py:35-91 (SigningSerializer.serialize)
and common/serializers/serialization.py:116-125 (serialize_msg_for_signing):
  str -> itself; dict -> sorted keys (top level minus topLevelKeysToIgnore),
  "k:v" joined by "|"; other iterables -> ","-joined; None -> ""; other
  acceptable scalars -> str(x) (bool -> "True", float -> Python repr);
  anything outside (str, int, float, list, dict, None) raises Exception
  ("invalid type found ...", plenum/common/error.py:9-16); UTF-8 encoded.
Pinned against the reference's own serializer by tests/golden/serializer_kat.json."""
from collections.abc import Iterable

acceptableTypes = (str, int, float, list, dict, type(None))


def _text(obj, top, path, ignore):
    """The signing text of obj.  top: obj is the message itself (only there are
    the ignored keys dropped); path: the dotted key path of obj, used in the
    error text and -- as the reference's does -- joined with each dict key, so a
    non-str key below the top level raises TypeError just as the reference's
    join does."""
    if not isinstance(obj, acceptableTypes):
        raise Exception("invalid type found {}: {}".format(path, obj))
    if isinstance(obj, str):
        return obj
    if isinstance(obj, dict):
        names = [k for k in obj.keys() if not top or k not in ignore]
        names.sort()
        fields = []
        for name in names:
            sub = ".".join([path, name]) if path else name
            head = str(name) + ":"
            fields.append(head + _text(obj[name], False, sub, ()))
        return "|".join(fields)
    if isinstance(obj, Iterable):  # a list: its items' texts, comma-separated, same path
        return ",".join([_text(item, False, path, ()) for item in obj])
    return "" if obj is None else str(obj)


class SigningSerializer:
    """The reference's serializer interface (serialize(obj, level, objname,
    topLevelKeysToIgnore, toBytes)) over _text."""

    def serialize(self, obj, level=0, objname=None, topLevelKeysToIgnore=None, toBytes=True):
        text = _text(obj, level == 0, objname, topLevelKeysToIgnore or [])
        return text.encode("utf-8") if toBytes else text


signing_serializer = SigningSerializer()


try:  # native fast path (csrc/hostpack.cpp): exact bytes or None -> this module's code
    from . import _hostpack
except ImportError:  # pragma: no cover - built by __graft_entry__.build() / make
    _hostpack = None


def serialize_msg_for_signing(msg, topLevelKeysToIgnore=None):
    if _hostpack is not None:
        r = _hostpack.serialize_for_signing(msg, topLevelKeysToIgnore)
        if r is not None:
            return r
    return signing_serializer.serialize(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)
