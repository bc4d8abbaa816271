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


def _error(msg):
    raise Exception(msg)


class SigningSerializer:
    def serialize(self, obj, level=0, objname=None, topLevelKeysToIgnore=None, toBytes=True):
        res = None
        if not isinstance(obj, acceptableTypes):
            _error("invalid type found {}: {}".format(objname, obj))
        elif isinstance(obj, str):
            res = obj
        elif isinstance(obj, dict):
            if level > 0:
                keys = list(obj.keys())
            else:
                topLevelKeysToIgnore = topLevelKeysToIgnore or []
                keys = [k for k in obj.keys() if k not in topLevelKeysToIgnore]
            keys.sort()
            strs = []
            for k in keys:
                onm = ".".join([objname, k]) if objname else k
                strs.append(str(k) + ":" + self.serialize(obj[k], level + 1, onm, toBytes=False))
            res = "|".join(strs)
        elif isinstance(obj, Iterable):
            res = ",".join(self.serialize(o, level + 1, objname, toBytes=False) for o in obj)
        elif obj is None:
            res = ""
        else:
            res = str(obj)
        if not toBytes:
            return res
        return res.encode("utf-8")


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
