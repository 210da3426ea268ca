"""Canonical signing bytes M of a client request.

Restates common/serializers/signing_serializer.py:31-92 and
serialize_msg_for_signing (common/serializers/serialization.py:23-32): dict keys
sorted and joined as "k:v" with "|", the ignore list applied at the top level
only, lists joined with ",", None -> "", everything else str(x); UTF-8 out.
Pinned by tests/golden/serializer_golden.json, produced by the reference's own
SigningSerializer (tests/golden/make_serializer_golden.py).
"""
from collections.abc import Iterable

acceptableTypes = (str, int, float, list, dict, type(None))


def error(msg, exc_type=Exception):
    raise exc_type(msg)


class SigningSerializer:
    def serialize(self, obj, level=0, objname=None, topLevelKeysToIgnore=None, toBytes=True):
        res = None
        if not isinstance(obj, acceptableTypes):
            error("invalid type found {}: {}".format(objname, obj))
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
        return res.encode('utf-8')


signing_serializer = SigningSerializer()

try:  # native fast path (csrc/edv_host.cpp, row f-1); NotImplemented -> the class above
    from . import _edvhost as _native
except ImportError:  # pragma: no cover - the in-tree build always provides it
    _native = None


def serialize_msg_for_signing(msg, topLevelKeysToIgnore=None):
    if _native is not None:
        r = _native.serialize(msg, topLevelKeysToIgnore)
        if r is not NotImplemented:
            return r
    return signing_serializer.serialize(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)
