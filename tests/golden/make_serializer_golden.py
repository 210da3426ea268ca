#!/opt/conda/bin/python3.9
"""Generate tests/golden/serializer_golden.json by running the REFERENCE's own
SigningSerializer (common/serializers/signing_serializer.py) on a set of
request dicts.  Must run under /opt/conda/bin/python3.9 with
PYTHONPATH=/root/reference (the module needs collections.Iterable, gone in 3.10).
Only the outputs (data) are committed; nothing of the reference is copied.

Also records the reference's DID fixtures (plenum/test/common/test_verifier.py:6-8,
test_signers.py:36-43) expanded through base58 arithmetic done here with plain
integers, and the two signed-request KATs.
"""
import json
import os
import random
import sys

from common.serializers.signing_serializer import SigningSerializer  # reference module

_ss = SigningSerializer()


def serialize_msg_for_signing(msg, topLevelKeysToIgnore=None):
    # common/serializers/serialization.py:23-32 is exactly this call on its module-level
    # SigningSerializer; that module itself imports base58/msgpack, absent here.
    return _ss.serialize(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)

HERE = os.path.dirname(os.path.abspath(__file__))


def cases():
    r = random.Random(11)
    out = [
        {"identifier": "5rArie7XKukPCaEwq5XGQJnM9Fc5aZE3M9HAPVfMU2xC",
         "operation": {"amount": 62, "type": "buy"}, "reqId": 1499782864169193},
        {"identifier": "5rArie7XKukPCaEwq5XGQJnM9Fc5aZE3M9HAPVfMU2xC",
         "operation": {"amount": 62, "type": "buy"}, "reqId": 1499782864169193, "protocolVersion": 1},
        {"identifier": "L5AD5g65TDQr1PPHHRoiGf", "reqId": 1513945121191691, "protocolVersion": 1,
         "operation": {"dest": "GEzcdDLhCpGCYRHW82kjHd", "verkey": "~HmUWn928bnFT6Ephf65YXv", "role": "101",
                       "type": "1"}},
        {"a": 1, "b": [1, 2, {"c": None, "d": True}], "e": 1.5, "f": "", "g": {}, "h": []},
        {"nested": {"z": {"y": {"x": [1, [2, [3, "four"]]]}}}, "uni": "é中\U0001F600"},
        {"float": 0.1, "neg": -5, "big": 2**70, "bool": False, "none": None},
        {"signature": "sig", "signatures": {"x": "y"}, "fees": [1], "identifier": "id", "reqId": 1},
    ]
    alphabet = "abcXYZ019_:|,"
    for i in range(40):
        def rv(depth):
            t = r.randrange(7 if depth < 3 else 4)
            if t == 0:
                return "".join(r.choice(alphabet) for _ in range(r.randrange(8)))
            if t == 1:
                return r.randrange(-10**6, 10**6)
            if t == 2:
                return None
            if t == 3:
                return r.choice([True, False, 3.25, -0.5, 1e-7])
            if t == 4:
                return [rv(depth + 1) for _ in range(r.randrange(4))]
            return {"k" + str(r.randrange(20)): rv(depth + 1) for _ in range(r.randrange(4))}
        out.append({"identifier": "idr" + str(i), "reqId": r.randrange(10**16),
                    "operation": {"type": r.choice(["0", "1", "3", "101"]), "payload": rv(0)},
                    "extra": rv(0)})
    return out


def main():
    rows = []
    for c in cases():
        rows.append({"msg": c, "ignore": None, "ser": serialize_msg_for_signing(c).decode("utf-8")})
        rows.append({"msg": c, "ignore": ["signature", "signatures"],
                     "ser": serialize_msg_for_signing(c, topLevelKeysToIgnore=["signature", "signatures"]).decode()})
    with open(os.path.join(HERE, "serializer_golden.json"), "w") as f:
        json.dump({"generated_with": "reference common.serializers.signing_serializer.SigningSerializer.serialize "
                                     "(python %s)" % sys.version.split()[0], "cases": rows}, f, indent=1,
                  ensure_ascii=False)
    print(len(rows), "serializer cases")


if __name__ == "__main__":
    main()
