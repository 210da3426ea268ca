"""base58 (base58==1.0.0 semantics) and SigningSerializer restatements, pinned
by the reference's own fixtures and by outputs of the reference's
SigningSerializer (tests/golden/serializer_golden.json)."""
import json
import os
import random

import pytest

import kats
from indy_plenum_amd import base58
from indy_plenum_amd.signing_serializer import serialize_msg_for_signing

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_did_expansion_fixture():
    # plenum/test/common/test_verifier.py:19-21
    v = base58.b58encode(base58.b58decode(kats.SAMPLE_IDENTIFIER) +
                         base58.b58decode(kats.SAMPLE_ABBR_VERKEY[1:])).decode()
    assert v == kats.EXPECTED_VERKEY
    # plenum/test/common/test_signers.py:36-43
    c = base58.b58encode(base58.b58decode(kats.KAT2_IDR) + base58.b58decode(kats.KAT2_ABBR_VERKEY[1:])).decode()
    assert c == kats.KAT2_CRYPTONYM


def test_roundtrip_and_leading_zeros():
    r = random.Random(1)
    for n in range(0, 70):
        for lead in (0, 1, 3):
            b = b"\0" * lead + bytes(r.getrandbits(8) for _ in range(n))
            e = base58.b58encode(b)
            assert isinstance(e, bytes)
            assert base58.b58decode(e) == b
            assert base58.b58decode(e.decode()) == b
    assert base58.b58encode(b"") == b""
    assert base58.b58decode("") == b""
    assert base58.b58decode("1") == b"\0"
    assert base58.b58decode("111") == b"\0\0\0"
    assert base58.b58decode("5Q ") == base58.b58decode("5Q")  # trailing whitespace stripped


@pytest.mark.parametrize("bad", ["0", "O", "I", "l", "abc+", "é"])
def test_invalid_characters_raise_value_error(bad):
    with pytest.raises(ValueError):
        base58.b58decode(bad)


def test_type_errors():
    with pytest.raises((TypeError, AttributeError)):
        base58.b58decode(None)
    with pytest.raises(TypeError):
        base58.b58encode(12)


def test_signing_serializer_matches_reference_outputs():
    with open(os.path.join(GOLDEN, "serializer_golden.json")) as f:
        rows = json.load(f)["cases"]
    assert len(rows) >= 90
    for row in rows:
        got = serialize_msg_for_signing(row["msg"], topLevelKeysToIgnore=row["ignore"])
        assert got == row["ser"].encode("utf-8")


def test_signing_serializer_rules():
    assert serialize_msg_for_signing({2: 'b', 1: 'a'}) == b'1:a|2:b'
    assert serialize_msg_for_signing({'x': [1, 2, 3]}) == b'x:1,2,3'
    assert serialize_msg_for_signing({'x': None, 'y': True, 'z': 1.5}) == b'x:|y:True|z:1.5'
    assert serialize_msg_for_signing({'a': 1, 'b': 2}, topLevelKeysToIgnore=['b']) == b'a:1'
    assert serialize_msg_for_signing({'a': {'b': 1, 'c': 2}}, topLevelKeysToIgnore=['b']) == b'a:b:1|c:2'
    with pytest.raises(Exception):
        serialize_msg_for_signing({'a': (1, 2)})  # tuples are not acceptable types


def test_signing_state_matches_request_semantics():
    """digest.signing_state restates Request.signingState (request.py:77-87) and
    Request.identifier (request.py:110-112, 124-126) for request dicts."""
    from indy_plenum_amd import digest
    req = {"identifier": "L5AD5g65TDQr1PPHHRoiGf", "reqId": 1513945121191691, "protocolVersion": 1,
           "operation": {"dest": "GEzcdDLhCpGCYRHW82kjHd", "type": "1"}, "signature": "xyz"}
    assert digest.signing_state(req) == {"identifier": "L5AD5g65TDQr1PPHHRoiGf", "reqId": 1513945121191691,
                                         "operation": {"dest": "GEzcdDLhCpGCYRHW82kjHd", "type": "1"},
                                         "protocolVersion": 1}
    multi = {"reqId": 5, "operation": {"type": "1"}, "signatures": {"b": "s1", "a": "s2"}}
    assert digest.signing_state(multi) == {"identifier": "a,b", "reqId": 5, "operation": {"type": "1"}}
    assert digest.signing_state(multi, identifier="z")["identifier"] == "z"
    import pytest
    with pytest.raises(AttributeError):
        digest.signing_state({"reqId": 1, "operation": {}})
