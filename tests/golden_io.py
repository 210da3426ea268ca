"""Readers for the committed golden fixtures (tests/golden/)."""
import json
import os
import struct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_ed25519_golden():
    """-> list of (verdict, category, sig, pk, msg) from ed25519_golden.bin."""
    with open(os.path.join(GOLDEN, "ed25519_golden.bin"), "rb") as f:
        data = f.read()
    assert data[:8] == b"EDVGOLD1"
    (count,) = struct.unpack_from("<I", data, 8)
    pos = 12
    out = []
    for _ in range(count):
        v, c, _r, mlen = struct.unpack_from("<BBHI", data, pos)
        pos += 8
        sig = data[pos:pos + 64]
        pk = data[pos + 64:pos + 96]
        msg = data[pos + 96:pos + 96 + mlen]
        pos += 96 + mlen
        out.append((v, c, sig, pk, msg))
    assert pos == len(data)
    return out


def golden_meta():
    with open(os.path.join(GOLDEN, "ed25519_golden.json")) as f:
        return json.load(f)


def load_open_golden():
    with open(os.path.join(GOLDEN, "ed25519_open_golden.json")) as f:
        rows = json.load(f)["cases"]
    return [(bytes.fromhex(r["sig"]), bytes.fromhex(r["msg"]), bytes.fromhex(r["pk"]), r["accept"]) for r in rows]


def pack_batch(recs):
    """(sigs, pks, msgs, offsets) in the edv_verify_batch layout."""
    import numpy as np
    sigs = b"".join(r[2] for r in recs)
    pks = b"".join(r[3] for r in recs)
    msgs = b"".join(r[4] for r in recs)
    off = np.zeros(len(recs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r[4]) for r in recs])
    return sigs, pks, msgs, off


def load_serializer_golden():
    """Reference SigningSerializer outputs: [{"msg", "ignore", "ser"}] (make_serializer_golden.py)."""
    with open(os.path.join(GOLDEN, "serializer_golden.json")) as f:
        return json.load(f)["cases"]


def load_sign_golden():
    """libsodium signing vectors (make_sign_golden.py): list of (seed, msg, pk, sig)."""
    with open(os.path.join(GOLDEN, "sign_golden.bin"), "rb") as f:
        data = f.read()
    assert data[:8] == b"EDVSIGN1"
    (count,) = struct.unpack_from("<I", data, 8)
    pos, out = 12, []
    for _ in range(count):
        (mlen,) = struct.unpack_from("<I", data, pos)
        pos += 4
        seed, pk, sig = data[pos:pos + 32], data[pos + 32:pos + 64], data[pos + 64:pos + 128]
        msg = data[pos + 128:pos + 128 + mlen]
        pos += 128 + mlen
        out.append((seed, msg, pk, sig))
    assert pos == len(data)
    return out


def pack_sign_batch(recs):
    """(seeds, msgs, offsets) of signing vectors in the edv_sign_batch_dev layout."""
    import numpy as np
    seeds = b"".join(r[0] for r in recs)
    msgs = b"".join(r[1] for r in recs)
    off = np.zeros(len(recs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r[1]) for r in recs])
    return seeds, msgs, off
