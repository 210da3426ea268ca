"""The CPU oracle (oracle/ed25519_oracle.c) is pinned to libsodium 1.0.18's own
verdicts (tests/golden/, made by make_golden.py) before it is trusted."""
import hashlib
import random

import golden_io
import oracle_lib as orc


def test_golden_file_integrity(golden_meta):
    with open(golden_io.GOLDEN + "/ed25519_golden.bin", "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == golden_meta["sha256"]


def test_oracle_matches_libsodium_on_every_golden_case(golden, golden_meta):
    cats = golden_meta["categories"]
    bad = [(i, cats[c]) for i, (v, c, sig, pk, msg) in enumerate(golden) if orc.verify(sig, msg, pk) != bool(v)]
    assert bad == []
    # every category the survey lists is present
    present = {cats[c] for _v, c, *_ in golden}
    for need in ("valid", "flip_msg", "flip_r", "flip_s", "s_plus_kl", "small_order_a", "noncanon_a",
                 "offcurve_a", "small_order_r", "small_order_r_eq_holds", "mixed_order_a", "mixed_order_r",
                 "wrong_key", "empty_msg", "valid_long"):
        assert need in present


def test_mixed_order_a_accepts_iff_cofactorless_equation(golden, golden_meta):
    cat = golden_meta["categories"].index("mixed_order_a")
    vs = [v for v, c, *_ in golden if c == cat]
    assert 0 < sum(vs) < len(vs)  # some accepted (8 | h), most rejected


def test_oracle_open_positional_split():
    for sig, msg, pk, acc in golden_io.load_open_golden():
        assert orc.sign_open(sig + msg, pk) == bool(acc)


def test_oracle_signer_is_rfc8032_deterministic():
    # RFC 8032 section 7.1, TEST 1 (empty message)
    seed = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    pk, sk = orc.keypair(seed)
    assert pk.hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    sig = orc.sign(b"", sk)
    assert sig.hex() == ("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e06522490155"
                         "5fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert orc.verify(sig, b"", pk)


def test_oracle_sc_reduce_matches_python():
    L = 2**252 + 27742317777372353535851937790883648493
    r = random.Random(3)
    vals = [0, 1, L - 1, L, L + 1, 2**512 - 1, 8 * L, 2**252, 2**253] + [r.randrange(2**512) for _ in range(200)]
    for v in vals:
        assert int.from_bytes(orc.sc_reduce64(v.to_bytes(64, "little")), "little") == v % L
