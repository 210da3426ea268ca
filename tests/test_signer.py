"""Row f-4 (batch signer) parity: libsodium 1.0.18 crypto_sign_seed_keypair +
crypto_sign_detached outputs (tests/golden/sign_golden.bin, made by
tests/golden/make_sign_golden.py; RFC 8032 section 7.1 vectors 1-3 included and
checked against libsodium there) reproduced byte for byte by

  * hc_sign_batch: the kernel's own sign_one (edv_verify_core.h) compiled for the
    CPU (libedv_hostcheck.so, test harness), and the oracle's signer (CPU);
  * edv_sign_batch_dev: the gfx950 kernel (GPU test).

Reference signing path: stp_core/crypto/nacl_wrappers.py:162-176 (SigningKey.sign
-> libnacl.crypto_sign), plenum/common/signer_did.py:122-129 (DidSigner.sign).
"""
import ctypes

import numpy as np
import pytest

import golden_io
import hostcheck_lib
import oracle_lib as orc


@pytest.fixture(scope="module")
def vectors():
    v = golden_io.load_sign_golden()
    assert len(v) > 600
    return v


def test_rfc8032_vectors_present(vectors):
    pks = {r[2].hex() for r in vectors}
    assert "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a" in pks
    assert "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025" in pks


def test_kernel_signer_on_cpu_matches_libsodium(vectors):
    lib = hostcheck_lib.load()
    lib.hc_sign_batch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    seeds, msgs, off = golden_io.pack_sign_batch(vectors)
    n = len(vectors)
    s = np.frombuffer(seeds, np.uint8)
    m = np.frombuffer(msgs + b"\0" * 16, np.uint8)
    pks, sigs = np.zeros(32 * n, np.uint8), np.zeros(64 * n, np.uint8)
    assert lib.hc_sign_batch(s.ctypes.data, m.ctypes.data, off.ctypes.data, n, pks.ctypes.data, sigs.ctypes.data) == 0
    bad = [i for i, r in enumerate(vectors) if pks[32 * i:32 * i + 32].tobytes() != r[2]
           or sigs[64 * i:64 * i + 64].tobytes() != r[3]]
    assert bad == []


def test_oracle_signer_matches_libsodium(vectors):
    for seed, msg, pk, sig in vectors[:200]:
        opk, osk = orc.keypair(seed)
        assert opk == pk
        assert orc.sign(msg, osk) == sig
