"""Base58 (Bitcoin alphabet) with the semantics of base58==1.0.0, the version
the reference pins (setup.py:47) and calls on the hot path
(plenum/server/client_authn.py:94, plenum/common/verifier.py:29-50).

b58encode returns bytes; b58decode accepts str or bytes, strips trailing
whitespace, maps leading '1's to zero bytes and raises ValueError on a
character outside the alphabet.  (The package is not installed in this image;
this is a restatement, pinned by tests/test_base58.py against the reference's
own DID fixtures.)
"""

alphabet = b'123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz'
_INDEX = {c: i for i, c in enumerate(alphabet)}


def scrub_input(v):
    if isinstance(v, str) and not isinstance(v, bytes):
        v = v.encode('ascii')
    if not isinstance(v, bytes):
        raise TypeError("a bytes-like object is required (also str), not '%s'" % type(v).__name__)
    return v


def b58encode_int(i, default_one=True):
    if not i and default_one:
        return alphabet[0:1]
    string = b""
    while i:
        i, idx = divmod(i, 58)
        string = alphabet[idx:idx + 1] + string
    return string


try:  # native fast path (csrc/edv_host.cpp, row f-1); NotImplemented -> the restatement below
    from . import _edvhost as _native
except ImportError:  # pragma: no cover - the in-tree build always provides it
    _native = None


def b58encode(v):
    if _native is not None:
        r = _native.b58encode(v)
        if r is not NotImplemented:
            return r
    return _b58encode_py(v)


def b58decode(v):
    if _native is not None:
        r = _native.b58decode(v)
        if r is not NotImplemented:
            return r
    return _b58decode_py(v)


def _b58encode_py(v):
    v = scrub_input(v)
    n_pad = len(v)
    v = v.lstrip(b'\0')
    n_pad -= len(v)
    acc = int.from_bytes(v, 'big') if v else 0
    return alphabet[0:1] * n_pad + b58encode_int(acc, default_one=False)


def b58decode_int(v):
    v = v.rstrip()
    v = scrub_input(v)
    decimal = 0
    for char in v:
        try:
            decimal = decimal * 58 + _INDEX[char]
        except KeyError:
            raise ValueError("Invalid character {!r}".format(chr(char))) from None
    return decimal


def _b58decode_py(v):
    v = v.rstrip()
    v = scrub_input(v)
    origlen = len(v)
    v = v.lstrip(alphabet[0:1])
    newlen = len(v)
    acc = b58decode_int(v)
    body = acc.to_bytes((acc.bit_length() + 7) // 8, 'big') if acc else b''
    return b'\0' * (origlen - newlen) + body
