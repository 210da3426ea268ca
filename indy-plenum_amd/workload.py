"""Synthetic signed client requests for measurement and load generation
(SURVEY.md section 8d and row f-4), built without the oracle: messages are
NYM-shaped signing bytes made on the host with numpy, keys and signatures come
from the GPU batch signer (edv_sign_batch_dev), so a batch lands directly in
HBM, already resident, as the verify kernels consume it.

Message shape (config C2/C3, 256 bytes; C4: 200..4096 bytes):
  identifier:<32 hex>|operation:dest:<32 hex>|type:1|verkey:~<32 hex>|
  protocolVersion:2|reqId:<16 digits>|zpad:<filler>
i.e. the SigningSerializer layout of a NYM request (sorted 'k:v' joined by '|',
common/serializers/signing_serializer.py:58-92) padded with a filler field.

A batch is generated, uploaded and signed in slices of SLICE requests, so C3's
16,777,216 requests on one GPU never need more than one slice of host arrays at
a time.  A request's content depends on (seed, its slice's first index, its
place in the slice); C3's shards start on slice boundaries, so the 16M requests
are the same at every GPU count.
"""
import numpy as np

from . import edv

_HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
SLICE = 1 << 20
L_ORDER = 2**252 + 27742317777372353535851937790883648493
P_FIELD = 2**255 - 19

# damage kinds (the invalid requests of C2 --invalid, C3 and C4)
DAMAGE_KINDS = ("r_bit", "s_plus_l", "msg_byte", "key_bit",                 # C3: 4 kinds
                "small_order_r", "noncanonical_a", "small_order_a")          # C4 adds the strictness ones
# y = 1 (the identity, order 1) and y = p + 1 (a non-canonical encoding of y = 1)
_IDENTITY = (1).to_bytes(32, "little")
_NONCANON = (P_FIELD + 1).to_bytes(32, "little")
# an order-8 point encoding (libsodium's blocklist entry 26e8958f...)
_ORDER8 = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")


# byte -> its two ASCII hex digits as one little-endian uint16 (one gather per byte)
_HEX2 = (_HEX[np.arange(256) >> 4].astype(np.uint16) | (_HEX[np.arange(256) & 15].astype(np.uint16) << 8))
_AZ = (np.arange(256) % 26 + ord('a')).astype(np.uint8)   # random byte -> filler letter


def _hex_cols(b):
    """(n, k) uint8 -> (n, 2k) ASCII hex."""
    return np.ascontiguousarray(_HEX2[b]).view(np.uint8).reshape(b.shape[0], 2 * b.shape[1])


def _letters(rng, count):
    """count random filler letters a..z."""
    return _AZ[np.frombuffer(rng.bytes(count), dtype=np.uint8)]


def _decimal16(v):
    """uint64 values < 10^16 -> (n, 16) ASCII decimal digits, zero padded."""
    hi = (v // np.uint64(10 ** 8)).astype(np.uint32)
    lo = (v % np.uint64(10 ** 8)).astype(np.uint32)
    out = np.empty((len(v), 16), dtype=np.uint8)
    for d in range(8):
        out[:, 7 - d] = (hi % 10).astype(np.uint8) + ord('0')
        out[:, 15 - d] = (lo % 10).astype(np.uint8) + ord('0')
        hi //= 10
        lo //= 10
    return out


def message_lengths(n, seed=0x5EED2025, start=0, msg_len=256, var_range=None):
    """uint64 lengths of requests [start, start + n) (C4: uniform in var_range,
    drawn per SLICE-aligned block of global indices, so any sub-range agrees)."""
    if var_range is None:
        return np.full(n, msg_len, dtype=np.uint64)
    out = np.empty(n, dtype=np.uint64)
    lo = start
    while lo < start + n:
        blk = lo // SLICE
        hi = min(start + n, (blk + 1) * SLICE)
        lens = np.random.default_rng([seed, blk, 1]).integers(var_range[0], var_range[1] + 1, size=SLICE)
        out[lo - start:hi - start] = lens[lo - blk * SLICE:hi - blk * SLICE].astype(np.uint64)
        lo = hi
    return out


def nym_bodies(lens, seed, start):
    """Message bytes of requests [start, start + len(lens)) with the given
    lengths, concatenated (+64 bytes of tail slack)."""
    n = len(lens)
    rng = np.random.default_rng([seed, start, 2])
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    fields = rng.integers(0, 256, size=(n, 48), dtype=np.uint8)
    idh, dh, vh = _hex_cols(fields[:, :16]), _hex_cols(fields[:, 16:32]), _hex_cols(fields[:, 32:])
    # reqId = 1539648000000000 + global index, 16 decimal digits
    req = _decimal16(np.uint64(1539648000000000 + start) + np.arange(n, dtype=np.uint64))

    def lit(s):
        return np.broadcast_to(np.frombuffer(s, dtype=np.uint8), (n, len(s)))
    head = np.concatenate([lit(b"identifier:"), idh, lit(b"|operation:dest:"), dh, lit(b"|type:1|verkey:~"), vh,
                           lit(b"|protocolVersion:2|reqId:"), req, lit(b"|zpad:")], axis=1)
    hl = head.shape[1]
    msgs = np.zeros(int(off[-1]) + 64, dtype=np.uint8)
    if n and np.all(lens == lens[0]):
        m = int(lens[0])
        body = msgs[:n * m].reshape(n, m)
        body[:, :hl] = head
        body[:, hl:] = _letters(rng, n * (m - hl)).reshape(n, m - hl)
    elif n:
        msgs[:int(off[-1])] = _letters(rng, int(off[-1]))
        idx = off[:-1].astype(np.int64)[:, None] + np.arange(hl)[None, :]
        msgs[idx] = head
    return msgs, off


def nym_messages(n, seed=0x5EED2025, start=0, msg_len=256, var_range=None):
    """-> (msgs uint8 with 64 B of tail slack, offsets uint64[n+1]) for requests
    [start, start + n) (one slice's worth; DeviceBatch slices larger batches)."""
    return nym_bodies(message_lengths(n, seed, start, msg_len, var_range), seed, start)


def damage_positions(start, n, every):
    """Request indices i in [start, start + n) with i % every == every // 2 (a
    deterministic invalid set, ~1/every of the requests), relative to start."""
    if not every:
        return np.zeros(0, dtype=np.int64)
    first = (every // 2 - start) % every
    return np.arange(first, n, every, dtype=np.int64)


def damage_kind(global_idx, every, kinds):
    """Damage kind of damaged request i: the damaged requests cycle through the
    first `kinds` entries of DAMAGE_KINDS in index order."""
    return (np.asarray(global_idx, dtype=np.int64) // every) % kinds


def _add_l(s32):
    """(k, 32) little-endian scalars -> S + L (mod 2^256), vectorised."""
    sv = s32.copy().view(np.uint64)   # (k, 4) limbs
    carry = np.zeros(len(sv), dtype=np.uint64)
    for k in range(4):
        lw = np.uint64((L_ORDER >> (64 * k)) & (2**64 - 1))
        a = sv[:, k]
        t = a + lw
        c1 = (t < a).astype(np.uint64)
        t2 = t + carry
        c2 = (t2 < t).astype(np.uint64)
        sv[:, k] = t2
        carry = c1 | c2
    return sv.view(np.uint8).reshape(len(sv), 32)


class DeviceBatch:
    """A signed batch resident on one device: seeds -> (pks, sigs) signed on the GPU.

    damage_every=k corrupts the requests i % k == k // 2 (global index i =
    start + j), cycling over the first `damage_kinds` kinds of DAMAGE_KINDS (R
    bit flip, S + L malleation, message byte, key bit; with 7: small-order R,
    non-canonical A, small-order A), so the expected verdicts are known by
    construction: `expected()`.  keep_host: keep the host copy of the messages
    (host_copy(); default for batches up to 2^20 requests)."""

    def __init__(self, n, device=0, seed=0x5EED2025, start=0, msg_len=256, var_range=None, damage_every=0,
                 damage_kinds=4, keep_host=None):
        self.n, self.device, self.start = n, device, start
        self.damage_every, self.damage_kinds = damage_every, damage_kinds
        keep_host = n <= SLICE if keep_host is None else keep_host
        lens = message_lengths(n, seed, start, msg_len, var_range)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        self.host_off = off
        self.uniform = var_range is None
        self.d_msgs = edv.DeviceBuffer(int(off[-1]) + 64, device)
        self.d_off = edv.DeviceBuffer(off.nbytes, device)
        self.d_off.upload(off)
        self.d_pks = edv.DeviceBuffer(32 * n, device)
        self.d_sigs = edv.DeviceBuffer(64 * n, device)
        self.d_accept = edv.DeviceBuffer(max(n, 1), device)
        self._bits = None               # device bitmask buffer (accept_bits)
        self.bad = damage_positions(start, n, damage_every)
        host = np.empty(int(off[-1]) + 64, dtype=np.uint8) if keep_host else None
        d_seeds = edv.DeviceBuffer(32 * min(n, SLICE) + 64, device)
        for lo in range(0, n, SLICE):
            hi = min(n, lo + SLICE)
            m0, m1 = int(off[lo]), int(off[hi])
            msgs, _ = nym_bodies(lens[lo:hi], seed, start + lo)
            seeds = np.random.default_rng([seed, start + lo, 7]).integers(0, 256, size=32 * (hi - lo), dtype=np.uint8)
            edv._check(edv.lib().edv_h2d(device, self.d_msgs.ptr + m0, msgs.ctypes.data, msgs.nbytes))
            d_seeds.upload(seeds)
            # offsets are absolute; msg_base 0, slice [lo, hi)
            edv.sign_device(d_seeds.ptr, self.d_msgs.ptr, self.d_off.ptr + 8 * lo, hi - lo,
                            self.d_pks.ptr + 32 * lo, self.d_sigs.ptr + 64 * lo, device)
            sel = self.bad[(self.bad >= lo) & (self.bad < hi)]
            if sel.size:
                self._damage(lo, hi, sel, msgs, m0)
            if host is not None:
                host[m0:m1] = msgs[:m1 - m0]
        d_seeds.free()
        if host is not None:
            host[int(off[-1]):] = 0
        self.host_msgs = host
        # one SHA-512 block count for the whole batch: no length buckets needed (a
        # per-call hint; the device-wide mode stays untouched)
        self.flags = edv.FLAG_UNIFORM_LENGTH if self.uniform else 0

    def _damage(self, lo, hi, sel, msgs, m0):
        """Damage requests `sel` (batch-relative) of slice [lo, hi), vectorised
        (C3 damages 800k of 16M); msgs: the slice's host message bytes."""
        k = hi - lo
        sigs = self.d_sigs.download_at(64 * lo, 64 * k).reshape(k, 64).copy()
        pks = self.d_pks.download_at(32 * lo, 32 * k).reshape(k, 32).copy()
        kind = damage_kind(self.start + sel, self.damage_every, self.damage_kinds)
        rel = sel - lo
        by = [rel[kind == t] for t in range(len(DAMAGE_KINDS))]
        sigs[by[0], 5] ^= 0x10                                           # R bit
        if by[1].size:
            sigs[by[1], 32:] = _add_l(sigs[by[1], 32:])                  # S + L
        mo = (self.host_off[lo + by[2]] - self.host_off[lo]).astype(np.int64)
        msgs[mo + 3] ^= 0x01                                             # message byte
        pks[by[3], 9] ^= 0x04                                            # key bit
        sigs[by[4], :32] = np.frombuffer(_ORDER8, np.uint8)              # small-order R
        pks[by[5]] = np.frombuffer(_NONCANON, np.uint8)                  # non-canonical A (y = p + 1)
        pks[by[6]] = np.frombuffer(_IDENTITY, np.uint8)                  # small-order A (identity)
        h2d = edv.lib().edv_h2d
        edv._check(h2d(self.device, self.d_sigs.ptr + 64 * lo, sigs.ctypes.data, sigs.nbytes))
        edv._check(h2d(self.device, self.d_pks.ptr + 32 * lo, pks.ctypes.data, pks.nbytes))
        if by[2].size:
            m1 = int(self.host_off[hi])
            edv._check(h2d(self.device, self.d_msgs.ptr + m0, msgs.ctypes.data, m1 - m0))

    def expected(self):
        """The verdict bytes this batch must produce (1 except at the damaged positions)."""
        e = np.ones(self.n, dtype=np.uint8)
        e[self.bad] = 0
        return e

    def verify(self, stream=None):
        edv.verify_device(self.d_sigs.ptr, self.d_pks.ptr, self.d_msgs.ptr, self.d_off.ptr, self.n,
                          self.d_accept.ptr, self.device, stream=stream, flags=self.flags)

    def submit(self, extra_flags=0):
        """Pipelined verify (edv_verify_batch_dev_pipelined); results after edv.pipeline_sync.
        extra_flags: edv.FLAG_SPLIT_PREP runs the hash side beside the previous main kernel."""
        edv.verify_device_pipelined(self.d_sigs.ptr, self.d_pks.ptr, self.d_msgs.ptr, self.d_off.ptr, self.n,
                                    self.d_accept.ptr, self.device, flags=self.flags | extra_flags)

    def accept(self, out=None):
        """The verdict bytes (D2H), into `out` (a host slice of n bytes) if given."""
        if out is None:
            return self.d_accept.download(self.n)
        assert out.nbytes == self.n and out.flags.c_contiguous
        if self.n:
            edv._check(edv.lib().edv_d2h(self.device, out.ctypes.data, self.d_accept.ptr, self.n))
        return out

    def accept_bits(self):
        """The verdicts as a bitmask (packed on the device, ceil(n/8) bytes D2H):
        bit i % 8 of byte i / 8 = verdict i."""
        nb = (self.n + 7) // 8
        if self._bits is None:
            self._bits = edv.DeviceBuffer(max(nb, 1), self.device)
        edv.pack_bits_device(self.d_accept.ptr, self.n, self._bits.ptr, self.device)
        return self._bits.download(nb)

    def host_prefix(self, k):
        """(sigs, pks, msgs, off, expected) host arrays of the first k requests,
        read back from the device (the message bytes included, so it works for
        batches built with keep_host=False); offsets rebased to 0."""
        k = min(k, self.n)
        off = self.host_off[:k + 1] - self.host_off[0]
        mb = int(off[-1])
        msgs = np.zeros(mb + 64, np.uint8)
        msgs[:mb] = self.d_msgs.download_at(int(self.host_off[0]), mb)
        return (self.d_sigs.download_at(0, 64 * k), self.d_pks.download_at(0, 32 * k), msgs,
                np.ascontiguousarray(off), self.expected()[:k])

    def host_copy(self):
        """(sigs, pks, msgs, off) host arrays of this batch."""
        if self.host_msgs is None:
            raise ValueError("batch built with keep_host=False")
        return (self.d_sigs.download(64 * self.n), self.d_pks.download(32 * self.n), self.host_msgs, self.host_off)
