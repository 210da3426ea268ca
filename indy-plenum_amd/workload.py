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
"""
import numpy as np

from . import edv

_HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)


def _hex_cols(b):
    """(n, k) uint8 -> (n, 2k) ASCII hex."""
    out = np.empty((b.shape[0], 2 * b.shape[1]), dtype=np.uint8)
    out[:, 0::2] = _HEX[b >> 4]
    out[:, 1::2] = _HEX[b & 15]
    return out


def nym_messages(n, seed=0x5EED2025, start=0, msg_len=256, var_range=None):
    """-> (msgs uint8 with 64 B of tail slack, offsets uint64[n+1])."""
    rng = np.random.default_rng([seed, start])
    if var_range is None:
        lens = np.full(n, msg_len, dtype=np.uint64)
    else:
        lens = rng.integers(var_range[0], var_range[1] + 1, size=n).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    fields = rng.integers(0, 256, size=(n, 48), dtype=np.uint8)
    idh, dh, vh = _hex_cols(fields[:, :16]), _hex_cols(fields[:, 16:32]), _hex_cols(fields[:, 32:])
    # reqId = 1539648000000000 + global index, 16 decimal digits (vectorised: C3 builds 16M)
    rid = np.uint64(1539648000000000 + start) + np.arange(n, dtype=np.uint64)
    req = np.empty((n, 16), dtype=np.uint8)
    for d in range(16):
        req[:, 15 - d] = (rid // np.uint64(10 ** d) % np.uint64(10)).astype(np.uint8) + ord('0')

    def lit(s):
        return np.broadcast_to(np.frombuffer(s, dtype=np.uint8), (n, len(s)))
    head = np.concatenate([lit(b"identifier:"), idh, lit(b"|operation:dest:"), dh, lit(b"|type:1|verkey:~"), vh,
                           lit(b"|protocolVersion:2|reqId:"), req, lit(b"|zpad:")], axis=1)
    hl = head.shape[1]
    msgs = np.zeros(int(off[-1]) + 64, dtype=np.uint8)
    if var_range is None:
        body = msgs[:n * msg_len].reshape(n, msg_len)
        body[:, :hl] = head
        body[:, hl:] = (rng.integers(0, 26, size=(n, msg_len - hl), dtype=np.uint8) + ord('a'))
    else:
        filler = (rng.integers(0, 26, size=int(off[-1]), dtype=np.uint8) + ord('a'))
        msgs[:int(off[-1])] = filler
        starts = off[:-1].astype(np.int64)
        idx = starts[:, None] + np.arange(hl)[None, :]
        msgs[idx] = head
    return msgs, off


def damage_positions(start, n, every):
    """Request indices i in [start, start + n) with i % every == every // 2 (a
    deterministic invalid set, ~1/every of the requests), relative to start."""
    if not every:
        return np.zeros(0, dtype=np.int64)
    first = (every // 2 - start) % every
    return np.arange(first, n, every, dtype=np.int64)


class DeviceBatch:
    """A signed batch resident on one device: seeds -> (pks, sigs) signed on the GPU.

    damage_every=k corrupts the signatures of requests i % k == k // 2 (global
    index i = start + j), cycling over four kinds of damage (R bit flip, S + L
    malleation, message byte, key bit), so the expected verdicts are known by
    construction: `expected()`."""

    def __init__(self, n, device=0, seed=0x5EED2025, start=0, msg_len=256, var_range=None, damage_every=0):
        self.n, self.device = n, device
        self.start = start
        msgs, off = nym_messages(n, seed, start, msg_len, var_range)
        seeds = np.random.default_rng([seed, start, 7]).integers(0, 256, size=32 * n, dtype=np.uint8)
        self.host_msgs, self.host_off = msgs, off
        self.d_msgs = edv.DeviceBuffer(msgs.nbytes, device)
        self.d_msgs.upload(msgs)
        self.d_off = edv.DeviceBuffer(off.nbytes, device)
        self.d_off.upload(off)
        d_seeds = edv.DeviceBuffer(seeds.nbytes, device)
        d_seeds.upload(seeds)
        self.d_pks = edv.DeviceBuffer(32 * n, device)
        self.d_sigs = edv.DeviceBuffer(64 * n, device)
        self.d_accept = edv.DeviceBuffer(n, device)
        edv.sign_device(d_seeds.ptr, self.d_msgs.ptr, self.d_off.ptr, n, self.d_pks.ptr, self.d_sigs.ptr, device)
        d_seeds.free()
        # one SHA-512 block count for the whole batch: no length buckets needed (a
        # per-call hint; the device-wide mode stays untouched)
        self.flags = edv.FLAG_UNIFORM_LENGTH if var_range is None else 0
        self.bad = damage_positions(start, n, damage_every)
        if self.bad.size:
            self._damage()

    def _damage(self):
        """Vectorised over the damaged positions (C3 damages 800k of 16M)."""
        L = 2**252 + 27742317777372353535851937790883648493
        sigs = self.d_sigs.download(64 * self.n).copy()
        pks = self.d_pks.download(32 * self.n).copy()
        msgs = self.host_msgs.copy()
        bad = self.bad
        kind = (self.start + bad) % 4
        i0, i1, i2, i3 = (bad[kind == k] for k in range(4))
        sigs[64 * i0 + 5] ^= 0x10                                           # R bit
        if i1.size:                                                         # S + L (256-bit add)
            sv = sigs.reshape(self.n, 64)[i1, 32:].copy().view(np.uint64)   # 4 little-endian limbs
            lw = [np.uint64((L >> (64 * k)) & (2**64 - 1)) for k in range(4)]
            carry = np.zeros(len(i1), dtype=np.uint64)
            for k in range(4):
                a = sv[:, k]
                t = a + lw[k]
                c1 = (t < a).astype(np.uint64)
                t2 = t + carry
                c2 = (t2 < t).astype(np.uint64)
                sv[:, k] = t2
                carry = c1 | c2
            sigs.reshape(self.n, 64)[i1, 32:] = sv.view(np.uint8).reshape(len(i1), 32)
        msgs[self.host_off[i2].astype(np.int64) + 3] ^= 0x01                # message byte
        pks[32 * i3 + 9] ^= 0x04                                            # key bit
        self.d_sigs.upload(sigs)
        self.d_pks.upload(pks)
        self.host_msgs = msgs
        self.d_msgs.upload(msgs)

    def expected(self):
        """The verdict bytes this batch must produce (1 except at the damaged positions)."""
        e = np.ones(self.n, dtype=np.uint8)
        e[self.bad] = 0
        return e

    def verify(self, stream=None):
        edv.verify_device(self.d_sigs.ptr, self.d_pks.ptr, self.d_msgs.ptr, self.d_off.ptr, self.n,
                          self.d_accept.ptr, self.device, stream=stream, flags=self.flags)

    def submit(self):
        """Pipelined verify (edv_verify_batch_dev_pipelined); results after edv.pipeline_sync."""
        edv.verify_device_pipelined(self.d_sigs.ptr, self.d_pks.ptr, self.d_msgs.ptr, self.d_off.ptr, self.n,
                                    self.d_accept.ptr, self.device, flags=self.flags)

    def accept(self):
        return self.d_accept.download(self.n)

    def host_copy(self):
        """(sigs, pks, msgs, off) host arrays of this batch."""
        return (self.d_sigs.download(64 * self.n), self.d_pks.download(32 * self.n), self.host_msgs, self.host_off)
