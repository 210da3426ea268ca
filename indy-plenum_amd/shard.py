"""Multi-GPU sharding of a verify batch by request index.

Verification has no exchange step: shard k of G gets a contiguous index range
and nothing crosses devices until the verdicts are gathered back into request
order: the shards' accept bytes land in their slices of the caller's array in
edv_verify_batch (one host thread per device); in bench.py's
one-process-per-GPU layout each rank packs its verdicts into a bitmask on its
GPU (edv_pack_bits_dev, N/8 bytes), copies it to the host and sends it to rank
0 over a loopback TCP rendezvous after the timed region (no torch, no RCCL:
nothing in the product or the bench needs a collective).

Two splits:
  shard_range   equal counts, [k*N/G, (k+1)*N/G)   (C2/C3: one message length)
  shard_bounds  the split edv_verify_batch applies (include/edv.h
                edv_shard_split): equal counts when every message has the same
                SHA-512 block count, else equal estimated cost, the sum over a
                shard of (VERIFY_BLOCKS + SHA-512 blocks of R||A||M)  (C4)
"""
import numpy as np

# fixed per-verify work in SHA-512-block units: W(m) = 217,600 + 5,500 * blocks
# INT32 ops, 217,600 / 5,500 ~ 40
VERIFY_BLOCKS = 40


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous [lo, hi) of request indices for `rank`, equal counts."""
    return n_total * rank // world, n_total * (rank + 1) // world


def sha512_blocks(offsets):
    """SHA-512 compressions of R || A || M per request (64-byte prefix + padding)."""
    off = np.asarray(offsets, dtype=np.uint64)
    lens = (off[1:] - off[:-1]).astype(np.int64)
    return (64 + lens + 17 + 127) // 128


def shard_bounds(offsets, g: int):
    """g+1 bounds of the split edv_verify_batch uses (numpy restatement of
    edv_shard_split, checked against it in tests/test_shard_cpu.py)."""
    off = np.asarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    b = np.zeros(g + 1, dtype=np.int64)
    b[g] = n
    if n <= 0:
        return np.zeros(g + 1, dtype=np.int64)
    blocks = sha512_blocks(off)
    if np.all(blocks == blocks[0]):
        for k in range(1, g):
            b[k] = n * k // g
        return b
    w = VERIFY_BLOCKS + blocks
    pre = np.concatenate([[0], np.cumsum(w)])  # pre[i] = cost of requests [0, i)
    total = int(pre[-1])
    for k in range(1, g):
        # first i (0 <= i < n) with pre[i] * g >= total * k, else n
        i = int(np.searchsorted(pre[:n] * g, total * k, side="left"))
        b[k] = min(i, n)
    return b


def slice_batch(sigs, pks, msgs, off, lo, hi):
    """The C-ABI arrays of requests [lo, hi) (offsets re-based to the shard's message bytes)."""
    o = np.asarray(off[lo:hi + 1], dtype=np.uint64)
    m0, m1 = int(o[0]), int(o[-1])
    return (sigs[64 * lo:64 * hi], pks[32 * lo:32 * hi], msgs[m0:m1 + 64] if m1 + 64 <= len(msgs) else
            np.concatenate([msgs[m0:m1], np.zeros(64, np.uint8)]), o - np.uint64(m0))
