"""Multi-GPU sharding of a verify batch by request index.

Verification has no exchange step: shard k of G gets the contiguous index range
[k*N/G, (k+1)*N/G) and nothing crosses devices until the per-request accept
bytes are gathered back into request order (host memcpy in edv_verify_batch;
an all-gather over torch.distributed -- RCCL over xGMI on the GPU box, gloo in
the CPU tests -- in the one-process-per-GPU layout bench.py uses).
"""
import numpy as np


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous [lo, hi) of request indices for `rank` (same split as edv_verify_batch)."""
    return n_total * rank // world, n_total * (rank + 1) // world


def slice_batch(sigs, pks, msgs, off, lo, hi):
    """The C-ABI arrays of requests [lo, hi) (offsets re-based to the shard's message bytes)."""
    o = np.asarray(off[lo:hi + 1], dtype=np.uint64)
    m0, m1 = int(o[0]), int(o[-1])
    return (sigs[64 * lo:64 * hi], pks[32 * lo:32 * hi], msgs[m0:m1 + 64] if m1 + 64 <= len(msgs) else
            np.concatenate([msgs[m0:m1], np.zeros(64, np.uint8)]), o - np.uint64(m0))


def gather_accept(dist, local_accept, n_total: int, device=None):
    """All-gather every rank's accept bytes back into request order -> np.uint8[n_total].

    `dist` is torch.distributed (initialised); shards may differ by one in size,
    so each rank pads to the largest shard before the all-gather.
    """
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = [shard_range(n_total, world, r) for r in range(world)]
    mx = max(hi - lo for lo, hi in sizes)
    buf = np.zeros(mx, dtype=np.uint8)
    buf[:len(local_accept)] = local_accept
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    full = np.zeros(n_total, dtype=np.uint8)
    for (lo, hi), o in zip(sizes, outs):
        full[lo:hi] = o.cpu().numpy()[:hi - lo]
    return full
