"""The N>1 path on CPU: world_size-2 torch.distributed (gloo) run of the
shard-by-request-index + accept all-gather logic bench.py uses with RCCL on
the GPU box.  Each rank verifies its shard with the checker (this is a test of
the sharding, not of the kernels)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N = 3001  # odd: shards differ in size


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    import oracle_lib as orc
    from indy_plenum_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sigs, pks, msgs, off = orc.corpus(0x51A2D, 0, N, mode=1, invalid_permille=200, threads=2)
        lo, hi = shard.shard_range(N, world, rank)
        s, p, m, o = shard.slice_batch(sigs, pks, msgs, off, lo, hi)
        local = np.frombuffer(orc.verify_batch(s.tobytes(), p.tobytes(), m.tobytes(), o, hi - lo, 2), np.uint8)
        full = shard.gather_accept(dist, local, N)
        if rank == 0:
            whole = np.frombuffer(orc.verify_batch(sigs.tobytes(), pks.tobytes(), msgs.tobytes(), off, N, 4),
                                  np.uint8)
            q.put((full.tobytes(), whole.tobytes()))
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_exactly():
    from indy_plenum_amd import shard
    for n in (0, 1, 7, 65536, 16777216):
        for g in (1, 2, 3, 4, 8):
            rs = [shard.shard_range(n, g, r) for r in range(g)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[k][1] == rs[k + 1][0] for k in range(g - 1))
            assert max(hi - lo for lo, hi in rs) - min(hi - lo for lo, hi in rs) <= 1


@pytest.mark.timeout(300)
def test_two_rank_gloo_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, whole = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert full == whole
    acc = np.frombuffer(full, np.uint8)
    assert 0 < acc.sum() < N
