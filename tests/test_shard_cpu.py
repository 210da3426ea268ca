"""The N>1 path on CPU.

* The shard split edv_verify_batch applies (edv_shard_split in libedv.so, host
  code, callable without a GPU) against its numpy restatement
  (indy-plenum_amd/shard.py) and against the properties SURVEY.md section 8e
  asks for: contiguous, covering, equal counts for one message length, equal
  estimated cost (sum of 40 + SHA-512 blocks) for C4's 200 B - 4 KB lengths.
* A world_size-2 torch.distributed (gloo) run of the shard split and the
  gather of per-shard accept bytes into request order; each rank verifies its
  shard with the checker (this tests the sharding, not the kernels).  bench.py's
  own rank rendezvous (no torch) is tested in tests/test_bench_cpu.py.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 3001  # odd: shards differ in size


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
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
        bounds = shard.shard_bounds(off, world)           # C4 lengths: cost-balanced split
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        s, p, m, o = shard.slice_batch(sigs, pks, msgs, off, lo, hi)
        local = np.frombuffer(orc.verify_batch(s.tobytes(), p.tobytes(), m.tobytes(), o, hi - lo, 2), np.uint8)
        parts = [None] * world
        dist.all_gather_object(parts, local.tobytes())
        full = np.zeros(N, np.uint8)
        for r, p in enumerate(parts):
            full[int(bounds[r]):int(bounds[r + 1])] = np.frombuffer(p, np.uint8)
        if rank == 0:
            whole = np.frombuffer(orc.verify_batch(sigs.tobytes(), pks.tobytes(), msgs.tobytes(), off, N, 4),
                                  np.uint8)
            q.put((full.tobytes(), whole.tobytes(), bounds.tolist()))
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


def _offsets(lens):
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(np.asarray(lens, dtype=np.uint64))
    return off


def _cases():
    rng = np.random.default_rng(8)
    yield "empty", _offsets([])
    yield "one", _offsets([256])
    yield "c2_fixed", _offsets([256] * 65536)
    yield "same_blocks_diff_len", _offsets(rng.integers(175, 303, size=1000))  # all 3 SHA-512 blocks
    yield "c4_uniform", _offsets(rng.integers(200, 4097, size=20000))
    yield "c4_sorted", _offsets(np.sort(rng.integers(200, 4097, size=20000)))   # skewed: cost grows with index
    yield "bimodal", _offsets(np.where(rng.random(5000) < 0.1, 65536, 200))
    yield "tiny", _offsets([0, 0, 5000, 0, 0, 0, 7])


def _cost(off, lo, hi):
    from indy_plenum_amd import shard
    return int((shard.VERIFY_BLOCKS + shard.sha512_blocks(off[lo:hi + 1])).sum()) if hi > lo else 0


@pytest.mark.parametrize("g", [1, 2, 3, 4, 8])
def test_shard_split_cabi_matches_restatement(g):
    from indy_plenum_amd import edv, shard
    for name, off in _cases():
        got = edv.shard_split(off, g).astype(np.int64)
        want = shard.shard_bounds(off, g)
        assert got.tolist() == want.tolist(), name
        n = len(off) - 1
        assert got[0] == 0 and got[-1] == n and np.all(np.diff(got) >= 0), name


@pytest.mark.parametrize("g", [2, 4, 8])
def test_shard_split_properties(g):
    from indy_plenum_amd import edv, shard
    for name, off in _cases():
        n = len(off) - 1
        b = edv.shard_split(off, g).astype(np.int64)
        blocks = shard.sha512_blocks(off) if n else np.zeros(0, np.int64)
        if n and np.all(blocks == blocks[0]):
            # one block count: equal counts, exactly the index split of shard_range
            assert b.tolist() == [shard.shard_range(n, g, r)[0] for r in range(g)] + [n], name
        elif n:
            costs = [_cost(off, int(b[k]), int(b[k + 1])) for k in range(g)]
            wmax = int((shard.VERIFY_BLOCKS + blocks).max())
            ideal = sum(costs) / g
            # every shard within one request's cost of the ideal share
            assert max(costs) <= ideal + wmax and min(costs) >= ideal - 2 * wmax, (name, costs)


def test_shard_split_balances_skewed_lengths():
    """Sorted C4 lengths: a count split would give the last shard ~3x the first's
    hashing; the cost split gives the long-message shard fewer requests."""
    from indy_plenum_amd import edv
    off = dict(_cases())["c4_sorted"]
    b = edv.shard_split(off, 4).astype(np.int64)
    sizes = np.diff(b)
    assert sizes[0] > sizes[-1]
    costs = [_cost(off, int(b[k]), int(b[k + 1])) for k in range(4)]
    assert max(costs) / min(costs) < 1.01


def test_shard_split_rejects_bad_arguments():
    from indy_plenum_amd import edv
    with pytest.raises(edv.EdvError):
        edv.shard_split(np.array([0, 10, 5], np.uint64), 2)   # offsets decrease
    with pytest.raises(edv.EdvError):
        edv.shard_split(np.array([0, 10], np.uint64), 0)


@pytest.mark.timeout(300)
def test_two_rank_gloo_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, whole, bounds = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert full == whole
    assert 0 < bounds[1] < N
    acc = np.frombuffer(full, np.uint8)
    assert 0 < acc.sum() < N
