"""bench.py's multi-GPU plumbing on CPU (the N>1 path of the
driver's bench contract): the loopback rendezvous its ranks use for the
barriers, the max over ranks of the timed region and the gather of every
shard's accept bytes into its slice of one host array -- exercised here by 2
and 3 spawned processes, no GPU and no torch -- and the launcher's loud
failure when --gpus asks for more devices than are visible."""
import json
import multiprocessing as mp
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOTAL = 100003   # odd: shards differ in size


def _rank(rank, world, token, q):
    sys.path.insert(0, ROOT)
    import bench
    from indy_plenum_amd import shard, workload
    rdv = bench.Rendezvous(rank, world, token, timeout=60)
    try:
        rdv.barrier()
        m = rdv.max(float(rank * 10 + 1))
        lo, hi = shard.shard_range(TOTAL, world, rank)
        # this shard's verdicts: the C3 damage pattern, as a rank's accept bytes would be
        acc = np.ones(hi - lo, np.uint8)
        acc[workload.damage_positions(lo, hi - lo, 20)] = 0
        # rank 0 alone (the one-GPU same-workload reference), then all ranks
        import time as _t
        own = []
        alone = bench.timed_steps(lambda: _t.sleep(0.02), lambda: None, 3, 1, rdv, only_rank=0, own=own)
        joint = bench.timed_steps(lambda: _t.sleep(0.01 * (rank + 1)), lambda: None, 2, 2, rdv, own=own)
        assert alone[0] >= 0.06 and (rank == 0) == (own[0] >= 0.06)
        assert all(j >= 0.02 * world for j in joint) and all(o >= 0.02 * (rank + 1) for o in own[1:])
        parts = rdv.gather(acc.tobytes(), broadcast=False)
        allv = rdv.gather(b"r%d" % rank)
        rdv.barrier()
        if rank == 0:
            full = np.empty(TOTAL, np.uint8)
            for r, p in enumerate(parts):
                a, b = shard.shard_range(TOTAL, world, r)
                full[a:b] = np.frombuffer(p, np.uint8)
            exp = np.ones(TOTAL, np.uint8)
            exp[workload.damage_positions(0, TOTAL, 20)] = 0
            q.put(("root", m, bool(np.array_equal(full, exp)), [x.decode() for x in allv]))
        else:
            q.put(("peer", m, parts is None, [x.decode() for x in allv]))
    finally:
        rdv.close()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_barrier_max_and_slice_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    token = "pytest%d_%d" % (os.getpid(), world)
    procs = [ctx.Process(target=_rank, args=(r, world, token, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=90) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    want_names = ["r%d" % r for r in range(world)]
    for kind, m, ok, names in res:
        assert m == float((world - 1) * 10 + 1)        # every rank gets the max
        assert ok                                      # root: slices reassembled in order; peer: no copy sent back
        assert names == want_names                     # broadcast gather, rank order
    assert sorted(k for k, *_ in res) == ["peer"] * (world - 1) + ["root"]


def test_launcher_fails_loudly_without_devices():
    """--gpus 2 on a host with no gfx950: the launcher starts two ranks, they
    stop with a message naming the device count, and the launcher's exit status
    is non-zero (nothing hangs at a barrier)."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "gfx950 device(s) are visible" in r.stderr
    assert r.stdout.strip() == ""                      # no JSON line from a failed run


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=60, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_bench_imports_no_torch():
    """The bench and the product import no torch (the multi-rank path used to
    load torch's HIP runtime beside libedv's)."""
    code = ("import sys; sys.path.insert(0, %r); import bench; from indy_plenum_amd import edv, workload, shard, "
            "client_authn, req_authenticator, pool, digest; print(json.dumps('torch' in sys.modules))" % ROOT)
    r = subprocess.run([sys.executable, "-c", "import json; " + code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip()) is False


@pytest.mark.parametrize("vis,local,world,want", [
    (None, 3, 8, (0, "3")), ("4,5,6,7", 2, 4, (0, "6")), (" 0 , 1", 1, 2, (0, "1")),
    ("", 1, 2, (1, None)), ("0", 0, 1, (0, None))])
def test_each_rank_sees_only_its_gpu(monkeypatch, vis, local, world, want):
    """N > 1: every rank narrows HIP_VISIBLE_DEVICES to its LOCAL_RANK-th device
    before the HIP runtime loads, so it initialises one GPU;
    not under EDV_VIRTUAL_DEVICES (ranks share logical devices of one GPU)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("EDV_VIRTUAL_DEVICES", raising=False)
    if vis is None:
        monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    else:
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", vis)
    assert bench.narrow_to_own_gpu(local, world) == want
    if want[1] is not None:
        assert os.environ["HIP_VISIBLE_DEVICES"] == want[1]
    monkeypatch.setenv("EDV_VIRTUAL_DEVICES", "8")
    assert bench.narrow_to_own_gpu(5, 8) == (5, None)
