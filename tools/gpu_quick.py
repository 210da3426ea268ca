"""First GPU bring-up: golden parity through the C-ABI + a 64k x 256 B timing."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from indy_plenum_amd import edv
import golden_io, oracle_lib as orc

print("version", edv.version(), "devices", edv.device_count(), flush=True)
recs = golden_io.load_ed25519_golden()
sigs, pks, msgs, off = golden_io.pack_batch(recs)
t = time.time()
acc = edv.verify_arrays(sigs, pks, msgs, off)
print("golden verify s", time.time() - t, flush=True)
exp = np.array([r[0] for r in recs], dtype=np.uint8)
bad = np.nonzero(acc != exp)[0]
print("golden mismatches", len(bad), bad[:20].tolist(), flush=True)
# 64k x 256 B distinct signers (oracle signer)
n = int(os.environ.get("N", 65536))
rng = np.random.default_rng(1)
seeds = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
msg = rng.integers(0, 256, size=(n, 256), dtype=np.uint8)
S, P = bytearray(), bytearray()
t = time.time()
for i in range(n):
    pk, sk = orc.keypair(seeds[i].tobytes())
    S += orc.sign(msg[i].tobytes(), sk); P += pk
print("gen s", time.time() - t, flush=True)
offs = np.arange(n + 1, dtype=np.uint64) * 256
t = time.time()
acc = edv.verify_arrays(bytes(S), bytes(P), msg.tobytes(), offs)
print("host-path verify s", time.time() - t, "accepted", int(acc.sum()), "of", n, flush=True)
dS, dP, dM, dO, dA = (edv.DeviceBuffer(len(S)), edv.DeviceBuffer(len(P)), edv.DeviceBuffer(msg.nbytes + 64),
                      edv.DeviceBuffer(offs.nbytes), edv.DeviceBuffer(n))
dS.upload(np.frombuffer(bytes(S), np.uint8)); dP.upload(np.frombuffer(bytes(P), np.uint8)); dM.upload(msg); dO.upload(offs)
ms = edv.time_device(dS.ptr, dP.ptr, dM.ptr, dO.ptr, n, dA.ptr, iters=1)
ms = edv.time_device(dS.ptr, dP.ptr, dM.ptr, dO.ptr, n, dA.ptr, iters=5)
print("kernel ms/launch", ms / 5, "verifies/s", n / (ms / 5e3), flush=True)
print("device accept", int(dA.download(n).sum()))
