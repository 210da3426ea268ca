"""All-gather of per-shard accept bytes over torch.distributed (RCCL over xGMI on
the GPU box, gloo in the CPU tests) for the one-process-per-GPU layout of
bench.py.  Measurement/test infrastructure: the product package
(indy-plenum_amd/) has no torch dependency."""
import numpy as np


def gather_accept(dist, local_accept, bounds, device=None):
    """Every rank's accept bytes back into request order -> np.uint8[bounds[-1]].

    bounds[r]..bounds[r+1] is rank r's shard (shard sizes may differ), so each
    rank pads to the largest shard before the all-gather."""
    import torch
    world = dist.get_world_size()
    sizes = [int(bounds[r + 1]) - int(bounds[r]) for r in range(world)]
    mx = max(sizes) if sizes else 0
    buf = np.zeros(max(mx, 1), dtype=np.uint8)
    buf[:len(local_accept)] = local_accept
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    full = np.zeros(int(bounds[-1]), dtype=np.uint8)
    for r, o in enumerate(outs):
        full[int(bounds[r]):int(bounds[r + 1])] = o.cpu().numpy()[:sizes[r]]
    return full
