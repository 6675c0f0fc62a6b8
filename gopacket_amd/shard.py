"""Multi-GPU sharding of a packet batch.

Every packet decodes independently (DecodeLayers resets its state per packet,
parser.go:304, layers_decoder.go:20), so a batch splits into contiguous
per-GPU ranges with no collective on the data path; results are disjoint
index ranges that concatenate. One process per GPU (torch.distributed),
each decoding its range on its own HIP stream.
"""
import numpy as np


def weak_range(rank, n_per_rank):
    """Weak scaling (bench.py): rank r owns packets [r*n, (r+1)*n)."""
    return rank * n_per_rank, n_per_rank


def byte_balanced_bounds(caplens, world):
    """Strong scaling of one batch: split at sum(caplen)*k/world so every GPU
    reads about the same number of bytes (IMIX batches are size-skewed).
    Returns world+1 packet indices."""
    caplens = np.asarray(caplens, dtype=np.uint64)
    csum = np.concatenate([[0], np.cumsum(caplens, dtype=np.uint64)])
    total = int(csum[-1])
    cuts = [0]
    for k in range(1, world):
        cuts.append(int(np.searchsorted(csum, total * k // world, side="left")))
    cuts.append(len(caplens))
    return cuts


def max_over_ranks(x, world, device=None):
    """Job time = the slowest rank's time (bench.py contract)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
