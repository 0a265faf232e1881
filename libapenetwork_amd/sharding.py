"""Block sharding across ranks for the batched codec.

The path shards naturally: blocks are independent, so rank r of W takes the
contiguous block range [r*N, (r+1)*N) of a global batch (weak scaling: N blocks
per rank), with its own inputs, output slots and size/status arrays.  There is no
collective on the data path; the only cross-rank operations are the benchmark's
barrier, the max-over-ranks step time and the sum of per-rank byte counts, all on
scalars.  Works with any torch.distributed backend (RCCL/"nccl" on the GPUs, "gloo"
in the CPU tests).
"""


def shard(rank, world, blocks_per_rank):
    """(first_block, nblocks) of `rank` in a weak-scaled batch of world*blocks_per_rank."""
    if world < 1 or not 0 <= rank < world or blocks_per_rank < 0:
        raise ValueError("bad shard request: rank %r of %r, %r blocks" % (rank, world,
                                                                          blocks_per_rank))
    return rank * blocks_per_rank, blocks_per_rank


def reduce_max(dist, value, device):
    """Max of a float over ranks (the benchmark's step time); identity without dist."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(dist, values, device):
    """Elementwise sum of a list of ints over ranks; identity without dist."""
    if dist is None:
        return [int(v) for v in values]
    import torch
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]
