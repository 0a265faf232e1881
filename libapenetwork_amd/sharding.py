"""Block sharding across ranks for the batched codec (BASELINE config 4).

The path shards naturally: blocks are independent.  BASELINE config 4 is "1M x 64 KiB
blocks sharded across 8 MI355X": a fixed total batch of N blocks split contiguously,
rank r of W taking blocks [r*N//W, (r+1)*N//W) (strong scaling; 131072 blocks per GPU
at N = 1M, W = 8), each rank with its own inputs, output slots and size/status arrays.
Weak scaling (N blocks per rank) stays available as an opt-in.

There is no collective on the data path and no RCCL at all: the only cross-rank
operations are the benchmark's barrier, the max-over-ranks step time and the gather of
per-rank scalars, all on host scalars over a gloo (CPU) process group.
"""
import os


def shard_strong(rank, world, total_blocks):
    """(first_block, nblocks) of `rank`: the contiguous split of a fixed batch."""
    if world < 1 or not 0 <= rank < world or total_blocks < 0:
        raise ValueError("bad shard request: rank %r of %r, %r blocks" % (rank, world,
                                                                          total_blocks))
    first = rank * total_blocks // world
    return first, (rank + 1) * total_blocks // world - first


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _visible(n, spec):
    """Devices left of `n` after a *_VISIBLE_DEVICES list (indices or UUIDs); the runtime
    stops at the first index that does not exist, and an empty list hides every device."""
    if spec is None:
        return n
    k = 0
    for tok in (t.strip() for t in spec.split(",")):
        if not tok:
            break
        if tok.isdigit() and int(tok) >= n:
            break
        k += 1
    return min(k, n)


def visible_gpu_count(nodes=None, environ=None):
    """GPUs this process would see, counted WITHOUT the HIP runtime: the KFD topology nodes
    with SIMDs (CPU nodes have none), then ROCR_VISIBLE_DEVICES, HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES and GPU_DEVICE_ORDINAL applied in the runtime's order.  bench.py's
    launcher calls this in the parent, which must not initialise a GPU before it starts the
    ranks (torch.cuda.device_count() may fall back to hipGetDeviceCount).  None when the
    topology is not readable but /dev/kfd exists (the ranks then check for their device
    themselves); 0 without /dev/kfd."""
    env = os.environ if environ is None else environ
    nodes = KFD_NODES if nodes is None else nodes
    try:
        names = os.listdir(nodes)
    except OSError:
        return None if os.path.exists("/dev/kfd") else 0
    n = 0
    for name in names:
        try:
            with open(os.path.join(nodes, name, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    n = _visible(n, env.get("ROCR_VISIBLE_DEVICES"))
    n = _visible(n, env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES")))
    return _visible(n, env.get("GPU_DEVICE_ORDINAL"))


def launch_plan(ngpus, total_blocks, device_count, rehearsal_device=None, weak=False,
                master_port=29500):
    """The ranks `bench.py --gpus N` starts by itself (one process per GPU):
    a list of {rank, device, first_block, nblocks, env} with the RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* environment of each child.  Raises ValueError when fewer than N
    devices are visible, unless `rehearsal_device` (APE_BENCH_DEVICE) puts every rank on
    that one device.  device_count None (not known without the runtime) starts the ranks
    and leaves the check to them."""
    if ngpus < 1:
        raise ValueError("--gpus must be >= 1, got %r" % (ngpus,))
    if rehearsal_device is None and device_count is not None and device_count < ngpus:
        raise ValueError("--gpus %d but only %d device(s) visible" % (ngpus, device_count))
    plan = []
    for r in range(ngpus):
        first, nb = shard(r, ngpus, total_blocks) if weak else shard_strong(r, ngpus,
                                                                            total_blocks)
        plan.append({
            "rank": r, "device": r if rehearsal_device is None else int(rehearsal_device),
            "first_block": first, "nblocks": nb,
            "env": {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(ngpus),
                    "LOCAL_WORLD_SIZE": str(ngpus), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(master_port)},
        })
    return plan


def shard(rank, world, blocks_per_rank):
    """(first_block, nblocks) of `rank` in a weak-scaled batch of world*blocks_per_rank."""
    if world < 1 or not 0 <= rank < world or blocks_per_rank < 0:
        raise ValueError("bad shard request: rank %r of %r, %r blocks" % (rank, world,
                                                                          blocks_per_rank))
    return rank * blocks_per_rank, blocks_per_rank


def reduce_max(dist, value, device="cpu"):
    """Max of a float over ranks (the benchmark's step time); identity without dist."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(dist, values, device="cpu"):
    """Elementwise sum of a list of ints over ranks; identity without dist."""
    if dist is None:
        return [int(v) for v in values]
    import torch
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]


def gather(dist, obj, world):
    """Every rank's `obj` (list indexed by rank); [obj] without dist."""
    if dist is None:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out
