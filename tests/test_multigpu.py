"""The N>1 path on CPU: world_size-2 gloo ranks run the benchmark's sharding and
reductions (libapenetwork_amd.sharding) over the same synthetic blocks, each rank
compressing/decompressing its own shard with the oracle (the GPU kernels are not
available here).  Checks: shards are disjoint and cover the batch, each rank's data
is the global data's slice, per-rank results reduce to the single-process totals,
and the max-over-ranks time is the slowest rank's.
"""
import ctypes as C
import os
import socket
import zlib

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, PER_RANK, WORLD = 4096, 6, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_stats(orc, first, count):
    """(compressed bytes, xor checksum of the blocks) of blocks [first, first+count)."""
    buf = C.create_string_buffer(N * count)
    orc.synth_blocks(buf, N, C.c_longlong(N), C.c_longlong(first), count, 1)
    cap = orc.orc_compressBound(N)
    out, dec = C.create_string_buffer(cap + 64), C.create_string_buffer(N + 64)
    total, ck = 0, 0
    for b in range(count):
        blk = buf.raw[b * N:(b + 1) * N]
        r = orc.orc_compress_default(C.create_string_buffer(blk, N + 16), out, N, cap)
        assert r > 0
        assert orc.orc_decompress_safe(out, dec, r, N) == N and dec.raw[:N] == blk
        total += r
        ck ^= zlib.crc32(blk)
    return total, ck


def _worker(rank, port, q):
    import torch.distributed as dist
    from libapenetwork_amd.sharding import reduce_max, reduce_sum, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        orc = C.CDLL(os.path.join(ROOT, "oracle", "liblz4_oracle.so"))
        first, count = shard(rank, WORLD, PER_RANK)
        comp, ck = _shard_stats(orc, first, count)
        elapsed = reduce_max(dist, 1.0 + rank, "cpu")   # rank 1 is the slow one
        tot_comp, tot_ok = reduce_sum(dist, [comp, 1], "cpu")
        ranges = [None] * WORLD
        dist.all_gather_object(ranges, (first, count, ck))
        q.put((rank, elapsed, tot_comp, tot_ok, ranges))
    finally:
        dist.destroy_process_group()


def test_sharding_unit():
    from libapenetwork_amd.sharding import reduce_max, reduce_sum, shard
    assert [shard(r, 4, 10) for r in range(4)] == [(0, 10), (10, 10), (20, 10), (30, 10)]
    with pytest.raises(ValueError):
        shard(4, 4, 10)
    assert reduce_max(None, 2.5, "cpu") == 2.5
    assert reduce_sum(None, [3, 4], "cpu") == [3, 4]


def test_two_rank_gloo(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference over the whole batch
    total, _ = _shard_stats(oracle, 0, WORLD * PER_RANK)
    for rank, elapsed, tot_comp, tot_ok, ranges in res:
        assert elapsed == 2.0                      # max over ranks
        assert tot_comp == total and tot_ok == WORLD
        covered = sorted((f, f + c) for f, c, _ in ranges)
        assert covered == [(0, PER_RANK), (PER_RANK, 2 * PER_RANK)]   # disjoint, covering
        for f, c, ck in ranges:
            assert ck == _shard_stats(oracle, f, c)[1]
