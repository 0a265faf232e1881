"""The N>1 path on CPU (BASELINE config 4): world_size-2 gloo ranks run the
benchmark's strong sharding and host-scalar reductions (libapenetwork_amd.sharding) over
one fixed batch of synthetic blocks.  Each rank compresses and decompresses its own shard
through the PRODUCT library's host codec (ape_lz4_host.c: the reference's compress_default
/ decompress_safe restated bit-exactly -- the GPU kernels are not available here), and
the oracle checks the bytes.  Checks: shards are disjoint, contiguous and cover the batch;
each rank's blocks are the global batch's slice; per-rank compressed sizes reduce to the
single-process totals; the max-over-ranks time is the slowest rank's; no collective other
than the gloo scalar ones is used.
"""
import ctypes as C
import os
import socket
import zlib

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, TOTAL, WORLD = 4096, 13, 2     # 13 blocks: an uneven split (6 + 7)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _product_host_codec():
    import libapenetwork_amd as amd
    L = amd.lib()
    L.hst_compress_extstate.restype = C.c_int
    L.hst_compress_extstate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                        C.c_int]
    L.hst_decompress_usingDict.restype = C.c_int
    L.hst_decompress_usingDict.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                           C.c_void_p, C.c_int]
    return L


def _shard_stats(orc, first, count):
    """Product host codec over blocks [first, first+count): (compressed bytes, crc list)."""
    L = _product_host_codec()
    buf = C.create_string_buffer(N * max(count, 1))
    if count:
        orc.synth_blocks(buf, N, C.c_longlong(N), C.c_longlong(first), count, 1)
    cap = orc.orc_compressBound(N)
    out, dec = C.create_string_buffer(cap + 64), C.create_string_buffer(N + 64)
    state = C.create_string_buffer(16416)
    ref = C.create_string_buffer(cap + 64)
    total, cks = 0, []
    for b in range(count):
        blk = buf.raw[b * N:(b + 1) * N]
        src = C.create_string_buffer(blk, N + 16)
        r = L.hst_compress_extstate(state, src, out, N, cap, 1)
        # the product's host codec is the reference's compress_default (oracle-checked)
        er = orc.orc_compress_default(src, ref, N, cap)
        assert r == er and out.raw[:r] == ref.raw[:r]
        assert L.hst_decompress_usingDict(out, dec, r, N, 1, None, 0) == N and dec.raw[:N] == blk
        total += r
        cks.append(zlib.crc32(blk))
    return total, cks


def _worker(rank, port, q):
    import torch.distributed as dist
    from libapenetwork_amd.sharding import gather, reduce_max, reduce_sum, shard_strong
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        orc = C.CDLL(os.path.join(ROOT, "oracle", "liblz4_oracle.so"))
        first, count = shard_strong(rank, WORLD, TOTAL)
        comp, cks = _shard_stats(orc, first, count)
        dist.barrier()
        elapsed = reduce_max(dist, 1.0 + rank)   # rank 1 is the slow one
        tot_comp, tot_ok = reduce_sum(dist, [comp, 1])
        ranges = gather(dist, (first, count, cks), WORLD)
        q.put((rank, elapsed, tot_comp, tot_ok, ranges))
    finally:
        dist.destroy_process_group()


def test_strong_shard_mapping():
    """Config 4: 1,048,576 blocks over N = 1, 2, 4, 8 GPUs -> contiguous equal shards
    (131072 per GPU at N = 8); uneven totals differ by at most one block per rank."""
    from libapenetwork_amd.sharding import shard, shard_strong
    for world in (1, 2, 4, 8):
        parts = [shard_strong(r, world, 1 << 20) for r in range(world)]
        assert all(c == (1 << 20) // world for _, c in parts)
        assert [f for f, _ in parts] == [r * ((1 << 20) // world) for r in range(world)]
    assert shard_strong(7, 8, 1 << 20) == (7 * 131072, 131072)
    for total in (0, 1, 7, 13, 1000003):
        for world in (1, 2, 3, 8):
            parts = [shard_strong(r, world, total) for r in range(world)]
            assert sum(c for _, c in parts) == total
            assert all(parts[r][0] + parts[r][1] == parts[r + 1][0] for r in range(world - 1))
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    assert [shard(r, 4, 10) for r in range(4)] == [(0, 10), (10, 10), (20, 10), (30, 10)]
    with pytest.raises(ValueError):
        shard_strong(8, 8, 10)


def test_reductions_without_dist():
    from libapenetwork_amd.sharding import gather, reduce_max, reduce_sum
    assert reduce_max(None, 2.5) == 2.5
    assert reduce_sum(None, [3, 4]) == [3, 4]
    assert gather(None, {"a": 1}, 1) == [{"a": 1}]


def test_bench_uses_no_rccl():
    """bench.py's process group is gloo (host scalars only): no RCCL on the path."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'init_process_group("gloo")' in src and '"nccl"' not in src


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
    total, all_cks = _shard_stats(oracle, 0, TOTAL)   # single process over the whole batch
    for rank, elapsed, tot_comp, tot_ok, ranges in res:
        assert elapsed == 2.0                      # max over ranks
        assert tot_comp == total and tot_ok == WORLD
        assert [(f, c) for f, c, _ in ranges] == [(0, 6), (6, 7)]   # disjoint, covering
        assert [ck for _, _, cks in ranges for ck in cks] == all_cks


def test_launch_plan_for_gpus_flag():
    """`bench.py --gpus N` (no torchrun) starts N ranks itself: one per device, each with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and its contiguous shard."""
    from libapenetwork_amd.sharding import launch_plan
    for n in (2, 8):
        plan = launch_plan(n, 1 << 20, device_count=8, master_port=12345)
        assert [p["rank"] for p in plan] == list(range(n))
        assert [p["device"] for p in plan] == list(range(n))
        assert [p["nblocks"] for p in plan] == [(1 << 20) // n] * n
        assert [p["first_block"] for p in plan] == [r * ((1 << 20) // n) for r in range(n)]
        for p in plan:
            e = p["env"]
            assert e["RANK"] == e["LOCAL_RANK"] == str(p["rank"])
            assert e["WORLD_SIZE"] == str(n) and e["MASTER_ADDR"] == "127.0.0.1"
            assert e["MASTER_PORT"] == "12345"
    assert launch_plan(8, 1 << 20, 8)[7]["nblocks"] == 131072
    # weak scaling: every rank its own --blocks
    assert [(p["first_block"], p["nblocks"]) for p in launch_plan(2, 10, 2, weak=True)] == \
        [(0, 10), (10, 10)]
    # too few devices is an error, unless a rehearsal device is named
    with pytest.raises(ValueError):
        launch_plan(8, 1 << 20, device_count=1)
    plan = launch_plan(2, 131072, device_count=1, rehearsal_device="0")
    assert [p["device"] for p in plan] == [0, 0]
    assert [p["nblocks"] for p in plan] == [65536, 65536]


def _fake_topology(root, gpus, cpus=1):
    """A KFD topology tree like /sys/class/kfd/kfd/topology/nodes: CPU nodes have no SIMDs."""
    for i in range(cpus + gpus):
        d = os.path.join(root, str(i))
        os.makedirs(d)
        simd = 0 if i < cpus else 256
        with open(os.path.join(d, "properties"), "w") as f:
            f.write("cpu_cores_count %d\nsimd_count %d\ngfx_target_version %d\n" % (
                64 if i < cpus else 0, simd, 0 if i < cpus else 90500))
    return root


def test_visible_gpu_count_without_runtime(tmp_path):
    """The launcher's device count comes from sysfs, with the runtime's visibility lists."""
    from libapenetwork_amd.sharding import visible_gpu_count
    nodes = _fake_topology(str(tmp_path / "nodes"), gpus=8, cpus=2)
    assert visible_gpu_count(nodes, {}) == 8
    assert visible_gpu_count(nodes, {"HIP_VISIBLE_DEVICES": "0,3"}) == 2
    assert visible_gpu_count(nodes, {"CUDA_VISIBLE_DEVICES": "5"}) == 1
    assert visible_gpu_count(nodes, {"ROCR_VISIBLE_DEVICES": "1,2,3,4",
                                     "HIP_VISIBLE_DEVICES": "0,1,7"}) == 2   # 7 >= 4 stops
    assert visible_gpu_count(nodes, {"HIP_VISIBLE_DEVICES": ""}) == 0
    assert visible_gpu_count(nodes, {"GPU_DEVICE_ORDINAL": "2,9"}) == 1


_LAUNCHER_PROBE = r"""
import json, os, subprocess, sys
sys.path.insert(0, sys.argv[1])
import bench
from libapenetwork_amd import sharding
sharding.KFD_NODES = sys.argv[2]
started = []
class FakeProc:
    def __init__(self, cmd, env=None, stdout=None):
        started.append({k: env[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")})
        self.pid = 0
    def poll(self):
        return 0
subprocess.Popen = FakeProc
import argparse
rc = bench.launch_ranks(argparse.Namespace(gpus=8, blocks=1 << 20, weak=False))
maps = open("/proc/self/maps").read()
print(json.dumps({"rc": rc, "started": started, "torch": "torch" in sys.modules,
                  "hip": ("libamdhip64" in maps) or ("libhsa-runtime" in maps)}))
"""


def test_launcher_touches_no_gpu_runtime(tmp_path):
    """`bench.py --gpus 8`'s parent counts devices from sysfs and starts the ranks without
    importing torch or mapping the HIP/HSA runtime: the children begin
    in a process tree where nothing initialised a GPU."""
    import json
    import subprocess
    import sys
    nodes = _fake_topology(str(tmp_path / "nodes"), gpus=8)
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "APE_BENCH_DEVICE", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
              "ROCR_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _LAUNCHER_PROBE, ROOT, nodes], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["rc"] == 0 and not res["torch"] and not res["hip"]
    assert [s["RANK"] for s in res["started"]] == [str(i) for i in range(8)]
    assert all(s["WORLD_SIZE"] == "8" and s["MASTER_ADDR"] == "127.0.0.1"
               for s in res["started"])


def _bench(args, env_extra):
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("APE_BENCH_DEVICE", None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_refuses_to_misreport_world_size():
    """bench.py exits non-zero instead of timing one GPU and printing n_gpus: 1 when --gpus
    and the launcher's world size disagree, or when fewer devices than --gpus are visible."""
    import torch
    r = _bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""
    if torch.cuda.device_count() < 2:
        r = _bench(["--gpus", "2"], {})
        assert r.returncode == 2 and "device(s) visible" in r.stderr and r.stdout == ""
