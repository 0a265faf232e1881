#!/usr/bin/env python3
"""bench.py -- LZ4 GiB/s device-resident (compress+decompress), 1M x 64 KiB blocks.

BASELINE.json metric / configs 3 and 4: 1,048,576 x 64 KiB compressible blocks,
compress+decompress.  With --gpus N under torch.distributed.run the fixed batch is split
contiguously (rank r takes blocks [r*N_total/N, (r+1)*N_total/N), 131072 per GPU at N = 8;
strong scaling, "scaling": "strong"), with no collective on the data path: a gloo process
group carries the barrier, the max-over-ranks time and the per-rank numbers (`per_gpu`).
--weak gives every rank its own 1M blocks instead.  `python bench.py --gpus N` starts the N
ranks itself (one child process per GPU, before anything touches a GPU); under
torch.distributed.run the launcher's WORLD_SIZE must equal --gpus.  Fewer than N visible
devices is an error, unless APE_BENCH_DEVICE=d puts every rank on device d (a rehearsal of
the N > 1 path on one GPU).

One step = compress every block of the rank (one launch of lz4_encode_kernel) then
decompress every compressed block (one launch of lz4_decode_kernel); inputs are generated
on the device before timing (SURVEY App. C `gen_comp`, seed = block id).  value =
uncompressed bytes of the job / max-over-ranks step time.  Correctness is checked after
timing (every decoded block == its source; sampled GPU-compressed blocks restored by the
oracle = the reference decoder restated) and the compression ratio is reported.

Also in the line (rank 0, N = 1): `config2` = BASELINE config 2 (256K x 4 KiB random blocks
compressed by the reference algorithm, decode only) with its own roofline and CPU baseline;
`config5` = BASELINE config 5 through a real byte path: GPU encode -> frames -> loopback TCP
connection(s) (--sock-conns, default 1) -> pinned growable rxbuf + frame
parser -> GPU decode (sock_leg, 8 GiB);
`cpu_baseline` = the reference src/ape_lz4.c built from its own source with gcc and clang
(oracle/_ref), a 1..N thread sweep over the box's usable cores on a 4 GiB sample;
`roofline` = the dominant kernel's algorithmic bytes / its HIP-event time, plus the
decoder's and the whole step's fractions and the HBM-read roofline the north_star names.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table (8.0 TB/s spec)
METRIC = "LZ4 GiB/s device-resident (compress+decompress), 1M×64KiB blocks, 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """Usable host cores of this box and how they were determined (BASELINE.md section 4:
    state nproc / lscpu).  usable = the affinity mask, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS when the harness sets it as the job's CPU share (the GPU box exposes the
    whole machine's CPUs to os.cpu_count() but grants one GPU job a share of them)."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    info["affinity"] = aff
    usable = aff
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
            usable = min(usable, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp:
        info["OMP_NUM_THREADS"] = omp
        if omp < usable:
            usable = omp
            info["limited_by"] = "OMP_NUM_THREADS (the job's CPU share on this box)"
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    if model is None:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
    info["model"] = model
    if usable > 256:   # oracle/cpu_bench.c runs at most 256 threads
        info["clamped_from"] = usable
        usable = 256
    info["usable"] = usable
    return usable, info


def _ref_libs():
    """(label, path, symbol prefix, kind) of the CPU codecs to time: the reference
    compiled from its own source with gcc and with clang (oracle/_ref, BASELINE.md
    section 4), else the oracle restatement."""
    libs = []
    for label, name in (("gcc", "libape_lz4_ref.so"), ("clang", "libape_lz4_ref_clang.so")):
        p = os.path.join(ROOT, "oracle", "_ref", name)
        if os.path.exists(p):
            libs.append((label, p, b"APE_LZ4_", "reference"))
    if not libs:
        libs.append(("gcc", os.path.join(ROOT, "oracle", "liblz4_oracle.so"), b"orc_", "port"))
    return libs


def _cpubench():
    lib = C.CDLL(os.path.join(ROOT, "oracle", "libcpubench.so"))
    lib.cpu_bench_prepare.restype = C.c_void_p
    lib.cpu_bench_prepare.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int]
    lib.cpu_bench_time.restype = C.c_int
    lib.cpu_bench_time.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
    lib.cpu_bench_free.argtypes = [C.c_void_p]
    return lib


def _sweep_threads(usable):
    ts, t = [], 1
    while t < usable:
        ts.append(t)
        t *= 2
    return ts + [usable]


def cpu_baseline(block, kind, nblocks, mode=0, min_seconds=0.0, repeats=1):
    """The reference codec on this host's cores: one block per
    task, static partition, a 1..N thread sweep, gcc and clang builds.  mode 0 =
    compress_default + decompress_safe (config 3), 1 = decompress_safe only (config 2).
    The sample is generated and compressed once untimed; each sweep point times whole
    passes over it (after a warm-up pass) and checks every decoded block.  With
    min_seconds, a measurement repeats the pass until it lasts that long (a 1 GiB config-2
    pass takes ~10 ms on 16 cores: too short to time alone), and the sweep point is the
    median of `repeats` such measurements."""
    usable, cores = host_cores()
    lib = _cpubench()
    out = (C.c_double * 5)()
    sweep, best, split, kindname = [], None, {}, None
    threads = _sweep_threads(usable)
    for label, path, prefix, kname in _ref_libs():
        kindname = kname
        h = lib.cpu_bench_prepare(path.encode(), prefix, nblocks, block, kind, usable)
        if not h:
            return None
        try:
            for t in threads:
                reps = 1
                if min_seconds > 0:   # size the repetition count from one pass
                    if lib.cpu_bench_time(h, t, 1, mode, out) != 0 or out[3] != 0:
                        return None
                    reps = max(1, int(min_seconds / max(out[0] + out[1], 1e-6)) + 1)
                meas = []
                for _ in range(max(1, repeats)):
                    if lib.cpu_bench_time(h, t, reps, mode, out) != 0 or out[3] != 0:
                        return None
                    meas.append((out[4] * reps / (out[0] + out[1]), out[0], out[1]))
                meas.sort()
                med = meas[len(meas) // 2]
                tc, td, csz, byt = med[1], med[2], out[2], out[4] * reps
                v = byt / (tc + td) / GIB
                row = next((r for r in sweep if r["threads"] == t), None)
                if row is None:
                    row = {"threads": t}
                    sweep.append(row)
                row[label] = round(v, 3)
                if repeats > 1:
                    row.setdefault("spread_" + label, [round(m[0] / GIB, 3) for m in meas])
                    row["reps"] = reps
                if t == usable:
                    split[label] = {"value": round(v, 3),
                                    "decompress_GiBps": round(byt / td / GIB, 3),
                                    "ratio": round(out[4] / csz, 4)}
                    if mode == 0:
                        split[label]["compress_GiBps"] = round(byt / tc / GIB, 3)
                    if best is None or v > best[1]:
                        best = (label, v)
        finally:
            lib.cpu_bench_free(h)
    label, v = best
    what = ("compress_default + decompress_safe" if mode == 0 else "decompress_safe only")
    res = {
        "value": round(v, 3), "unit": "GiB/s", "cores": usable, "kind": kindname,
        "compiler": label,
        "sample": "%d x %d KiB %s blocks (%.2f GiB), %s, one block per task, static partition "
                  "over %d threads; best of %s at %d threads%s" % (
                      nblocks, block >> 10, "compressible" if kind else "random",
                      nblocks * block / GIB, what, usable, "/".join(split), usable,
                      (", each sweep point the median of %d measurements of >= %.1f s" % (
                          repeats, min_seconds)) if repeats > 1 else ""),
        "host": cores, "sweep": sweep, "by_compiler": split,
    }
    res.update({k: v2 for k, v2 in split[label].items() if k != "value"})
    return res


def pmc_traffic(kernel, blocks):
    """HBM bytes per launch, PROFILE-DERIVED: FETCH_SIZE (x2, gfx950) + WRITE_SIZE per block
    from the committed rocprofv3 --pmc passes (profiles/pmc_traffic.json), times the blocks
    of this launch -- not measured by this run."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))[kernel]
        return int(d["bytes_per_block"] * blocks), d.get("source", "profiles/pmc_traffic.json")
    except Exception:
        return None, None


def e2e_bench(args):
    """Host -> GPU -> host rate of the socket path (BASELINE config 5 / north_star e2e).

    Compress (TX): pinned host blocks --H2D--> encode --> framed stream
    [le32 c][block]... (frame_offsets + frame_pack) --D2H--> pinned host stream.
    Decompress (RX): pinned framed stream --H2D--> decode straight out of the frames
    --D2H--> pinned host blocks.  Chunks of `--e2e-chunk` blocks (8192 = 512 MiB: a sweep of
    16384 / 8192 / 4096 measured TX 41.7 / 44.9 / 44.2 GiB/s) rotate over `--e2e-streams`
    streams, each with its own device buffers (stream order protects their reuse), so
    copies in both directions overlap the kernels.  Rates are
    uncompressed bytes / wall time.  Never the headline `value`.
    """
    import torch

    import libapenetwork_amd as amd

    torch.cuda.set_device(0)
    if amd.gpu_init() != 0:
        raise SystemExit("GPU codec unavailable: %s" % amd.gpu_last_error())
    n, nb, ch = args.block_size, args.e2e_blocks, args.e2e_chunk
    nch = (nb + ch - 1) // ch
    slot = (amd.compressBound(n) + 15) // 16 * 16
    kind = 1 if args.kind == "comp" else 0
    t0 = time.time()
    h_src = torch.empty((nb, n), dtype=torch.uint8, pin_memory=True)
    h_frames = torch.empty(nb * (slot + 4), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty((nb, n), dtype=torch.uint8, pin_memory=True)
    log("[e2e] pinned %.1f GiB host in %.1f s" % ((2 * nb * n + nb * (slot + 4)) / GIB,
                                                  time.time() - t0))
    NS = args.e2e_streams
    streams = [torch.cuda.Stream() for _ in range(NS)]
    bufs = []
    for _ in range(NS):
        bufs.append({
            "src": torch.empty((ch, n), dtype=torch.uint8, device="cuda"),
            "comp": torch.empty((ch, slot), dtype=torch.uint8, device="cuda"),
            "csz": torch.zeros(ch, dtype=torch.int32, device="cuda"),
            "off": torch.zeros(ch + 1, dtype=torch.int64, device="cuda"),
            "frames": torch.empty(ch * (slot + 4), dtype=torch.uint8, device="cuda"),
            "out": torch.empty((ch, n), dtype=torch.uint8, device="cuda"),
            "res": torch.zeros(ch, dtype=torch.int32, device="cuda"),
            "sizes": torch.full((ch,), n, dtype=torch.int32, device="cuda"),
            "tot": torch.zeros(1, dtype=torch.int64, pin_memory=True),
        })
    for b in bufs:
        b["scratch"] = amd.frame_offsets(b["csz"], b["off"])   # allocate scratch once
    # input blocks: generated on the device, copied to pinned host memory (untimed)
    for c in range(nch):
        lo, hi = c * ch, min(nb, (c + 1) * ch)
        amd.synth_blocks(bufs[0]["src"][:hi - lo], n, lo, kind)
        h_src[lo:hi].copy_(bufs[0]["src"][:hi - lo])
    torch.cuda.synchronize()

    # plain pinned copy rates over one chunk (the PCIe ceiling of both directions)
    probe = bufs[0]["src"]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    probe.copy_(h_src[:ch], non_blocking=True)
    ev[1].record()
    h_out[:ch].copy_(probe, non_blocking=True)
    ev[2].record()
    torch.cuda.synchronize()
    h2d = ch * n / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9
    d2h = ch * n / (ev[1].elapsed_time(ev[2]) * 1e-3) / 1e9

    def run_tx():
        chunk_frames = []        # (host byte offset, bytes, host copy of offsets)
        pos, pending = 0, None
        for c in range(nch + 1):
            if c < nch:
                lo, hi = c * ch, min(nb, (c + 1) * ch)
                b, s = bufs[c % NS], streams[c % NS]
                with torch.cuda.stream(s):
                    k = hi - lo
                    b["src"][:k].copy_(h_src[lo:hi], non_blocking=True)
                    amd.compress_batch(b["src"][:k], b["sizes"][:k], b["comp"][:k], b["csz"][:k],
                                       stream=s)
                    amd.frame_offsets(b["csz"][:k], b["off"][:k + 1], b["scratch"], stream=s)
                    amd.frame_pack(b["comp"][:k], b["csz"][:k], b["off"][:k + 1], b["frames"],
                                   stream=s)
                    b["tot"].copy_(b["off"][k:k + 1], non_blocking=True)
                    b["tev"] = torch.cuda.Event()
                    b["tev"].record(s)
            if pending is not None:      # issue the previous chunk's D2H once its size is known
                pc, pb, ps = pending
                pb["tev"].synchronize()
                t = int(pb["tot"].item())
                with torch.cuda.stream(ps):
                    h_frames[pos:pos + t].copy_(pb["frames"][:t], non_blocking=True)
                chunk_frames.append((pos, t))
                pos += t
            pending = (c, bufs[c % NS], streams[c % NS]) if c < nch else None
        torch.cuda.synchronize()
        return chunk_frames, pos

    def run_rx(chunk_frames, offs):
        for c in range(nch):
            lo, hi = c * ch, min(nb, (c + 1) * ch)
            k = hi - lo
            b, s = bufs[c % NS], streams[c % NS]
            fpos, t = chunk_frames[c]
            with torch.cuda.stream(s):
                b["frames"][:t].copy_(h_frames[fpos:fpos + t], non_blocking=True)
                b["off"][:k + 1].copy_(offs[c], non_blocking=True)
                amd.decompress_frames(b["frames"], b["off"], b["out"][:k], b["res"][:k],
                                      dst_caps=b["sizes"][:k], nblocks=k, stream=s)
                h_out[lo:hi].copy_(b["out"][:k], non_blocking=True)
        torch.cuda.synchronize()

    run_tx()                                   # warm-up
    t0 = time.perf_counter()
    chunk_frames, total = run_tx()
    t_tx = time.perf_counter() - t0
    # the receiver's frame offsets (from the headers; taken from the TX side, untimed)
    offs = []
    for c in range(nch):
        k = min(nb, (c + 1) * ch) - c * ch
        fpos, t = chunk_frames[c]
        o = np.zeros(k + 1, dtype=np.int64)
        fb = h_frames[fpos:fpos + t].numpy()
        p = 0
        for i in range(k):
            o[i] = p
            p += 4 + int(fb[p]) + (int(fb[p + 1]) << 8) + (int(fb[p + 2]) << 16) + (int(fb[p + 3]) << 24)
        o[k] = p
        offs.append(torch.from_numpy(o).pin_memory())
    run_rx(chunk_frames, offs)                 # warm-up
    t0 = time.perf_counter()
    run_rx(chunk_frames, offs)
    t_rx = time.perf_counter() - t0
    ok = bool(torch.equal(h_out, h_src))
    byt = nb * n
    line = {
        "metric": "LZ4 GiB/s end-to-end host->GPU->host (pinned H2D + kernels + D2H), socket path",
        "value": round(byt / (t_tx + t_rx) / GIB, 2), "unit": "GiB/s", "n_gpus": 1,
        "higher_is_better": True, "dtype": "u8",
        "data": "synthetic (SURVEY App. C gen_%s)" % args.kind,
        "config": {"workload": "%d x %d KiB blocks, chunks of %d over %d streams" % (
            nb, n >> 10, ch, NS)},
        "compress_e2e_GiBps": round(byt / t_tx / GIB, 2),
        "decompress_e2e_GiBps": round(byt / t_rx / GIB, 2),
        "framed_bytes": int(total), "ratio": round(byt / (total - 4 * nb), 4),
        "pcie_h2d_GBps": round(h2d, 1), "pcie_d2h_GBps": round(d2h, 1),
        "verified": ok,
    }
    print(json.dumps(line), flush=True)


def rand4k_bench(args):
    """BASELINE config 2: 256K x 4 KiB random blocks, decompress only, 1 MI355X.

    The blocks are generated (App. C gen_rand) and compressed once on the device
    (untimed; the reference emits 4114 bytes for every such block -- our encoder's
    sizes are reported beside it), then each step decodes all of them."""
    import torch

    import libapenetwork_amd as amd

    torch.cuda.set_device(0)
    if amd.gpu_init() != 0:
        raise SystemExit("GPU codec unavailable: %s" % amd.gpu_last_error())
    n, nb = 4096, args.rand4k_blocks
    slot = (amd.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, 0)
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.compress_batch(src, sizes, comp, csz)
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    res = torch.zeros(nb, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        amd.decompress_batch(comp, csz, out, res, dst_caps=sizes, stream=stream)
    torch.cuda.synchronize()
    steps = max(20, args.steps)   # (as the nested config-2 leg)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for e in evs:
        e[0].record(stream)
        amd.decompress_batch(comp, csz, out, res, dst_caps=sizes, stream=stream)
        e[1].record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ms = sum(a.elapsed_time(b) for a, b in evs) / steps
    ok = bool((res == n).all().item()) and bool(torch.equal(out, src))
    c = csz.to(torch.int64)
    cbytes = int(c.sum().item())
    alg = nb * n + cbytes
    line = {
        "metric": "LZ4 GiB/s decompress-only, 256K x 4 KiB random blocks (BASELINE config 2)",
        "value": round(nb * n / (wall) / GIB, 2), "unit": "GiB/s", "n_gpus": 1,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(wall * 1e3, 3),
        "higher_is_better": True, "dtype": "u8", "data": "synthetic (SURVEY App. C gen_rand)",
        "config": {"workload": "%d x 4 KiB random blocks, decompress only" % nb},
        "comp_bytes_min": int(c.min().item()), "comp_bytes_max": int(c.max().item()),
        "reference_comp_bytes": 4114, "verified": ok,
        "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "kernel": "lz4_decode_kernel", "bytes_per_launch": alg,
                     "avg_launch_ms": round(ms, 3)},
    }
    print(json.dumps(line), flush=True)


def cpu_stream_baseline(n, chunk, target_s):
    """Reference chained stream on host cores: compress_fast_continue +
    decompress_safe_continue per chunk, one stream per thread (oracle/cpu_bench.c)."""
    lib = C.CDLL(os.path.join(ROOT, "oracle", "libcpubench.so"))
    lib.cpu_stream_run.restype = C.c_int
    lib.cpu_stream_run.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_int, C.POINTER(C.c_double)]
    ref = os.path.join(ROOT, "oracle", "_ref", "libape_lz4_ref.so")
    if os.path.exists(ref):
        path, prefix, kindname = ref, b"APE_LZ4_", "reference"
    else:
        path, prefix, kindname = os.path.join(ROOT, "oracle", "liblz4_oracle.so"), b"orc_", "port"
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    out = (C.c_double * 5)()
    nb = 1024
    if lib.cpu_stream_run(path.encode(), prefix, threads, nb, n, chunk, 1, 1, out) != 0:
        return None
    per_block = (out[0] + out[1]) / nb
    nb = int(min(32768, max(1024, target_s / max(per_block, 1e-9) / 2)))
    reps = max(1, int(target_s / max(per_block * nb, 1e-9)))
    if lib.cpu_stream_run(path.encode(), prefix, threads, nb, n, chunk, 1, reps, out) != 0 or out[3]:
        return None
    tc, td, csz, bytes_ = out[0], out[1], out[2], out[4]
    return {
        "value": round(bytes_ * reps / (tc + td) / GIB, 3), "unit": "GiB/s", "cores": threads,
        "kind": kindname,
        "sample": "%d threads x one stream each over %d x 64 KiB compressible blocks in %d-byte "
                  "chunks x %d reps, compress_fast_continue + decompress_safe_continue, %.1f s" % (
                      threads, nb, chunk, reps, tc + td),
        "compress_GiBps": round(bytes_ * reps / tc / GIB, 3),
        "decompress_GiBps": round(bytes_ * reps / td / GIB, 3),
        "ratio": round(bytes_ / csz, 4),
    }


def stream_bench(args):
    """Chained-stream socket codec: many connections, 8 KiB chunks,
    each compressed against its stream's previous bytes (withPrefix) and decoded with
    them as dictionary (usingDict), device-resident, 1 MI355X.

    Connection b's stream is synthetic block b (64 KiB, App. C); its chunk j has the
    previous 8 KiB x j bytes of the stream as history (the GPU encoder uses up to
    65536 - 8192 of them).  A step = TX of all chunks + RX of all chunks."""
    import torch

    import libapenetwork_amd as amd

    torch.cuda.set_device(0)
    if amd.gpu_init() != 0:
        raise SystemExit("GPU codec unavailable: %s" % amd.gpu_last_error())
    n, ch, nb = 65536, args.stream_chunk, args.stream_blocks
    per = n // ch
    nc = nb * per
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, 1)
    cap = amd.compressBound(ch)
    slot = (cap + 15) // 16 * 16
    comp = torch.empty((nc, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    j = torch.arange(per, dtype=torch.int64, device="cuda").repeat(nb)
    b = torch.arange(nb, dtype=torch.int64, device="cuda").repeat_interleave(per)
    src_ptr = src.data_ptr() + b * n + j * ch
    dst_ptr = comp.data_ptr() + torch.arange(nc, dtype=torch.int64, device="cuda") * slot
    out_ptr = out.data_ptr() + b * n + j * ch
    sizes = torch.full((nc,), ch, dtype=torch.int32, device="cuda")
    caps = torch.full((nc,), cap, dtype=torch.int32, device="cuda")
    pre = (j * ch).to(torch.int32)                 # history = the stream so far
    dict_ptr = src.data_ptr() + b * n               # RX dictionary: the same bytes
    csz = torch.zeros(nc, dtype=torch.int32, device="cuda")
    res = torch.zeros(nc, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def tx():
        amd.compress_prefix_batch(src_ptr, sizes, pre, dst_ptr, caps, csz, stream=stream)

    def rx():
        amd.decompress_dict_batch(dst_ptr, csz, out_ptr, sizes, dict_ptr, pre, res, stream=stream)

    for _ in range(args.warmup):
        tx()
        rx()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for e in ev:
        e[0].record(stream)
        tx()
        e[1].record(stream)
        rx()
        e[2].record(stream)
    torch.cuda.synchronize()
    tx_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    rx_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps
    ok = bool((res == ch).all().item()) and bool(torch.equal(out, src))
    cbytes = int(csz.to(torch.int64).sum().item())
    cpu = None if args.no_cpu_baseline else cpu_stream_baseline(n, ch, args.cpu_seconds)
    line = {
        "metric": "LZ4 GiB/s chained-stream socket codec (withPrefix TX + usingDict RX), "
                  "%d-byte chunks" % ch,
        "value": round(nb * n / ((tx_ms + rx_ms) * 1e-3) / GIB, 2), "unit": "GiB/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(tx_ms + rx_ms, 3), "higher_is_better": True, "dtype": "u8",
        "data": "synthetic (SURVEY App. C gen_comp, one stream per block)",
        "config": {"workload": "%d connections x 64 KiB streams = %d chunks of %d B, history "
                               "up to 64 KiB" % (nb, nc, ch)},
        "tx_ms": round(tx_ms, 3), "rx_ms": round(rx_ms, 3),
        "tx_GiBps": round(nb * n / (tx_ms * 1e-3) / GIB, 2),
        "rx_GiBps": round(nb * n / (rx_ms * 1e-3) / GIB, 2),
        "ratio": round(nb * n / cbytes, 4), "verified": ok, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


def sock_leg(args):
    """BASELINE config 5 through a real byte path: loopback TCP connections.

    Per connection, a TX thread: APE_LZ4_socket_send_blocks -- host blocks --H2D--> encode
    --> frames --D2H--> write(); an RX thread: APE_LZ4_socket_recv_blocks -- read() into the
    pinned growable rxbuf (the ape_buffer analogue) --> frame parser (K7 rewritten) --H2D-->
    decode from the frames --D2H--> host blocks.  Both sides double-buffer, so the socket
    I/O of one batch overlaps the GPU work of the next.  The blocks are split contiguously
    over --sock-conns connections (a server's sockets share one GPU); the one-connection run
    is reported beside it.  Rate = uncompressed bytes / wall time from the first send to the
    last received block; every block is compared."""
    import socket
    import threading

    import torch

    import libapenetwork_amd as amd

    torch.cuda.set_device(0)
    if amd.gpu_init() != 0:
        raise SystemExit("GPU codec unavailable: %s" % amd.gpu_last_error())
    n, nb, batch = args.block_size, args.sock_blocks, args.sock_batch
    kind = 1 if args.kind == "comp" else 0
    h_src = torch.empty((nb, n), dtype=torch.uint8, pin_memory=True)
    h_dst = torch.zeros((nb, n), dtype=torch.uint8, pin_memory=True)
    res = np.zeros(nb, dtype=np.int32)
    g = torch.empty((min(nb, 8192), n), dtype=torch.uint8, device="cuda")
    for lo in range(0, nb, g.shape[0]):
        k = min(g.shape[0], nb - lo)
        amd.synth_blocks(g[:k], n, lo, kind)
        h_src[lo:lo + k].copy_(g[:k])
    torch.cuda.synchronize()
    del g
    src_np, dst_np = h_src.numpy(), h_dst.numpy()

    def run(k, conns):
        """k blocks over `conns` connections (contiguous shares), a TX and an RX thread each."""
        pairs = []
        for _ in range(conns):
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind(("127.0.0.1", 0))
            srv.listen(1)
            tx = socket.create_connection(srv.getsockname())
            rx, _ = srv.accept()
            srv.close()
            for s_ in (tx, rx):
                s_.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
                s_.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
            pairs.append((tx, rx))
        cut = [k * c // conns for c in range(conns + 1)]
        out = [{} for _ in range(conns)]

        def txf(c):
            tx, lo, hi = pairs[c][0], cut[c], cut[c + 1]
            try:
                out[c]["sent"] = amd.socket_send_blocks(tx.fileno(), src_np[lo:hi], n, batch)
            except Exception as e:   # reported below
                out[c]["err"] = e
            finally:
                tx.shutdown(socket.SHUT_WR)

        def rxf(c):
            rx, lo, hi = pairs[c][1], cut[c], cut[c + 1]
            try:
                out[c]["got"] = amd.socket_recv_blocks(rx.fileno(), dst_np[lo:hi], n, batch,
                                                       res[lo:hi])
            except Exception as e:
                out[c]["err"] = e

        ths = [threading.Thread(target=f, args=(c,)) for c in range(conns) for f in (txf, rxf)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        wall = time.perf_counter() - t0
        for tx, rx in pairs:
            tx.close()
            rx.close()
        for o in out:
            if "err" in o:
                raise o["err"]
        return wall, sum(o["got"] for o in out), sum(o["sent"] for o in out)

    def measure(conns):
        h_dst.zero_()
        res[:] = -9
        amd.socket_stats(reset=True)
        wall, got, wire = run(nb, conns)
        split = amd.socket_stats(reset=True)
        ok = got == nb and bool((res == n).all()) and bool(torch.equal(h_dst, h_src))
        # the same wire bytes through as many connections without the codec
        ceiling, ceiling_cold = sock_ceilings(int(wire), conns)
        r = {"value": round(nb * n / wall / GIB, 3), "connections": conns,
             "wall_s": round(wall, 3), "wire_bytes": int(wire),
             "ratio": round(nb * n / (wire - 4 * nb), 4),
             "wire_GBps": round(wire / wall / 1e9, 3), "verified": ok,
             "ceiling_GBps": ceiling, "ceiling_cold_GBps": ceiling_cold,
             "wire_frac_of_ceiling": round(wire / wall / 1e9 / ceiling, 3) if ceiling else None,
             "wire_frac_of_cold_ceiling": (round(wire / wall / 1e9 / ceiling_cold, 3)
                                           if ceiling_cold else None),
             "split_ms": split}
        r["bound"] = ("socket" if ceiling_cold and r["wire_GBps"] >= 0.8 * ceiling_cold
                      else "pipeline")
        return r

    conns = max(1, args.sock_conns)
    run(min(nb, 2 * batch * conns), conns)      # warm-up (kernels, allocations)
    main = measure(conns)
    one = measure(1) if conns > 1 else None
    cpu = None if args.no_cpu_baseline else cpu_sock_baseline(n)
    line = {
        "metric": "LZ4 GiB/s through loopback TCP sockets (GPU encode -> frames -> socket -> "
                  "pinned rxbuf -> GPU decode), BASELINE config 5",
        "value": main["value"], "unit": "GiB/s", "n_gpus": 1,
        "higher_is_better": True, "dtype": "u8",
        "data": "synthetic (SURVEY App. C gen_%s)" % args.kind,
        "config": {"workload": "%d x %d KiB blocks over %d 127.0.0.1 TCP connection(s) (a TX and "
                               "an RX thread each, contiguous shares), %d blocks per GPU batch" % (
                                   nb, n >> 10, conns, batch)},
        **{k: v for k, v in main.items() if k != "value"},
        "ceiling": "plain bytes over as many 127.0.0.1 TCP connections in parallel, 4 MiB "
                   "write()s / read()s, no codec, same wire bytes (oracle/cpu_bench.c "
                   "sock_ceiling_buf): ceiling_GBps with one 4 MiB buffer per side (cache-hot), "
                   "ceiling_cold_GBps walking 1 GiB buffers (every syscall copies cache-cold "
                   "memory, as the codec path's do: its frames arrive by DMA and its receive "
                   "buffer is read by DMA)",
        "split_note": "summed over the connections; GPU phases from timing events per batch (they "
                      "overlap each other and the socket I/O: double-buffered); write/read = time "
                      "in the syscalls; gpu_wait = host blocked on the GPU",
        "one_connection": one,
        "cpu_baseline": cpu,
    }
    return line


def sock_ceilings(nbytes, conns=1):
    """(hot, cold) plain-bytes loopback rates in GB/s for nbytes over `conns` connections in
    parallel (oracle/cpu_bench.c; one thread pair per connection, ctypes releases the GIL):
    total bytes / the slowest connection's time."""
    import threading
    try:
        cb = C.CDLL(os.path.join(ROOT, "oracle", "libcpubench.so"))
        cb.sock_ceiling_buf.argtypes = [C.c_longlong, C.c_int, C.c_longlong, C.POINTER(C.c_double)]
        res = []
        for buf in (4 << 20, 1 << 30):
            outs = [(C.c_double * 2)() for _ in range(conns)]
            rcs = [None] * conns
            per = max(4 << 20, nbytes // conns)

            def one(c):
                rcs[c] = cb.sock_ceiling_buf(per, 4 << 20, buf, outs[c])

            ths = [threading.Thread(target=one, args=(c,)) for c in range(conns)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            ok = all(r == 0 for r in rcs)
            res.append(round(sum(o[1] for o in outs) / max(o[0] for o in outs) / 1e9, 3)
                       if ok else None)
        return tuple(res)
    except OSError:
        return None, None


def sock_chained_leg(args):
    """The reference wire format through the GPU over many sockets (VERDICT r3
    item 6): M loopback TCP connections, each a chained stream exactly as ape_socket writes it
    (64 KiB messages in 8 KiB chunks, each compressed against the stream's previous <= 64 KiB,
    [int32 size][block] frames; ref src/ape_socket.c:811-871) and reads it (decompress against
    the last 64 KiB, :1333-1467).  TX thread: APE_LZ4_chain_send -- per round one message per
    connection, all chunks in one withPrefix launch, frames written to each socket.  RX (this
    thread): APE_LZ4_chain_recv -- poll + split-safe parser per connection, per round nch
    usingDict launches of M blocks.  Every byte is compared.  Beside it: the reference's own
    socket codec on the same number of connections (oracle/cpu_bench.c cpu_sock_run)."""
    import socket
    import threading

    import torch

    import libapenetwork_amd as amd

    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = 4 * args.chain_conns + 256        # GPU and reference legs: 2 fds per connection each
    if soft < want:
        resource.setrlimit(resource.RLIMIT_NOFILE, (min(want, hard), hard))
    torch.cuda.set_device(0)
    if amd.gpu_init() != 0:
        raise SystemExit("GPU codec unavailable: %s" % amd.gpu_last_error())
    M, nmsg, n = args.chain_conns, args.chain_msgs, 65536
    h_msgs = torch.empty((nmsg, M, n), dtype=torch.uint8, pin_memory=True)
    h_out = torch.zeros((nmsg, M, n), dtype=torch.uint8, pin_memory=True)
    g = torch.empty((M, n), dtype=torch.uint8, device="cuda")
    for m in range(nmsg):   # App. C gen_comp, connection i's message m = block m * M + i (untimed)
        amd.synth_blocks(g, n, m * M, 1)
        h_msgs[m].copy_(g)
    torch.cuda.synchronize()
    del g
    msgs, out = h_msgs.numpy(), h_out.numpy()
    status = np.zeros(M, dtype=np.int32)

    def pairs():
        ps = []
        for _ in range(M):
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(1)
            t = socket.create_connection(srv.getsockname())
            r, _ = srv.accept()
            srv.close()
            for s_ in (t, r):
                s_.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
                s_.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
            ps.append((t, r))
        return ps

    def run(k):
        ps = pairs()
        tx, rx = amd.Chain(M, n), amd.Chain(M, n)
        res = {}

        def txf():
            try:
                res["wire"] = tx.send([t.fileno() for t, _ in ps], msgs[:k])
            except Exception as e:
                res["err"] = e
            finally:
                for t, _ in ps:
                    t.shutdown(socket.SHUT_WR)

        t0 = time.perf_counter()
        th = threading.Thread(target=txf)
        th.start()
        got = rx.recv([r.fileno() for _, r in ps], out[:k], status)
        th.join()
        wall = time.perf_counter() - t0
        for t, r in ps:
            t.close()
            r.close()
        tx.free()
        rx.free()
        if "err" in res:
            raise res["err"]
        return wall, got, res["wire"]

    run(min(nmsg, 2))               # warm-up
    h_out.zero_()
    amd.socket_stats(reset=True)
    wall, got, wire = run(nmsg)
    split = amd.socket_stats(reset=True)
    ok = got == nmsg * M * n and bool((status == 0).all()) and bool(torch.equal(h_out, h_msgs))
    payload = nmsg * M * n
    cpu = None
    if not args.no_cpu_baseline:
        lib = C.CDLL(os.path.join(ROOT, "oracle", "libcpubench.so"))
        lib.cpu_sock_run2.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, C.POINTER(C.c_double)]
        ref = os.path.join(ROOT, "oracle", "_ref", "libape_lz4_ref.so")
        path, prefix, kind = ((ref, b"APE_LZ4_", "reference") if os.path.exists(ref) else
                              (os.path.join(ROOT, "oracle", "liblz4_oracle.so"), b"orc_", "port"))
        o = (C.c_double * 4)()
        cmsg = max(4, args.chain_cpu_bytes // (M * n))
        usable, cores = host_cores()
        if lib.cpu_sock_run2(path.encode(), prefix, M, n, cmsg, 1, usable, o) == 0 and o[3] == 0:
            cpu = {"value": round(o[1] / o[0] / GIB, 3), "unit": "GiB/s", "cores": usable,
                   "kind": kind, "connections": M, "threads": 2 * min(usable, M),
                   "wire_GBps": round(o[2] / o[0] / 1e9, 3), "seconds": round(o[0], 2),
                   "sample": "the same %d connections x %d x 64 KiB App. C messages through the "
                             "reference socket codec (compress_fast_continue + saveDict / "
                             "decompress_safe_continue + 64 KiB ring), an event loop per usable "
                             "core: %d TX and %d RX threads, each serving every %d-th connection "
                             "(poll); generated before and compared after the clock" % (
                                 M, cmsg, min(usable, M), min(usable, M), min(usable, M)),
                   "host": cores}
    ceiling, ceiling_cold = sock_ceilings(int(wire))
    return {
        "metric": "LZ4 GiB/s, the reference socket wire format (chained 8 KiB blocks) through the "
                  "GPU over %d loopback TCP connections" % M,
        "value": round(payload / wall / GIB, 3), "unit": "GiB/s", "n_gpus": 1,
        "higher_is_better": True, "dtype": "u8",
        "data": "synthetic (SURVEY App. C gen_comp), one 64 KiB message per connection per round",
        "config": {"workload": "%d connections x %d x 64 KiB messages = %.2f GiB, 8 KiB chained "
                               "chunks, [int32 size][block] frames" % (M, nmsg, payload / GIB)},
        "wall_s": round(wall, 3), "wire_bytes": int(wire), "ratio": round(payload / (wire - 4 * nmsg * M * 8), 4),
        "wire_GBps": round(wire / wall / 1e9, 3), "verified": ok,
        "ceiling_GBps": ceiling, "ceiling_cold_GBps": ceiling_cold,
        "ceiling": "plain bytes over one 127.0.0.1 TCP connection, 4 MiB write()s (sock_ceiling_buf), "
                   "same wire bytes; hot: one 4 MiB buffer per side, cold: 1 GiB buffers",
        "split_ms": {k: v for k, v in split.items() if k in (
            "tx_write_ms", "tx_gpu_wait_ms", "tx_batches", "tx_total_ms", "rx_total_ms",
            "rx_read_ms", "rx_parse_ms", "rx_gpu_wait_ms", "rx_batches")},
        "split_note": "rx_read_ms = poll + read() until every connection holds a round; "
                      "rx_parse_ms = payload staging; rx_gpu_wait_ms = waiting on round m - 2",
        "cpu_baseline": cpu,
    }


def sock_chained_bench(args):
    print(json.dumps(sock_chained_leg(args)), flush=True)


def cpu_sock_baseline(n):
    """The reference's own socket codec over loopback TCP on this host's cores (BASELINE
    config 5; oracle/cpu_bench.c cpu_sock_run: ape_socket.c's TX -- 8 KiB blocks with
    compress_fast_continue + saveDict -- and RX -- decompress_safe_continue against the 64 KiB
    dictionary buffer -- without the event loop): one connection (a TX and an RX thread,
    as one event loop would serve it) and usable/2 connections in parallel."""
    lib = C.CDLL(os.path.join(ROOT, "oracle", "libcpubench.so"))
    lib.cpu_sock_run.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.POINTER(C.c_double)]
    ref = os.path.join(ROOT, "oracle", "_ref", "libape_lz4_ref.so")
    if os.path.exists(ref):
        path, prefix, kind = ref, b"APE_LZ4_", "reference"
    else:
        path, prefix, kind = os.path.join(ROOT, "oracle", "liblz4_oracle.so"), b"orc_", "port"
    usable, cores = host_cores()
    out = (C.c_double * 4)()
    res = {}
    for label, nconn, nmsg in (("one_connection", 1, 16384), ("all_cores", max(1, usable // 2), 4096)):
        if lib.cpu_sock_run(path.encode(), prefix, nconn, n, nmsg, 1, out) != 0 or out[3] != 0:
            return None
        res[label] = {"value": round(out[1] / out[0] / GIB, 3), "connections": nconn,
                      "wire_GBps": round(out[2] / out[0] / 1e9, 3), "seconds": round(out[0], 2)}
    return {"value": res["one_connection"]["value"], "unit": "GiB/s", "cores": 2, "kind": kind,
            "sample": "1 connection x %d x 64 KiB App. C messages (1 TX + 1 RX thread); also "
                      "%d connections x 4096 messages on %d threads" % (
                          16384, res["all_cores"]["connections"], 2 * res["all_cores"]["connections"]),
            "host": cores, **res}


def sock_bench(args):
    print(json.dumps(sock_leg(args)), flush=True)


def sq_issue(kernel):
    """Instruction-issue occupancy of `kernel` from the committed SQ PMC passes
    (profiles/sq_issue.json, PROFILE-DERIVED): the binding resource of this integer
    byte-shuffling path is instruction issue, not HBM."""
    p = os.path.join(ROOT, "profiles", "sq_issue.json")
    try:
        d = json.load(open(p))[kernel]
        return {"pipe": "valu", "busy": d["valu_pipe_busy"], "salu_busy": d["salu_busy"],
                "source": "profiles/sq_issue.json (profile-derived)"}
    except Exception:
        return None


def config2_leg(args, amd, torch, stream):
    """BASELINE config 2 inside the default run: 262144 x 4 KiB random blocks, decompress
    only, 1 MI355X.  The blocks are compressed by the reference algorithm -- the product's
    host codec (ape_lz4_host.c, byte-identical to src/ape_lz4.c's compress_default on the
    golden KATs) -- on the host, untimed, so the GPU decodes the reference's 4114-byte blocks,
    not its own encoder's.  Timed: the decode kernel over all blocks, device-resident."""
    n, nb = 4096, args.config2_blocks
    L = amd.lib()
    f = L.hst_compress_extstate
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, 0)
    host = src.cpu().numpy()
    cap = amd.compressBound(n)
    slot = (cap + 15) // 16 * 16
    comp_h = np.zeros((nb, slot), dtype=np.uint8)
    csz_h = np.zeros(nb, dtype=np.int32)
    state = C.create_string_buffer(16416)
    t0 = time.time()
    base_in, base_out = host.ctypes.data, comp_h.ctypes.data
    for b in range(nb):
        csz_h[b] = f(state, base_in + b * n, base_out + b * slot, n, cap, 1)
    log("[config2] %d blocks compressed by the host (reference) codec in %.1f s" % (
        nb, time.time() - t0))
    comp = torch.from_numpy(comp_h).cuda()
    csz = torch.from_numpy(csz_h).cuda()
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    res = torch.zeros(nb, dtype=torch.int32, device="cuda")
    for _ in range(max(1, args.warmup)):
        amd.decompress_batch(comp, csz, out, res, dst_caps=sizes, stream=stream)
    torch.cuda.synchronize()
    steps = max(20, args.steps)   # a 0.4 ms kernel: enough steps that launch jitter averages out
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        e[0].record(stream)
        amd.decompress_batch(comp, csz, out, res, dst_caps=sizes, stream=stream)
        e[1].record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ms = sum(a.elapsed_time(b) for a, b in evs) / steps
    ok = bool((res == n).all().item()) and bool(torch.equal(out, src))
    cbytes = int(csz_h.astype(np.int64).sum())
    alg = nb * n + cbytes
    value = nb * n / wall / GIB
    rd_bound = HBM_PEAK_GBPS * 1e9 / GIB * (nb * n) / cbytes   # read-only: c bytes per block
    return {
        "metric": "LZ4 GiB/s decompress-only, 256K x 4 KiB random blocks (BASELINE config 2)",
        "value": round(value, 2), "unit": "GiB/s", "steps": steps,
        "ms_per_step": round(wall * 1e3, 3),
        "config": {"workload": "%d x 4 KiB random blocks (SURVEY App. C gen_rand), compressed "
                               "by the reference algorithm on the host, decompress only" % nb},
        "comp_bytes_min": int(csz_h.min()), "comp_bytes_max": int(csz_h.max()),
        "reference_comp_bytes": 4114, "verified": ok,
        "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "kernel": "lz4_decode_kernel", "bytes_per_launch": alg,
                     "avg_launch_ms": round(ms, 3),
                     "hbm_read_roofline_GiBps": round(rd_bound, 1),
                     "hbm_read_frac": round(value / rd_bound, 4)},
    }


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N` without a launcher: start N ranks of this script (one process per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set) and exit with their status.
    Nothing here loads torch or the HIP runtime: the devices are counted from the KFD
    topology in sysfs (sharding.visible_gpu_count), so the children start from a process
    that never touched a GPU (tests/test_multigpu.py checks this).  Rank 0's stdout is this
    process's stdout (the one JSON line); the other ranks' stdout goes to stderr."""
    import signal

    from libapenetwork_amd.sharding import launch_plan, visible_gpu_count
    try:
        plan = launch_plan(args.gpus, args.blocks, visible_gpu_count(),
                           os.environ.get("APE_BENCH_DEVICE"), args.weak, _free_port())
    except ValueError as e:
        log("bench.py: %s (set APE_BENCH_DEVICE=<id> to rehearse N ranks on one device)" % e)
        return 2
    procs = []
    for p in plan:
        env = dict(os.environ)
        env.update(p["env"])
        log("[launch] rank %d on device %d: blocks [%d, %d)" % (
            p["rank"], p["device"], p["first_block"], p["first_block"] + p["nblocks"]))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] +
                                      sys.argv[1:], env=env,
                                      stdout=None if p["rank"] == 0 else sys.stderr.fileno()))
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                log("bench.py: rank pid %d exited with %d; stopping the others" % (pr.pid, code))
                for other in live:
                    other.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.2)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--blocks", type=int, default=1 << 20,
                    help="total blocks of the job, split contiguously over the ranks "
                         "(BASELINE config 4); per rank with --weak")
    ap.add_argument("--weak", action="store_true", help="--blocks per rank (weak scaling)")
    ap.add_argument("--block-size", type=int, default=65536)
    ap.add_argument("--kind", choices=["comp", "rand"], default="comp")
    ap.add_argument("--cpu-blocks", type=int, default=65536,
                    help="CPU-baseline sample (65536 x 64 KiB = 4 GiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config2", action="store_true")
    ap.add_argument("--no-config5", action="store_true")
    ap.add_argument("--config2-blocks", type=int, default=1 << 18)
    ap.add_argument("--verify-sample", type=int, default=64)
    ap.add_argument("--e2e", action="store_true",
                    help="host->GPU->host socket-path rate instead of the device-resident line")
    ap.add_argument("--e2e-blocks", type=int, default=1 << 17)
    ap.add_argument("--e2e-chunk", type=int, default=1 << 13)
    ap.add_argument("--e2e-streams", type=int, default=3)
    ap.add_argument("--rand4k", action="store_true",
                    help="BASELINE config 2 alone: decompress-only over 4 KiB random blocks")
    ap.add_argument("--rand4k-blocks", type=int, default=1 << 18)
    ap.add_argument("--stream", action="store_true",
                    help="chained-stream socket codec (withPrefix TX + usingDict RX)")
    ap.add_argument("--stream-blocks", type=int, default=1 << 17)
    ap.add_argument("--stream-chunk", type=int, default=8192)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--sock", action="store_true",
                    help="config 5: loopback TCP socket TX/RX through the GPU codec")
    ap.add_argument("--sock-blocks", type=int, default=1 << 17,
                    help="config 5 sample (131072 x 64 KiB = 8 GiB)")
    ap.add_argument("--sock-batch", type=int, default=2048)
    ap.add_argument("--sock-conns", type=int, default=1,
                    help="config 5: loopback connections in parallel (a TX and an RX thread each)")
    ap.add_argument("--sock-chained", action="store_true",
                    help="the reference wire format (chained 8 KiB blocks) over many sockets")
    ap.add_argument("--chain-conns", type=int, default=512)
    ap.add_argument("--chain-msgs", type=int, default=64,
                    help="64 KiB messages per connection (512 x 64 x 64 KiB = 2 GiB)")
    ap.add_argument("--chain-cpu-bytes", type=int, default=1 << 30,
                    help="payload of the reference socket-codec baseline run")
    args = ap.parse_args()
    if args.e2e:
        return e2e_bench(args)
    if args.sock:
        return sock_bench(args)
    if args.sock_chained:
        return sock_chained_bench(args)
    if args.stream:
        return stream_bench(args)
    if args.rand4k:
        return rand4k_bench(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args)

    import torch

    import libapenetwork_amd as amd
    from libapenetwork_amd.sharding import gather, reduce_max, reduce_sum, shard, shard_strong

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log("bench.py: --gpus %d but WORLD_SIZE=%d (the launcher's rank count)" % (args.gpus,
                                                                                world))
        return 2
    if os.environ.get("APE_BENCH_DEVICE") is None and torch.cuda.device_count() < world:
        log("bench.py: %d ranks but only %d device(s) visible" % (world,
                                                                 torch.cuda.device_count()))
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # APE_BENCH_DEVICE (rehearsal only): every rank on that device, to exercise the N > 1
    # path on a one-GPU box; the driver's multi-GPU runs leave it unset
    dev = os.environ.get("APE_BENCH_DEVICE")
    torch.cuda.set_device(int(dev) if dev is not None else local)
    dist = None
    if world > 1:
        # no collective on the data path: the process group (gloo, host scalars) carries
        # only the barrier, the max-over-ranks time and the per-rank numbers
        import torch.distributed as dist
        # gloo's C++ connect messages go to stdout; keep rank 0's stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    rc = amd.gpu_init()
    if rc != 0:
        raise SystemExit("GPU codec unavailable: %s" % amd.gpu_last_error())

    n = args.block_size
    if args.weak:
        first, nb = shard(rank, world, args.blocks)
        total_blocks = args.blocks * world
    else:
        first, nb = shard_strong(rank, world, args.blocks)
        total_blocks = args.blocks
    kind = 1 if args.kind == "comp" else 0
    slot = (amd.compressBound(n) + 15) // 16 * 16
    stream = torch.cuda.current_stream()
    log("[rank %d] blocks [%d, %d) of %d: allocating %.1f GiB (in %d x %d, slots %d)" % (
        rank, first, first + nb, total_blocks, nb * (2 * n + slot) / GIB, nb, n, slot))
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    dres = torch.zeros(nb, dtype=torch.int32, device="cuda")

    t0 = time.time()
    chunk = 1 << 16
    for b0 in range(0, nb, chunk):
        amd.synth_blocks(src[b0:b0 + chunk], n, first + b0, kind)
        torch.cuda.synchronize()
        log("[rank %d] synth %d/%d blocks (%.0f s)" % (rank, min(b0 + chunk, nb), nb,
                                                        time.time() - t0))

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        amd.compress_batch(src, sizes, comp, csz, stream=stream)
        if ev:
            ev[1].record(stream)
        amd.decompress_batch(comp, csz, out, dres, dst_caps=sizes, stream=stream)
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    # poison every output of the step before the timed region, so the verification below
    # can only pass on bytes, sizes and results that the timed steps themselves produced
    comp.fill_(0xA5)
    out.fill_(0x5A)
    csz.fill_(-1)
    dres.fill_(-7)
    torch.cuda.synchronize()

    evs =[[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    mine = time.perf_counter() - t_start       # this rank's own time
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    elapsed = reduce_max(dist, elapsed)

    # ---- correctness + ratio (outside the timed region) ----
    ok = bool((dres == n).all().item())
    for b0 in range(0, nb, 1 << 14):  # chunked: a whole-tensor compare would need 64 GiB
        ok = ok and bool(torch.equal(out[b0:b0 + (1 << 14)], src[b0:b0 + (1 << 14)]))
    comp_bytes = int(csz.to(torch.int64).sum().item())
    sample_ok = None
    if rank == 0 and args.verify_sample > 0:
        try:
            orc = C.CDLL(os.path.join(ROOT, "oracle", "liblz4_oracle.so"))
            idx = torch.linspace(0, nb - 1, args.verify_sample).long()
            cs = csz[idx].cpu().tolist()
            cb = comp[idx].cpu().numpy()
            sb = src[idx].cpu().numpy()
            sample_ok = True
            for j in range(len(cs)):
                blk = cb[j, :cs[j]].tobytes()
                ob = C.create_string_buffer(n + 64)
                r = orc.orc_decompress_safe(C.create_string_buffer(blk + b"\0" * 16, len(blk) + 16),
                                            ob, len(blk), n)
                sample_ok &= (r == n and ob.raw[:n] == sb[j].tobytes())
        except OSError:
            sample_ok = None
    per_rank = gather(dist, {"rank": rank, "blocks": nb, "first_block": first,
                             "GiBps": round(nb * n / (mine / args.steps) / GIB, 2),
                             "ms_per_step": round(mine / args.steps * 1e3, 3),
                             "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3)},
                      world)
    comp_total, nok = reduce_sum(dist, [comp_bytes, int(ok)])
    ok = nok == world

    total_bytes = total_blocks * n
    ms_step = elapsed / args.steps * 1e3
    value = total_bytes / (elapsed / args.steps) / GIB
    ratio = total_bytes / max(comp_total, 1)

    # ---- roofline (rank 0's kernels; algorithmic bytes) ----
    # encode: read n + write c per block; decode: read c + write n per block.
    alg = nb * n + comp_bytes
    enc_gbps = alg / (enc_ms * 1e-3) / 1e9
    dec_gbps = alg / (dec_ms * 1e-3) / 1e9
    enc_dom = enc_ms >= dec_ms
    dom = "lz4_encode_kernel" if enc_dom else "lz4_decode_kernel"
    traffic, tsrc = pmc_traffic(dom, nb)
    step_s = ms_step * 1e-3
    step_rw = 2 * (total_bytes + comp_total) / step_s / 1e9        # R+W of a round trip
    step_rd = (total_bytes + comp_total) / step_s / 1e9            # reads only
    # the north_star's "HBM-read roofline" in uncompressed GiB/s: a round trip reads
    # n + c bytes per block, so HBM read peak x n / (n + c) bounds `value` (per GPU)
    read_bound = HBM_PEAK_GBPS * 1e9 / GIB * total_bytes / (total_bytes + comp_total) * world
    roof = {"bound": "hbm", "achieved": round(enc_gbps if enc_dom else dec_gbps, 1),
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round((enc_gbps if enc_dom else dec_gbps) / HBM_PEAK_GBPS, 4),
            "traffic": traffic, "traffic_source": "profile-derived per block x blocks: %s" % tsrc,
            "kernel": dom, "bytes_per_launch": int(alg),
            "avg_launch_ms": round(enc_ms if enc_dom else dec_ms, 3),
            "issue": sq_issue(dom),
            "decoder": {"kernel": "lz4_decode_kernel", "achieved": round(dec_gbps, 1),
                        "frac": round(dec_gbps / HBM_PEAK_GBPS, 4), "avg_launch_ms": round(dec_ms, 3)},
            "encoder": {"kernel": "lz4_encode_kernel", "achieved": round(enc_gbps, 1),
                        "frac": round(enc_gbps / HBM_PEAK_GBPS, 4), "avg_launch_ms": round(enc_ms, 3)},
            "step": {"achieved_GBps": round(step_rw, 1),
                     "frac": round(step_rw / (HBM_PEAK_GBPS * world), 4),
                     "read_GBps": round(step_rd, 1),
                     "read_frac": round(step_rd / (HBM_PEAK_GBPS * world), 4),
                     "basis": "sum(n + c) x 2 (R+W) / step time, all ranks, vs 8 TB/s x GPUs"}}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # after every rank's timed region (the gather above is a rendezvous), so at N > 1 the
        # reference's host run competes with no rank's GPU work; the other ranks only exit
        cpu = cpu_baseline(n, kind, args.cpu_blocks)
        if cpu is not None and world > 1:
            cpu["note"] = ("timed by rank 0 after every rank's timed steps (the other %d "
                           "ranks are exiting)" % (world - 1))
    c2 = None
    if rank == 0 and world == 1 and not args.no_config2:
        del src, comp, out
        torch.cuda.empty_cache()
        c2 = config2_leg(args, amd, torch, stream)
        if not args.no_cpu_baseline:
            c2["cpu_baseline"] = cpu_baseline(4096, 0, args.config2_blocks, mode=1,
                                              min_seconds=1.0, repeats=3)

    c5 = None
    if rank == 0 and world == 1 and not args.no_config5:
        try:
            torch.cuda.empty_cache()
            c5 = sock_leg(args)
        except Exception as e:   # the socket leg never masks the headline line
            c5 = {"error": repr(e)}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (SURVEY App. C gen_%s, seed = block id, generated on device)"
                    % args.kind,
            "config": {"workload": "%d x %d KiB %s blocks %s, compress+decompress" % (
                           total_blocks, n >> 10, "compressible" if kind else "random",
                           ("(%d per GPU)" % nb) if args.weak else "sharded over %d GPU" % world),
                       "total_blocks": total_blocks, "blocks_per_gpu": nb, "block_bytes": n,
                       "parallelism": "blocks%d" % world},
            "ratio": round(ratio, 4),
            "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
            "encode_GBps": round(enc_gbps, 1), "decode_GBps": round(dec_gbps, 1),
            "hbm_read_roofline": {"bound_GiBps": round(read_bound, 1),
                                  "frac": round(value / read_bound, 4)},
            "per_gpu": per_rank,
            "verified": bool(ok), "oracle_sample_ok": sample_ok,
            "roofline": roof, "cpu_baseline": cpu, "config2": c2, "config5": c5,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
