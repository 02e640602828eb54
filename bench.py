#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): device-resident GiB/s of LZ4 block
decompression, 4 MiB blocks, 4096 blocks in HBM per GPU (configs[1]).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

A step = one launch of the LZ4 decode kernel over the rank's whole batch.
Blocks are independent, so ranks shard them with no data-path collective
(weak scaling: every rank decodes its own 4096 blocks); torch.distributed is
used only for the barrier and the max-over-ranks time.  Inputs are synthetic
text-like blocks generated on the GPU and compressed by the GPU
encoder (byte-identical to LZ4_compress_default) before timing; the decoded
output is checked against the original on the device after timing.

Extra fields: roofline (HIP-event timed kernel, algorithmic bytes C+U per
launch vs 8 TB/s; traffic from profiles/traffic.json), cpu_baseline (the CPU
oracle on this host's cores, bounded sample), cpu_liblz4 (the C library
pkg/compress wraps, same sample), and with --host-path the PCIe-inclusive rate
through the C ABI's batch API (kept out of the default run so that every
decode launch in a default run is the headline launch).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from juicefs_amd import shard as S  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--blocks", type=int, default=4096)
    p.add_argument("--block-bytes", type=int, default=4 << 20)
    p.add_argument("--cls", default="T")
    p.add_argument("--codec", default="lz4", choices=["lz4", "zstd"],
                   help="lz4 = headline (configs[1]); zstd = level-3 decode (configs[3])")
    p.add_argument("--level", type=int, default=3, help="zstd level of the generated frames")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--host-path", action="store_true", help="(default) time the PCIe-inclusive batch path")
    p.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive batch path")
    p.add_argument("--host-blocks", type=int, default=2048, help="blocks in the --host-path sample")
    p.add_argument("--no-extras", action="store_true", help="skip the compress-side measurements")
    p.add_argument("--no-mixed", action="store_true", help="skip configs[4] (mixed LZ4/Zstd 64 KiB-4 MiB, host path)")
    p.add_argument("--mixed-blocks", type=int, default=4096)
    p.add_argument("--extra-blocks", type=int, default=1024, help="blocks in the Zstd compress sample")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="wall budget per CPU baseline leg")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return p.parse_args()


def host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # the GPU box's CPU share is 16


def cpu_baseline(comp_blocks, U, seconds, codec="lz4"):
    """Time the CPU oracle (test infrastructure, kind "port") decompressing a
    bounded sample of the same compressed blocks on this host's cores."""
    from tests.oracle_ctypes import Oracle
    so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        return None
    orc = Oracle(so)
    T = host_threads()
    bufs = [ctypes.create_string_buffer(c, len(c)) for c in comp_blocks]
    counts = [0] * T
    stop = [False]

    def work(t):
        out = ctypes.create_string_buffer(U)
        k = t
        while not stop[0]:
            c = bufs[k % len(bufs)]
            if codec == "lz4":
                r = orc.lib.oracle_lz4_decompress_safe(c, out, len(c), U)
            else:
                r = orc.lib.oracle_zstd_decompress(c, len(c), out, U)
            assert r == U
            counts[t] += 1
            k += T

    # size the run: each thread loops over the sample until the time budget ends
    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    t0 = time.perf_counter()
    [x.start() for x in th]
    time.sleep(seconds)
    stop[0] = True
    [x.join() for x in th]
    dt = time.perf_counter() - t0
    nb = sum(counts)
    return {"value": nb * U / dt / 2**30, "unit": "GiB/s", "cores": T, "kind": "port",
            "sample": f"{nb} decodes of {len(bufs)} distinct 4 MiB text blocks (oracle/{codec}_oracle.c, -O2), "
                      f"{T} threads, {dt:.1f} s wall"}


def liblz4_baseline(comp_blocks, U, seconds):
    """The C library pkg/compress reaches through cgo (LZ4_decompress_safe), if
    the host has one; reported beside the oracle."""
    for path in ("/opt/conda/lib/liblz4.so.1", "/usr/lib/x86_64-linux-gnu/liblz4.so.1"):
        if os.path.exists(path):
            break
    else:
        return None
    lz = ctypes.CDLL(path)
    T = host_threads()
    bufs = [ctypes.create_string_buffer(c, len(c)) for c in comp_blocks]
    counts = [0] * T
    stop = [False]

    def work(t):
        out = ctypes.create_string_buffer(U)
        k = t
        while not stop[0]:
            c = bufs[k % len(bufs)]
            r = lz.LZ4_decompress_safe(c, out, len(c), U)
            assert r == U
            counts[t] += 1
            k += T

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    t0 = time.perf_counter()
    [x.start() for x in th]
    time.sleep(seconds)
    stop[0] = True
    [x.join() for x in th]
    dt = time.perf_counter() - t0
    return {"value": sum(counts) * U / dt / 2**30, "unit": "GiB/s", "cores": T,
            "library": f"{path} v{lz.LZ4_versionNumber()}"}


def libzstd_baseline(comp_blocks, U, seconds):
    """ZSTD_decompress from the host's libzstd (the C library DataDog/zstd
    wraps; this image has 1.4.9, the reference pins 1.5.6)."""
    from juicefs_amd.device import _libzstd
    z = _libzstd()
    if z is None:
        return None
    z.ZSTD_versionNumber.restype = ctypes.c_uint
    T = host_threads()
    bufs = [ctypes.create_string_buffer(c, len(c)) for c in comp_blocks]
    counts = [0] * T
    stop = [False]

    def work(t):
        out = ctypes.create_string_buffer(U)
        k = t
        while not stop[0]:
            c = bufs[k % len(bufs)]
            r = z.ZSTD_decompress(out, U, c, len(c))
            assert r == U
            counts[t] += 1
            k += T

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    t0 = time.perf_counter()
    [x.start() for x in th]
    time.sleep(seconds)
    stop[0] = True
    [x.join() for x in th]
    dt = time.perf_counter() - t0
    return {"value": sum(counts) * U / dt / 2**30, "unit": "GiB/s", "cores": T,
            "library": f"{z.path} v{z.ZSTD_versionNumber()}"}


def host_path_rate(comp_blocks, raw_blocks, U, nblk, reps=2):
    """PCIe-inclusive: Go-heap-like host buffers -> pinned -> HBM -> kernel ->
    pinned -> host buffers, via the C ABI batch entry points (what the cgo
    drop-in calls), chunked and pipelined over two streams (capi.hip run_batch).
    Timed with the host clock around the whole call; best of `reps`."""
    from juicefs_amd import compress as C
    c = C.LZ4()
    k = max(1, nblk // len(comp_blocks))
    srcs = (comp_blocks * k)[:nblk]
    pairs = [(bytearray(U), cb) for cb in srcs]
    c.DecompressBatch(pairs[:4])
    res_d = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        res = c.DecompressBatch(pairs)
        dt = time.perf_counter() - t0
        assert all(n == U and e is None for n, e in res)
        res_d = max(res_d, len(pairs) * U / dt / 2**30)
    del pairs
    bound = c.CompressBound(U)
    ncb = min(nblk, 512)  # the encoder is latency-bound per block: a smaller sample
    raws = (raw_blocks * (ncb // len(raw_blocks) + 1))[:ncb]
    cpairs = [(bytearray(bound), rb) for rb in raws]
    res_c = 0.0
    for _ in range(1):
        t0 = time.perf_counter()
        res = c.CompressBatch(cpairs)
        dt = time.perf_counter() - t0
        assert all(n > 0 and e is None for n, e in res)
        res_c = max(res_c, len(cpairs) * U / dt / 2**30)
    return {"lz4_decompress": {"value": res_d, "unit": "GiB/s"},
            "lz4_compress": {"value": res_c, "unit": "GiB/s"},
            "blocks": nblk, "compress_blocks": ncb, "chunk_mb": int(os.environ.get("JFS_HOST_CHUNK_MB", "2048")),
            "path": "jfs_{de,}compress_batch: host buffers -> pinned (16 threads) -> H2D -> kernel -> D2H -> "
                    "host buffers, 2-stream chunk pipeline, 1 GPU, GiB/s of uncompressed bytes"}


def mixed_host_path(raw_src, nblk=4096, seed=11):
    """BASELINE configs[4] on one GPU: mixed LZ4/Zstd blocks of 64 KiB-4 MiB
    (log-uniform sizes, codec alternating), host buffers in and out through the
    C-ABI batch entry points (pinned staging, async H2D/D2H, capi.hip
    run_batch).  Compress = the GPU encoders (LZ4 byte-identical to
    LZ4_compress_default; Zstd level-1-style frames); decompress = the GPU
    decoders; every block is checked against its source.  GiB/s of
    uncompressed bytes over the whole mixed job (both codecs, host clock)."""
    from juicefs_amd import compress as C
    rng = np.random.default_rng(seed)
    lo, hi = 64 << 10, 4 << 20
    sizes = np.exp(rng.uniform(np.log(lo), np.log(hi), nblk)).astype(np.int64)
    raws = [raw_src[i % len(raw_src)][:int(n)] for i, n in enumerate(sizes)]
    codecs = {"lz4": C.LZ4(), "zstd": C.ZStandard()}
    idx = {"lz4": list(range(0, nblk, 2)), "zstd": list(range(1, nblk, 2))}
    total = int(sizes.sum())
    comp = [None] * nblk
    t0 = time.perf_counter()
    for name, cd in codecs.items():
        pairs = [(bytearray(cd.CompressBound(len(raws[i]))), raws[i]) for i in idx[name]]
        res = cd.CompressBatch(pairs)
        for (buf, _), (n, e), i in zip(pairs, res, idx[name]):
            if e is not None or n <= 0:
                raise RuntimeError(f"mixed compress failed: {name} block {i}: {e}")
            comp[i] = bytes(buf[:n])
    tc = time.perf_counter() - t0
    best = 0.0
    for _ in range(2):
        outs = {name: [(bytearray(len(raws[i])), comp[i]) for i in idx[name]] for name in codecs}
        t0 = time.perf_counter()
        res = {name: codecs[name].DecompressBatch(outs[name]) for name in codecs}
        td = time.perf_counter() - t0
        for name in codecs:
            for (buf, _), (n, e), i in zip(outs[name], res[name], idx[name]):
                if e is not None or n != len(raws[i]) or bytes(buf) != raws[i]:
                    raise RuntimeError(f"mixed round trip mismatch: {name} block {i}")
        best = max(best, total / td / 2**30)
    csz = sum(len(x) for x in comp)
    return {"decompress": {"value": best, "unit": "GiB/s"},
            "compress": {"value": total / tc / 2**30, "unit": "GiB/s"},
            "blocks": nblk, "bytes": total, "ratio": total / csz,
            "sizes": "log-uniform 64 KiB-4 MiB, LZ4 and Zstd alternating",
            "path": "BASELINE configs[4] on 1 GPU: jfs_{de,}compress_batch per codec, host buffers in and out, "
                    "GPU encoders and decoders, every block verified"}


def main():
    a = parse()
    env = S.rank_env()
    world, rank, local = env.world, env.rank, env.local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from juicefs_amd import device as D

    U, nblk = a.block_bytes, a.blocks
    t_setup = time.perf_counter()
    if a.codec == "lz4":
        batch = D.Lz4Batch(nblk, U, a.cls, seed_base=S.seed_base(rank, nblk), device=dev)
    else:
        batch = D.ZstdBatch(nblk, U, a.cls, level=a.level, distinct=16, seed_base=S.seed_base(rank, 16), device=dev)
    C = batch.comp_bytes
    setup_s = time.perf_counter() - t_setup

    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    k = [0]

    def step():
        if k[0] >= a.warmup:  # HIP events on the launch stream, timed steps only
            i = k[0] - a.warmup
            ev[i][0].record(stream)
            batch.decompress(stream)
            ev[i][1].record(stream)
        else:
            batch.decompress(stream)
        k[0] += 1

    # barrier + synchronize on both sides of exactly a.steps steps; max over ranks
    elapsed = S.timed_steps(step, a.steps, a.warmup, torch.cuda.synchronize, world)
    elapsed = S.max_over_ranks(elapsed, world, dev)
    kms = [s.elapsed_time(e) for s, e in ev]
    kern_s = float(np.mean(kms)) / 1e3
    if not S.all_ranks_ok(batch.verify(), world, dev):
        raise SystemExit("decoded output mismatch: benchmark invalid")

    ms_per_step = elapsed / a.steps * 1e3
    value = S.whole_job_gib_s(world, nblk, U, a.steps, elapsed)
    achieved = (C + nblk * U) / kern_s / 1e9
    traffic = None
    if a.codec == "lz4" and os.path.exists(a.traffic_file):
        try:
            tj = json.load(open(a.traffic_file))
            if tj.get("blocks") == nblk and tj.get("block_bytes") == U:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if a.codec == "lz4":
        workload = "LZ4 decompress, 4096x4MiB blocks already in HBM (BASELINE configs[1])"
        kernel = "jfs::lz4d::lz4_decode_kernel"
        data = "synthetic (text-like blocks generated on GPU, SURVEY.md 8d; LZ4-compressed on GPU)"
    else:
        workload = f"Zstd level-{a.level} decompress, {nblk}x4MiB frames already in HBM (BASELINE configs[3])"
        kernel = "zscan + zentropy + zexec (whole jfs_zstd_decompress_device call)"
        data = (f"synthetic text-like blocks (SURVEY.md 8d), {batch.distinct} distinct, compressed on the host by "
                f"libzstd level {a.level}, replicated to {nblk} frames")
        traffic = None
    out = {
        "metric": "device-resident GiB/s (de)compress, 4 MiB blocks, LZ4+Zstd, 1/2/4/8 MI355X",
        "value": value,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": data,
        "config": {
            "workload": workload,
            "blocks_per_gpu": nblk, "block_bytes": U, "class": a.cls,
            "compressed_bytes_per_gpu": C, "ratio": nblk * U / C,
            "parallelism": f"{world} process(es), one per GPU, blocks sharded, no collective",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": kernel, "kernel_ms": kern_s * 1e3,
            "algorithmic_bytes_per_launch": C + nblk * U,
            "u_only_TBps": nblk * U / kern_s / 1e12,
        },
        "setup_s": setup_s,
    }
    if rank == 0 and world == 1:
        # bounded sample for the CPU legs: 32 distinct blocks
        ns = min(32, nblk)
        comp_blocks = []
        for i in range(ns):
            s0 = i * batch.slot
            comp_blocks.append(batch.comp[s0:s0 + int(batch.csize[i])].cpu().numpy().tobytes())
        if not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(comp_blocks, U, a.cpu_seconds, a.codec)
            if a.codec == "lz4":
                lb = liblz4_baseline(comp_blocks, U, a.cpu_seconds / 2)
                if lb:
                    out["cpu_liblz4"] = lb
            else:
                lb = libzstd_baseline(comp_blocks, U, a.cpu_seconds / 2)
                if lb:
                    out["cpu_libzstd"] = lb
        if not a.no_extras:
            ex = {}
            if a.codec == "lz4":
                ex["lz4_compress"] = {"value": nblk * U / (batch.enc_ms / 1e3) / 2**30, "unit": "GiB/s",
                                      "kernel_ms": batch.enc_ms, "blocks": nblk,
                                      "note": "one GPU LZ4 encode launch (byte-identical to LZ4_compress_default)"}
            try:
                zr, zratio, zms = D.zstd_compress_rate(min(a.extra_blocks, nblk), U, a.cls, seed_base=7, device=dev)
                ex["zstd_compress"] = {"value": zr, "unit": "GiB/s", "ratio": zratio, "kernel_ms": zms,
                                       "blocks": min(a.extra_blocks, nblk),
                                       "note": "one GPU Zstd encode launch; frames verified by the GPU decoder"}
            except Exception as e:  # report, never fake
                ex["zstd_compress"] = {"error": str(e)}
            out["compress"] = ex
        if not a.no_host_path and a.codec == "lz4" and rank == 0:
            try:
                raw_blocks = [batch.raw[i * U:(i + 1) * U].cpu().numpy().tobytes() for i in range(len(comp_blocks))]
                out["host_path"] = host_path_rate(comp_blocks, raw_blocks, U, a.host_blocks)
            except Exception as e:  # report, never fake
                out["host_path"] = {"error": str(e)}
        if not a.no_mixed and not a.no_host_path and a.codec == "lz4" and rank == 0:
            try:
                src = [batch.raw[i * U:(i + 1) * U].cpu().numpy().tobytes() for i in range(min(32, nblk))]
                out["mixed_host_path"] = mixed_host_path(src, a.mixed_blocks)
            except Exception as e:  # report, never fake
                out["mixed_host_path"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
