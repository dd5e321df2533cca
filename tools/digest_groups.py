#!/usr/bin/env python3
"""Latency and throughput of the worker's batch digests by group size.

For each group size G (default 1, 8, 64, 1024, 100000) a burst of G config-4 batches (508,052 B,
drawn from a pool of distinct batches) is digested three ways:
  gpu_digester : the Processor path -- nwc_digester (max_group = G) from host memory: gather into
                 pinned stages, H2D, one k_sha512 launch, D2H (narwhal_amd/processor.py);
  gpu_digester_arena : the same burst received into the digester's pinned arena (nwc_digester_arena):
                 one DMA per group straight into HBM, no stage fill (groups up to --arena-max-gb);
  gpu_resident : the same G batches already in HBM, one nwc_dev_sha512_trunc32_ranges launch
                 (the kernel alone: what a node re-digesting stored batches would see);
  cpu          : hashlib (OpenSSL) SHA-512 on the host, 1 thread and every CPU the process is granted.
Per-batch latency = time from submission to the digest being back on the host; a burst's batches
all return together on the GPU, so the GPU latency of every batch is the burst's.  Every digest
is checked against hashlib.  Writes one JSON object (stdout, or --out).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BATCH = 508_052


def cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", default="1,8,64,1024,100000")
    ap.add_argument("--pool", type=int, default=256)
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of CPU hashing per group size, at most")
    ap.add_argument("--arena-max-gb", type=float, default=8.0, help="largest pinned receive arena to allocate")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from narwhal_amd import _lib
    from narwhal_amd.processor import Digester
    lib = _lib.load()
    rng = np.random.default_rng(11)
    pool = [rng.integers(0, 256, BATCH, dtype=np.uint8).tobytes() for _ in range(args.pool)]
    want = [hashlib.sha512(b).digest()[:32] for b in pool]
    th = cpu_threads()
    res = {"batch_bytes": BATCH, "pool_distinct": args.pool, "cpu_threads": th, "rows": []}
    STRIDE = (BATCH + 255) & ~255   # resident batches start 256-B aligned (the kernel's dwordx4 path)
    flat = bytearray(STRIDE * args.pool)
    for i, b in enumerate(pool):
        flat[i * STRIDE:i * STRIDE + BATCH] = b
    dev_pool = torch.frombuffer(flat, dtype=torch.uint8).cuda()
    for G in [int(x) for x in args.groups.split(",")]:
        row = {"group": G, "bytes": G * BATCH}
        # --- the Processor path from host memory
        dg = Digester(max_group=G, max_wait_us=30_000_000)
        try:
            for warm in range(2):   # first burst grows the digester's buffers
                t0 = time.perf_counter()
                for i in range(G):
                    dg.submit(pool[i % args.pool], i)
                t_sub = time.perf_counter() - t0
                got = []
                while len(got) < G:
                    got += dg.poll(1 << 16, 1_000_000)
                dt = time.perf_counter() - t0
            assert all(d == want[t % args.pool] for t, d in got) and [t for t, _ in got] == list(range(G))
            groups, _, _ = dg.stats()
        finally:
            dg.close()
        row["gpu_digester"] = {"latency_ms": dt * 1e3, "GBps": G * BATCH / dt / 1e9, "submit_ms": t_sub * 1e3,
                               "groups_total": groups, "parity_ok": True}
        # --- the same burst received straight into the digester's pinned arena (the copy into the
        # arena stands for the network read and is not timed): direct DMA, no stage fill
        STR16 = (BATCH + 15) & ~15
        if G * STR16 <= args.arena_max_gb * 1e9:
            dg = Digester(max_group=G, max_wait_us=30_000_000)
            try:
                arena = dg.arena(G * STR16)
                views = []
                for i in range(G):
                    v = arena[i * STR16:i * STR16 + BATCH]
                    v[:] = np.frombuffer(pool[i % args.pool], np.uint8)
                    views.append(v)
                for warm in range(2):
                    t0 = time.perf_counter()
                    for i in range(G):
                        dg.submit(views[i], i)
                    got = []
                    while len(got) < G:
                        got += dg.poll(1 << 16, 1_000_000)
                    dt = time.perf_counter() - t0
                assert all(d == want[t % args.pool] for t, d in got) and [t for t, _ in got] == list(range(G))
                direct = dg.direct_groups()
            finally:
                dg.close()
            row["gpu_digester_arena"] = {"latency_ms": dt * 1e3, "GBps": G * BATCH / dt / 1e9, "direct_groups": direct,
                                         "parity_ok": True}
        # --- resident in HBM: the kernel alone
        starts = torch.tensor([(i % args.pool) * STRIDE for i in range(G)], dtype=torch.int64, device="cuda")
        ends = starts + BATCH
        out = torch.empty((G, 32), dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream()
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _lib.check(lib.nwc_dev_sha512_trunc32_ranges(dev_pool.data_ptr(), starts.data_ptr(), ends.data_ptr(), G,
                                                         out.data_ptr(), s.cuda_stream))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        o = out.cpu().numpy()
        assert all(o[i].tobytes() == want[i % args.pool] for i in range(0, G, max(1, G // 64)))
        dt = min(ts[1:])
        row["gpu_resident"] = {"latency_ms": dt * 1e3, "GBps": G * BATCH / dt / 1e9}
        # --- CPU: one thread, and the process's CPUs (a bounded sample when G is large)
        for label, nt in (("cpu_1thread", 1), ("cpu_%dthreads" % th, th)):
            k = G
            t0 = time.perf_counter()
            with ThreadPoolExecutor(nt) as ex:
                done = 0
                while done < k:
                    chunk = min(k - done, 64 * nt)
                    list(ex.map(lambda i: hashlib.sha512(pool[i % args.pool]).digest(), range(done, done + chunk)))
                    done += chunk
                    if time.perf_counter() - t0 > args.cpu_budget and done < k:
                        k = done
                        break
            dt = time.perf_counter() - t0
            row[label] = {"latency_ms": dt * 1e3 * (G / k), "GBps": k * BATCH / dt / 1e9, "threads": nt,
                          "measured_batches": k, "extrapolated": k < G}
        res["rows"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    txt = json.dumps(res, indent=1)
    if args.out:
        open(args.out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
