#!/usr/bin/env python3
"""Benchmark of the MI355X Ed25519-verify / SHA-512-digest hot path.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU, RCCL)

Headline (BASELINE.json metric): Ed25519 verifies/s.  Workload = BASELINE config 2:
1M independent (32-byte msg, pk, sig) triples per GPU, all valid, `Signature::verify`
(verify_strict) semantics; weak scaling (every rank verifies its own 1M-triple shard of
distinct keys; no data-path collective).  A "step" is one verification pass over the 1M
triples with inputs resident in HBM.  The per-shard verdict bitmaps are all-gathered over
RCCL after the timed region and the gather is timed separately (it is not needed for
correctness: every rank already holds its verdicts).

Secondary leg (same JSON line, "digest"): BASELINE config 4, SHA-512[..32] of 100,000
worker batches of 508,052 B (977 x 512-B txs, bincode WorkerMessage::Batch), hashed from a
cycled pool of distinct batches resident in HBM.  `configs.cfg4_host` times the same batches
from host memory through the worker's digester (pinned stages, and the pinned receive arena).

cpu_baseline: the C restatement (oracle/, "port") of dalek verify_strict on the host cores of
the GPU box (rank 0, N = 1 only), on a bounded sample of the same workload, with OpenSSL's
EVP Ed25519 beside it ("openssl", a third-party point, not dalek semantics).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Ed25519 verifies/sec at 1/2/4/8 MI355X (+% int-VALU peak); batch digest GB/s"

# ---- frozen work model ------------------------------------------------------
# W_strict: field squarings / multiplications per verify_strict in the dalek 1.0.1 serial
# algorithm (2 decompressions, 2 small-order checks, width-5/8 NAF double-scalar-mult,
# projective compare) + one SHA-512 block.  Converted to 32-bit-lane VALU instructions with the
# per-op instruction counts of this build's fe_sq / fe_mul / sha512_compress (tools/count_ops.py).
W_S, W_M, W_SHA = 1546, 1429, 1
# Frozen at the round-1 build (tools/count_ops.py on commit dc19643, before any kernel tuning):
# later speedups of fe_mul/fe_sq must raise `frac`, not shrink the work they are measured against.
OPS_S, OPS_M, OPS_SHA = 134, 167, 5039
# VALU issue peak (MI355X_MICROARCH.md "Execution model": a wave64 VALU instruction issues over 2
# cycles on a SIMD-32 -> 128 lane-instructions / clk / CU) x 256 CU x 2.4 GHz.
VALU_PEAK_TOPS = 128 * 256 * 2.4e9 / 1e12     # 78.64 T lane-ops/s
# The measured issue rate of the VOP3 integer class that dominates these kernels
# (v_mad_i64_i32 / v_mad_u64_u32, v_alignbit, v_bitop3, v_lshl_add_u64: 4 cycles per wave64
# instruction at full occupancy; tools/microbench/int_rates.hip, profiles/r02/microbench/)
VOP3_RATE_TOPS = 64 * 256 * 2.4e9 / 1e12      # 39.32 T lane-ops/s
HBM_PEAK_GBS = 8000.0                          # MI355X_MICROARCH.md (spec)

CFG4_TXS, CFG4_TX_BYTES = 977, 512
CFG4_BATCH_BYTES = 12 + CFG4_TXS * (8 + CFG4_TX_BYTES)   # 508,052
CFG4_STRIDE = (CFG4_BATCH_BYTES + 255) & ~255


PROFILE_ROUND = "r06"   # profiles/<round>/<workload>/summary.json: rocprofv3 passes of this build (tools/profile_r06.sh)


def profile_counters(*kernel_names: str, workload: str = "head"):
    """Per-launch PMC figures of the first of `kernel_names` found in the committed rocprofv3 summary
    of `workload` (tools/profile_r06.sh -> tools/summarize_profile.py): HBM traffic = FETCH_SIZE x2
    (gfx950 wide-read correction) + WRITE_SIZE, VALU lane-ops per launch, the average duration and
    the shader clock during the kernel (GRBM_GUI_ACTIVE per XCD / duration).  None if absent."""
    path = os.path.join(ROOT, "profiles", PROFILE_ROUND, workload, "summary.json")
    try:
        summ = json.load(open(path))
    except (OSError, ValueError):
        return None
    for k in kernel_names:
        d = summ.get(k, {})
        if "hbm_traffic_bytes_per_launch" in d:
            return {"traffic": d["hbm_traffic_bytes_per_launch"], "valu_insts_per_lane": d.get("valu_insts_per_lane"),
                    "lane_ops_per_launch": d.get("SQ_INSTS_VALU", 0) * 64, "avg_ns": d.get("avg_ns"),
                    "calls": d.get("calls"), "clock_ghz": d.get("gui_active_clk_ghz_per_xcd"),
                    "source": "profiles/%s/%s/summary.json (%s)" % (PROFILE_ROUND, workload, k)}
    return None


def profile_kernel_ms(workload: str, kernel: str):
    """Average duration (ms) of `kernel` in the committed kernel trace of `workload`, or None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", PROFILE_ROUND, workload, "summary.json"))).get(kernel, {})
        return d["avg_ns"] * 1e-6
    except (OSError, ValueError, KeyError):
        return None


CENSUS = os.path.join(ROOT, "profiles", PROFILE_ROUND, "isa_census.json")   # tools/isa_census.py of this build


def issue_cycles(kernel: str):
    """Average issue cycles per wave64 VALU instruction of `kernel` (VOP3/VOP3P 4, VOP1/VOP2 2),
    from the committed ISA census (static counts x trip counts, tools/isa_census.py)."""
    try:
        k = json.load(open(CENSUS))["kernels"][kernel]
        return k["avg_issue_cycles"], k["share_4cycle"]
    except (OSError, ValueError, KeyError):
        return None, None


def roofline_extra(workload: str, kernel: str, census: str, units: int, unit: str, step_ms_live: float,
                   units_per_step: int, algo_bytes_per_unit: float, extra_kernels=()):
    """Roofline entry of a non-headline number (configs 3 and 5): the dominant kernel's VALU lane-ops
    per launch (SQ_INSTS_VALU x 64) over its average duration, both from the committed rocprofv3
    passes of this workload (`pmc_source`), against the guide's VALU issue peak (frac), priced per
    instruction class by the ISA census (frac_issue), with the shader clock the kernel held
    (GRBM_GUI_ACTIVE) and its HBM traffic per unit against the algorithmic input bytes.  Beside it,
    the live step time of this run and the dalek work model per unit over it (effective_frac: W_strict
    per unit / live step time; batch algorithms that do less work per vote exceed the hardware
    fraction).  `units` = the units one launch of the kernel processes."""
    out = {"bound": "valu", "unit": "T lane-ops/s", "peak": VALU_PEAK_TOPS, "kernel": kernel,
           "units_per_launch": units, "unit_name": unit, "step_ms_live": step_ms_live,
           "effective_frac": units_per_step / (step_ms_live * 1e-3) * ops_per_verify() / 1e12 / VALU_PEAK_TOPS,
           "algorithmic_bytes_per_unit": algo_bytes_per_unit}
    pc = profile_counters("nwc::" + kernel, workload=workload)
    if not pc:
        out.update({"frac": None, "pmc_source": "profiles/%s/%s/summary.json missing" % (PROFILE_ROUND, workload)})
        return out
    kms = pc["avg_ns"] * 1e-6
    ach = pc["lane_ops_per_launch"] / (kms * 1e-3) / 1e12
    out.update({"kernel_ms_rocprof": kms, "achieved": ach, "frac": ach / VALU_PEAK_TOPS,
                "frac_vop3_rate": ach / VOP3_RATE_TOPS, "valu_insts_per_unit": pc["lane_ops_per_launch"] / units,
                "traffic": pc["traffic"], "traffic_per_unit": pc["traffic"] / units,
                "traffic_over_algorithmic": pc["traffic"] / (algo_bytes_per_unit * units),
                "clock_ghz": pc["clock_ghz"], "pmc_source": pc["source"]})
    cyc, share = issue_cycles(census) if census else (None, None)
    if cyc:
        out["frac_issue"] = out["frac"] * cyc / 2
        out["issue_census"] = {"avg_issue_cycles": cyc, "share_4cycle": share,
                               "source": os.path.relpath(CENSUS, ROOT) + " (tools/isa_census.py)"}
        if pc["clock_ghz"]:
            out["frac_issue_at_clock"] = out["frac_issue"] * 2.4 / pc["clock_ghz"]
    others = {}
    for k in extra_kernels:
        ms = profile_kernel_ms(workload, "nwc::" + k)
        if ms is not None:
            others[k] = ms
    if others:
        out["other_kernels_ms_rocprof"] = others
    return out


def ops_per_verify() -> float:
    return W_S * OPS_S + W_M * OPS_M + W_SHA * OPS_SHA


# ---- distributed ---------------------------------------------------------------------------
def progress(msg: str) -> None:
    """One line per bench leg on stderr (the JSON line stays alone on stdout)."""
    print("[bench %.0f s] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def dist_setup(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d (launch N>1 with torch.distributed.run)" % (world, args.gpus))
    # NWC_BENCH_BACKEND=gloo rehearses the N>1 code path with more ranks than GPUs (ranks share
    # devices round-robin); the driver's runs use the default, RCCL with one GPU per rank.
    backend = os.environ.get("NWC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit("WORLD_SIZE=%d but only %d GPUs visible" % (world, ndev))
    local = local % max(1, ndev)
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def barrier(world):
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    import torch
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---- workloads -------------------------------------------------------------------------------
def make_cfg2(rank: int, n: int):
    """SURVEY.md §8(d) cfg 2: seed_i = SHA-512("nw-seed"||u64le(i))[..32],
    msg_i = SHA-512("nw-msg"||u64le(i))[..32], RFC 8032 keygen+sign (on the GPU)."""
    from narwhal_amd import device
    first = rank * n
    seeds = device.derive32(b"nw-seed", first, n)
    msgs = device.derive32(b"nw-msg", first, n)
    pks, sigs = device.keygen_sign(seeds, msgs)
    return msgs, pks, sigs


def make_cfg4_pool(pool: int):
    """`pool` distinct cfg-4 batches (bincode Batch of 977 x 512-B txs; tx = [1][u64 BE
    counter][zeros], node/src/benchmark_client.rs:117-130), batch b's counters b*977 + j."""
    import torch
    tmpl = bytearray(CFG4_STRIDE)
    tmpl[0:4] = (0).to_bytes(4, "little")
    tmpl[4:12] = CFG4_TXS.to_bytes(8, "little")
    pos = []
    o = 12
    for j in range(CFG4_TXS):
        tmpl[o:o + 8] = CFG4_TX_BYTES.to_bytes(8, "little")
        tmpl[o + 8] = 1
        pos.append(o + 9)
        o += 8 + CFG4_TX_BYTES
    assert o == CFG4_BATCH_BYTES
    data = torch.frombuffer(bytearray(tmpl), dtype=torch.uint8).cuda().repeat(pool)
    view = data.view(pool, CFG4_STRIDE)
    posj = torch.tensor(pos, dtype=torch.int64, device="cuda")
    for b0 in range(0, pool, 1024):
        b1 = min(pool, b0 + 1024)
        ctr = (torch.arange(b0, b1, device="cuda", dtype=torch.int64)[:, None] * CFG4_TXS
               + torch.arange(CFG4_TXS, device="cuda", dtype=torch.int64)[None, :])
        for k in range(8):
            byte = ((ctr >> (8 * (7 - k))) & 0xFF).to(torch.uint8)
            view[b0:b1].index_copy_(1, posj + k, byte)
    return data


def cfg4_host_batch(b: int) -> bytes:
    out = bytearray()
    out += (0).to_bytes(4, "little") + CFG4_TXS.to_bytes(8, "little")
    for j in range(CFG4_TXS):
        out += CFG4_TX_BYTES.to_bytes(8, "little") + bytes([1]) + (b * CFG4_TXS + j).to_bytes(8, "big") + bytes(503)
    return bytes(out)


def cfg4_pool_host(b0: int, b1: int) -> np.ndarray:
    """Pool batches b0 .. b1-1 built on the host with numpy, independently of the GPU construction
    (make_cfg4_pool) and with cfg4_host_batch's layout: (b1 - b0, CFG4_STRIDE) uint8, zero-padded."""
    k = b1 - b0
    out = np.zeros((k, CFG4_STRIDE), np.uint8)
    out[:, 4:12] = np.frombuffer(CFG4_TXS.to_bytes(8, "little"), np.uint8)
    pos = 12 + np.arange(CFG4_TXS) * (8 + CFG4_TX_BYTES)
    lenb = np.frombuffer(CFG4_TX_BYTES.to_bytes(8, "little"), np.uint8)
    for j in range(8):
        out[:, pos + j] = lenb[j]
    out[:, pos + 8] = 1
    ctr = np.arange(b0, b1, dtype=np.uint64)[:, None] * CFG4_TXS + np.arange(CFG4_TXS, dtype=np.uint64)[None, :]
    be = ctr.astype(">u8").view(np.uint8).reshape(k, CFG4_TXS, 8)
    for j in range(8):
        out[:, pos + 9 + j] = be[:, :, j]
    return out


def check_cfg4_digests(data, outs, pool: int, nb: int, threads: int, chunk: int = 512):
    """Every digest of the config-4 launch (nb ranges cycling a pool of `pool` batches, message i =
    pool batch i mod pool): out[i] == out[i mod pool] for all i (on the device), and for every pool
    batch its bytes equal the host construction (cfg4_pool_host) and its digest equals hashlib's
    (OpenSSL) SHA-512[..32], hashed on `threads` host threads.  worker/src/processor.rs:38."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    idx = torch.arange(nb, device=outs.device, dtype=torch.int64) % pool
    periodic = bool((outs == outs[idx]).all().item())
    npool = min(pool, nb)
    o = outs[:npool].cpu().numpy()
    bad_bytes = bad_dig = 0
    with ThreadPoolExecutor(threads) as ex:
        for b0 in range(0, npool, chunk):
            b1 = min(npool, b0 + chunk)
            dev = data[b0 * CFG4_STRIDE:b1 * CFG4_STRIDE].view(b1 - b0, CFG4_STRIDE).cpu().numpy()
            host = cfg4_pool_host(b0, b1)
            bad_bytes += int((dev[:, :CFG4_BATCH_BYTES] != host[:, :CFG4_BATCH_BYTES]).any(axis=1).sum())
            digs = list(ex.map(lambda r: hashlib.sha512(r[:CFG4_BATCH_BYTES]).digest()[:32], host))
            bad_dig += sum(d != o[b0 + i].tobytes() for i, d in enumerate(digs))
    ok = periodic and bad_bytes == 0 and bad_dig == 0
    return ok, {"digests_checked": nb, "pool_batches_vs_hashlib": npool, "periodic": periodic,
                "pool_bytes_mismatch": bad_bytes, "digest_mismatch": bad_dig}


def bench_cfg1(lib, calls: int = 10000, cpu_baseline: bool = False):
    """BASELINE config 1: Signature::verify_batch on the reference's 4-node
    certificate -- the crypto_tests.rs fixture keys (ChaCha20-seeded, tests/golden), digest =
    SHA-512("Hello, world!")[..32], votes of keys 3, 2, 1 (crypto_tests.rs:79-94) -- through the
    host ABI (H2D + kernel + D2H per call).  Latency-bound by design.  Timed without and with the
    committee cache (the 4 authorities' keys, as a node always has its committee:
    config/src/lib.rs Committee); the cached leg runs the latency kernel, and also times the
    reference's invalid variant (key 1's signature replaced by 64 zero bytes, :96-115)."""
    from narwhal_amd import _lib
    gv = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_verify.json")))
    gb = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_batch.json")))}
    committee = np.stack([np.frombuffer(bytes.fromhex(x), np.uint8) for x in gv["reference_keys"]["pks"]])

    def case(name):
        c = gb[name]
        d = bytes.fromhex(c["msg"])
        p = b"".join(bytes.fromhex(v[0]) for v in c["votes"])
        s = b"".join(bytes.fromhex(v[1]) for v in c["votes"])
        return d, p, s, len(c["votes"]), 0 if c["verdict"] is True else 1

    d, p, s, n, want = case("ref-verify_valid_batch")
    assert d.hex() == gv["hello_digest"] and n == 3 and want == 0
    out = {"workload": "cfg1: verify_batch, the reference's 3-vote certificate of its 4-node committee "
                       "(crypto_tests.rs:79-94), host ABI incl. H2D/D2H"}

    def timed(d, p, s, n, want):
        lat = []
        first_us = second_us = None
        for i in range(calls + 50):
            t0 = time.perf_counter()
            rc = lib.nwc_verify_batch(_lib.buf(d), _lib.buf(p), _lib.buf(s), n, None)
            dt = time.perf_counter() - t0
            assert rc == want, (rc, want)
            if i == 0:
                first_us = dt * 1e6
            if i == 1:
                second_us = dt * 1e6
            if i >= 50:
                lat.append(dt)
        lat = np.array(lat) * 1e6
        return {"calls": calls, "first_call_us": first_us, "second_call_us": second_us,
                "p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
                "calls_per_s": float(1e6 / lat.mean())}

    # no nwc_set_committee: the keys miss the committee cache; the library's auto key cache adds
    # them the second time they are seen (one build, ~3 ms, queued behind that call), after which
    # calls take the latency kernel.  The first call is the uncached figure (k_verify_cold).
    out["auto_cache"] = timed(d, p, s, n, want)
    out["auto_cache"]["note"] = ("no nwc_set_committee.  first_call_us: first sight, uncached (k_verify_cold, zero-copy "
                                 "launch); second_call_us: second sight, k_verify_cold again with the auto-cache build "
                                 "queued behind it (not waited for); the third call waits for that build; p50/p99 over "
                                 "calls 50.. (the auto-cache latency kernel)")
    out["cold"] = cfg1_cold(lib, min(calls, 200))
    _lib.check(lib.nwc_set_committee(_lib.buf(committee), len(committee)))
    out["cache"] = timed(d, p, s, n, want)
    out["cache_invalid_variant"] = timed(*case("ref-verify_invalid_batch"))
    _lib.check(lib.nwc_set_committee(None, 0))
    out["c_host"] = cfg1_c_host(case, committee, calls)
    if cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_cfg1(d, p, s, n, min(calls, 2000))
    return out


def cfg1_c_host(case, committee, calls: int):
    """The same three cfg-1 legs timed from a plain C process (tests/cpp/abi_host, the Rust shim's
    situation: no interpreter, no ctypes buffers, no GC in the loop), so the tail percentiles
    separate the library from the Python harness.  A separate process with its own nwc_init."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "build", "abi_host")
    if not os.path.exists(exe):
        return {"skipped": "tests/cpp/build/abi_host not built"}

    def lreq(name):
        d, p, s, n, _ = case(name)
        votes = " ".join("%s %s" % (p[32 * i:32 * i + 32].hex(), s[64 * i:64 * i + 64].hex()) for i in range(n))
        return "L %d 50 %s %d %s" % (calls + 50, d.hex(), n, votes)

    keys = " ".join(k.tobytes().hex() for k in committee)
    script = "\n".join([lreq("ref-verify_valid_batch"), "K %d %s" % (len(committee), keys),
                        lreq("ref-verify_valid_batch"), lreq("ref-verify_invalid_batch"), "K 0", ""])
    r = subprocess.run([exe], input=script, capture_output=True, text=True, timeout=300)
    lines = [l.split() for l in r.stdout.splitlines() if l.startswith("L ")]
    if r.returncode != 0 or len(lines) != 3:
        return {"error": "abi_host rc %d: %s" % (r.returncode, (r.stdout + r.stderr)[-300:])}
    keys_ = ("rc", "first_call_us", "second_call_us", "p50_us", "p90_us", "p99_us", "p999_us", "max_us", "mean_us")
    legs = {}
    for tag, f in zip(("auto_cache", "cache", "cache_invalid_variant"), lines):
        legs[tag] = {k: (int(v) if k == "rc" else float(v)) for k, v in zip(keys_, f[1:])}
        legs[tag]["calls"] = calls
    legs["note"] = "nwc_verify_batch timed with clock_gettime in a C process; percentiles over calls 50.."
    return legs


def cfg1_cold(lib, certs: int = 200):
    """First-sight keys: `certs` distinct 3-vote certificates, every vote by a key never seen before
    (so every call misses the committee and auto caches): each call is one zero-copy launch of
    k_verify_cold (limb-sliced, one 4-wave block per equation, the keys' batch-leaf torsion test
    folded in) reading the pinned inputs in place.  Per-call latency through the same host ABI."""
    import torch
    from narwhal_amd import _lib, device
    seeds = device.derive32(b"cfg1-cold-seed", 0, 3 * certs)
    digests = device.derive32(b"cfg1-cold-digest", 0, certs)
    msgs = digests.repeat_interleave(3, dim=0)
    pks, sigs = device.keygen_sign(seeds, msgs)
    torch.cuda.synchronize()
    P, S, D = (t.cpu().numpy().tobytes() for t in (pks, sigs, digests))
    lat = []
    for c in range(certs):
        d, p, s = D[32 * c:32 * c + 32], P[96 * c:96 * c + 96], S[192 * c:192 * c + 192]
        t0 = time.perf_counter()
        rc = lib.nwc_verify_batch(_lib.buf(d), _lib.buf(p), _lib.buf(s), 3, None)
        lat.append(time.perf_counter() - t0)
        assert rc == 0, rc
    lat = np.array(lat[5:]) * 1e6
    return {"calls": int(len(lat)), "p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
            "note": "every call a new certificate of 3 first-sight keys (no cache of any kind applies)"}


def cpu_baseline_cfg1(d: bytes, p: bytes, s: bytes, n: int, calls: int):
    """The same 3-vote verify_batch on one host core with the dalek algorithm (random z_i +
    Straus MSM; oracle/nwc_oracle.c orc_verify_batch_straus), per-call latency as on the GPU."""
    import ctypes
    from tests.oracle_lib import load_oracle
    orc = load_oracle().lib
    bd, bp, bs = (ctypes.create_string_buffer(x, len(x)) for x in (d, p, s))
    lat = []
    for i in range(calls + 20):
        t0 = time.perf_counter()
        rc = orc.orc_verify_batch_straus(bd, bp, bs, n, i + 1)
        dt = time.perf_counter() - t0
        assert rc == 1, rc   # 1 = Ok (all valid)
        if i >= 20:
            lat.append(dt)
    lat = np.array(lat) * 1e6
    out = {"p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)), "cores": 1,
           "kind": "port", "sample": "%d calls, C restatement of dalek verify_batch (Straus), 1 thread" % calls}
    # also throughput over independent calls on every CPU the box grants
    # (rayon-style, one certificate per task): the same certificate as k independent calls
    from tests.oracle_lib import load_oracle
    th = cpu_threads()
    k = 256 * th
    dg = np.frombuffer(d, np.uint8)[None, :].repeat(k, axis=0)
    pk = np.frombuffer(p, np.uint8).reshape(n, 32)
    sg = np.frombuffer(s, np.uint8).reshape(n, 64)
    offs = (np.arange(k + 1) * n).astype(np.uint32)
    P, S = np.ascontiguousarray(np.tile(pk, (k, 1))), np.ascontiguousarray(np.tile(sg, (k, 1)))
    orc2 = load_oracle()
    t0 = time.perf_counter()
    reps = 0
    while True:
        ok = orc2.batch_straus_many(dg, offs, P, S, threads=th)
        reps += 1
        if time.perf_counter() - t0 > 2.0:
            break
    dt = time.perf_counter() - t0
    out["throughput"] = {"calls_per_s": reps * k / dt, "cores": th, "parity_ok": bool(ok.all()),
                         "sample": "%d x %d independent verify_batch calls of the 3-vote certificate, %d threads, %.1f s"
                                   % (reps, k, th, dt)}
    return out


def cpu_baseline_cfg3(cdig, pks, sigs, m: int, Q: int, bad, budget_s: float):
    """dalek 1.0.1 verify_batch (random z_i + Straus MSM, oracle/nwc_oracle.c
    orc_verify_batch_straus) over whole certificates on the host cores, rayon-style (one
    certificate per task), on a bounded prefix of the same certificates."""
    from tests.oracle_lib import load_oracle
    orc = load_oracle()
    th = cpu_threads()
    k = min(m, 64 * th)
    while True:
        offs = (np.arange(k + 1) * Q).astype(np.uint32)
        d = cdig[:k].cpu().numpy()
        p = pks[:k * Q].cpu().numpy()
        s_ = sigs[:k * Q].cpu().numpy()
        t0 = time.perf_counter()
        got = orc.batch_straus_many(d, offs, p, s_, threads=th)
        dt = time.perf_counter() - t0
        if dt > budget_s / 4 or k == m:
            break
        k = min(m, int(k * max(2.0, budget_s / max(dt, 1e-3) * 0.8)))
    exp = ~bad[:k * Q].view(k, Q).any(dim=1).cpu().numpy()
    return {"value": k * Q / dt, "unit": "votes/s", "certs_per_s": k / dt, "cores": th, "kind": "port",
            "value_per_thread": k * Q / dt / th, "parity_ok": bool((got == exp).all()),
            "sample": "%d of the cfg-3 certificates (dalek verify_batch algorithm: random z, Straus MSM; "
                      "C restatement, %d threads, %.1f s)" % (k, th, dt)}


def make_cfg3(m: int, clean: bool = True):
    """BASELINE config 3's certificates: a 100-node committee (seeds "nw-committee"),
    m certificates (digests "nw-cert") x 67 distinct voters (seeded permutation, 0x4E57), each vote
    invalid with p = 0.01 (signed over the digest with one bit flipped); with clean=True also the same
    votes all valid.  Keys and signatures from the GPU signer; every tensor resident in HBM."""
    from narwhal_amd import device
    import torch
    N, Q = 100, 67
    nv = m * Q
    cseeds = device.derive32(b"nw-committee", 0, N)
    cdig = device.derive32(b"nw-cert", 0, m)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x4E57)
    voters = torch.rand((m, N), device="cuda", generator=g).argsort(dim=1)[:, :Q].reshape(-1)
    bad = torch.rand(nv, device="cuda", generator=g) < 0.01
    msg_index = torch.arange(m, device="cuda", dtype=torch.int32).repeat_interleave(Q)
    signed = cdig[msg_index.long()].clone()
    signed[bad, 0] ^= 1
    pks, sigs = device.keygen_sign(cseeds[voters], signed)
    offs = (torch.arange(m + 1, device="cuda", dtype=torch.int32) * Q)
    committee_pks, _ = device.keygen_sign(cseeds, torch.zeros((N, 32), dtype=torch.uint8, device="cuda"))
    out = {"N": N, "Q": Q, "nv": nv, "m": m, "cdig": cdig, "msg_index": msg_index, "offs": offs, "pks": pks,
           "sigs": sigs, "bad": bad, "committee_pks": committee_pks}
    if clean:
        # the same certificates with every vote valid (dalek's batch equation pays on clean traffic)
        out["clean_pks"], out["clean_sigs"] = device.keygen_sign(cseeds[voters], cdig[msg_index.long()])
        out["no_bad"] = torch.zeros_like(bad)
    torch.cuda.synchronize()
    return out


def cert_shard(offs, world: int, rank: int):
    """Certificates [c0, c1) of rank `rank`: whole certificates, balanced by votes -- the cut before
    rank r is the first certificate boundary at or past r/world of the votes (nwc_cert_cuts)."""
    offs = np.asarray(offs, dtype=np.int64)
    m, nv = len(offs) - 1, int(offs[-1])

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return m
        return int(np.searchsorted(offs, nv * r // world, side="left"))
    return cut(rank), cut(rank + 1)


def bench_cfg3(lib, m: int, steps: int, cpu_budget: float = 0.0):
    """BASELINE config 3: 100-node committee, m certificates x 67 votes (quorum 2N/3+1,
    config/src/lib.rs:181-186), each vote invalid with p = 0.01 (signed over another digest).
    Leaf equations for every vote + per-certificate AND; bad-vote sets checked against the
    construction.  Timed without any key cache (the per-vote ladder; dalek's batch equation over
    sub-batches), with the launch keys the library detects itself (no nwc_set_committee: first
    launch incl. the census and the 100 keys' comb builds, then steady state), and with the
    committee key cache."""
    from narwhal_amd import _lib, device
    import torch
    inst = make_cfg3(m)
    N, Q, nv = inst["N"], inst["Q"], inst["nv"]
    cdig, msg_index, offs, pks, sigs, bad = (inst[k] for k in ("cdig", "msg_index", "offs", "pks", "sigs", "bad"))
    committee_pks, clean_pks, clean_sigs, no_bad = (inst[k] for k in ("committee_pks", "clean_pks", "clean_sigs", "no_bad"))
    out = {}
    legs = (("no_cache", False, "leaf", pks, sigs, bad), ("no_cache_straus", False, "straus", pks, sigs, bad),
            ("clean_no_cache", False, "leaf", clean_pks, clean_sigs, no_bad),
            ("clean_no_cache_straus", False, "straus", clean_pks, clean_sigs, no_bad),
            ("no_cache_msm", False, "msm", pks, sigs, bad),
            ("clean_no_cache_msm", False, "msm", clean_pks, clean_sigs, no_bad),
            ("launch_keys", False, "launch", pks, sigs, bad), ("cache", True, "leaf", pks, sigs, bad),
            ("dalek_launch_keys", False, "dalek", pks, sigs, bad),
            ("clean_dalek_launch_keys", False, "dalek", clean_pks, clean_sigs, no_bad))
    only = os.environ.get("NWC_BENCH_CFG3_LEGS")   # profiling: a comma-separated subset of the legs
    for tag, use_cache, eq, P, S, want_bad in legs:
        if only and tag not in only.split(","):
            continue
        progress("config 3: " + tag)
        _lib.check(lib.nwc_set_committee(None, 0))   # no committee cache, launch keys emptied
        _lib.diag_set("launch_keys", 1 if eq in ("launch", "dalek") else 0)
        if use_cache:
            cpk = committee_pks.cpu().numpy()
            _lib.check(lib.nwc_set_committee(_lib.buf(cpk), N))
        words = torch.empty(device.words_for(nv), dtype=torch.int64, device="cuda")
        if eq == "straus":
            run = lambda: device.cert_reduce(device.verify_batch_straus(cdig, offs, msg_index, P, S, out=words),  # noqa
                                             offs, nv)
        elif eq in ("msm", "dalek"):
            # the same entry: launch keys off -> Pippenger groups first; on -> comb leaves + dalek's
            # equation per certificate over the failing votes (resolve.h)
            run = lambda: device.cert_reduce(device.verify_batch_msm(cdig, offs, msg_index, P, S, out=words),  # noqa
                                             offs, nv)
            st0 = device.msm_stats()
        else:
            run = lambda: device.cert_reduce(device.verify(cdig, P, S, strict=False, msg_index=msg_index,  # noqa
                                                           out=words), offs, nv)
        # the MSM entry's skip policy runs in cycles of 8 launches on a high bad-vote rate (one that
        # measures, 7 that skip the equation): its legs start from the measuring state (first call
        # with the policy off) and time whole cycles
        nsteps = max(8, (steps + 7) // 8 * 8) if eq == "msm" else steps
        if eq == "msm":
            _lib.diag_set("msm_adapt", 0)
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        first_ms = (time.perf_counter() - t0) * 1e3
        if eq == "msm":
            _lib.diag_set("msm_adapt", 1)
        t0 = time.perf_counter()
        for _ in range(nsteps):
            cw, bw = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / nsteps
        got_bad = torch.from_numpy(device.unpack_bits(bw, nv)).cuda()
        ok = bool((got_bad == want_bad).all())
        cert_ok = torch.from_numpy(device.unpack_bits(cw, m)).cuda()
        ok = ok and bool((cert_ok == ~want_bad.view(m, Q).any(dim=1)).all())
        out[tag] = {"votes_per_s": nv / dt, "certs_per_s": m / dt, "ms_per_step": dt * 1e3, "parity_ok": ok,
                    "first_call_ms": first_ms,
                    "equation": {"straus": "dalek batch equation over sub-batches of ~12 votes (Straus per lane), leaves for failing sub-batches",
                                 "msm": "dalek batch equation per group of up to 4,096 votes as a Pippenger MSM (one wave per group, keys "
                                        "aggregated, wavefront-level bucket reduction), Straus sub-batches for failing groups, "
                                        "leaves for failing sub-batches; device-side skip policy while most groups fail",
                                 "launch": "per-vote leaves; the launch's repeated keys detected by the library (no nwc_set_committee), "
                                           "their combs built on the first call, comb kernel from then on",
                                 "dalek": "dalek's batch semantics (nwc_dev_verify_batch_msm with launch keys): comb leaves for every vote, "
                                          "then dalek's equation once per certificate over the votes they reject, in E[8] (resolve.h)"
                                 }.get(eq, "per-vote leaves"),
                    "bad_rate": 0.01 if want_bad is bad else 0.0}
        if eq in ("msm", "dalek"):
            st1 = device.msm_stats()
            out[tag]["msm_groups"] = {"passed": st1[0] - st0[0], "failed": st1[1] - st0[1],
                                      "key_overflow": st1[2] - st0[2], "skipped": st1[3] - st0[3],
                                      "calls": nsteps + 1}
        if eq in ("launch", "dalek"):
            h = ctypes.c_uint32()
            _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
            out[tag]["launch_keys_held"] = h.value
        # input bytes per vote: key 32 + signature 64 + its certificate index 4 + a 67th of a digest
        prof = {"launch_keys": ("c3lk", "k_verify_comb", "k_verify_comb", ()),
                "dalek_launch_keys": ("c3dk", "k_verify_comb", "k_verify_comb",
                                      ("k_list_failing", "k_vote_resolve", "k_resolve_apply")),
                "clean_no_cache_msm": ("c3msm", "k_verify_msm", None, ())}.get(tag)
        if prof:
            out[tag]["roofline"] = roofline_extra(prof[0], prof[1], prof[2], nv, "vote", dt * 1e3, nv,
                                                  100 + 32.0 / Q, prof[3])
    _lib.check(lib.nwc_set_committee(None, 0))
    _lib.diag_set("launch_keys", 1)
    if not only or "host_abi_launch_keys" in only.split(","):
        out["host_abi_launch_keys"] = bench_cfg3_host_abi(lib, cdig, offs, pks, sigs, bad, m, Q)
    if cpu_budget > 0:
        out["cpu_baseline"] = cpu_baseline_cfg3(cdig, pks, sigs, m, Q, bad, cpu_budget)
    out["workload"] = "cfg3: %d certificates x %d votes, 1%% invalid, leaf equations + certificate AND + bad-vote set" % (m, Q)
    out["bad_votes"] = int(bad.sum().item())
    out["failing_certs"] = int(bad.view(m, Q).any(dim=1).sum().item())
    return out


def bench_cfg3_sharded(lib, rank: int, world: int, m: int, steps: int):
    """Config 3 at world > 1: whole certificates sharded over the ranks, balanced by
    votes (cert_shard = nwc_cert_cuts), no data-path collective.  Every rank builds the same
    instance (seeded), keeps its certificates' votes resident in its GPU's HBM and runs the
    production batch-leaf path (launch keys detected by the library: the first call includes the
    census and the comb builds, then `steps` timed calls); value = all ranks' votes / the slowest
    rank's time.  The certificate and bad-vote words are then all-gathered over the process group
    (timed separately; not needed for correctness: each rank holds its own verdicts) and rank 0
    checks the whole set against the construction."""
    from narwhal_amd import _lib, device
    import torch
    import torch.distributed as dist
    inst = make_cfg3(m, clean=False)
    Q, nv = inst["Q"], inst["nv"]
    c0, c1 = cert_shard(inst["offs"].cpu().numpy(), world, rank)
    v0, v1 = c0 * Q, c1 * Q
    mc, nvl = c1 - c0, v1 - v0
    cdig = inst["cdig"][c0:c1].contiguous()
    pks, sigs = inst["pks"][v0:v1].contiguous(), inst["sigs"][v0:v1].contiguous()
    offs = (inst["offs"][c0:c1 + 1] - v0).contiguous()
    msg_index = (inst["msg_index"][v0:v1] - c0).contiguous()
    bad = inst["bad"]
    del inst
    _lib.check(lib.nwc_set_committee(None, 0))
    _lib.diag_set("launch_keys", 1)
    words = torch.empty(device.words_for(max(nvl, 1)), dtype=torch.int64, device="cuda")
    run = lambda: device.cert_reduce(device.verify(cdig, pks, sigs, strict=False, msg_index=msg_index,  # noqa: E731
                                                   out=words), offs, nvl)
    barrier(world)
    t0 = time.perf_counter()
    run()
    barrier(world)
    first_ms = max_over_ranks((time.perf_counter() - t0) * 1e3, world)
    t0 = time.perf_counter()
    for _ in range(steps):
        cw, bw = run()
    barrier(world)
    dt = max_over_ranks((time.perf_counter() - t0) / steps, world)
    # gather: per rank its certificate words and bad-vote words, padded to the largest shard
    cmax = max(cert_shard(np.arange(m + 1) * Q, world, r)[1] - cert_shard(np.arange(m + 1) * Q, world, r)[0]
               for r in range(world))
    cwords, vwords = device.words_for(cmax), device.words_for(cmax * Q)
    pc = torch.zeros(cwords, dtype=torch.int64, device="cuda")
    pv = torch.zeros(vwords, dtype=torch.int64, device="cuda")
    pc[:cw.numel()] = cw
    pv[:bw.numel()] = bw
    allc = torch.empty(world * cwords, dtype=torch.int64, device="cuda")
    allv = torch.empty(world * vwords, dtype=torch.int64, device="cuda")
    barrier(world)
    tg = time.perf_counter()
    dist.all_gather_into_tensor(allc, pc)
    dist.all_gather_into_tensor(allv, pv)
    barrier(world)
    gather_ms = max_over_ranks((time.perf_counter() - tg) * 1e3, world)
    ok = True
    if rank == 0:
        got_cert, got_bad = [], []
        for r in range(world):
            r0, r1 = cert_shard(np.arange(m + 1) * Q, world, r)
            got_cert.append(device.unpack_bits(allc[r * cwords:(r + 1) * cwords], r1 - r0))
            got_bad.append(device.unpack_bits(allv[r * vwords:(r + 1) * vwords], (r1 - r0) * Q))
        want_bad = bad.cpu().numpy()
        ok = bool((np.concatenate(got_bad) == want_bad).all() and
                  (np.concatenate(got_cert) == ~want_bad.reshape(m, Q).any(axis=1)).all())
    okt = torch.tensor([1 if ok else 0], dtype=torch.int64, device="cuda")
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    h = ctypes.c_uint32()
    _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
    return {"workload": "cfg3: %d certificates x %d votes, 1%% invalid, whole certificates sharded %d ways (balanced by "
                        "votes), launch keys, certificate AND + bad-vote set" % (m, Q, world),
            "launch_keys": {"votes_per_s": nv / dt, "certs_per_s": m / dt, "ms_per_step": dt * 1e3,
                            "first_call_ms": first_ms, "launch_keys_held": h.value},
            "votes_per_gpu": nvl, "scaling": "strong", "verdict_allgather_ms": gather_ms,
            "allgather_needed": False, "parity_ok": bool(okt.item() == 1)}


def bench_cfg3_host_abi(lib, cdig, offs, pks, sigs, bad, m: int, Q: int, reps: int = 3):
    """Config 3 through the crate's drop-in entry: nwc_verify_batch_many from pageable host buffers
    (certificate digests, vote offsets, 6.7M keys and signatures in; certificate and bad-vote
    bitmaps out), no nwc_set_committee -- the launch keys pick the committee up on the first call.
    PCIe-inclusive; first call (keys join) and the median of the next `reps`."""
    from narwhal_amd import _lib
    # offsets are int32 < 2^31: the same bytes as the uint32 the ABI reads
    d, o, p, s = (np.ascontiguousarray(t.cpu().numpy()) for t in (cdig, offs, pks, sigs))
    nv = p.shape[0]
    cert = ctypes.create_string_buffer((m + 7) // 8)
    badb = ctypes.create_string_buffer((nv + 7) // 8)
    call = lambda: lib.nwc_verify_batch_many(_lib.buf(d), _lib.buf(o), _lib.buf(p), _lib.buf(s), m, cert, badb)  # noqa: E731
    t0 = time.perf_counter()
    _lib.check(call())
    first = time.perf_counter() - t0
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _lib.check(call())
        ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    want_bad = bad.cpu().numpy()
    got_bad = np.unpackbits(np.frombuffer(badb.raw, np.uint8), bitorder="little")[:nv].astype(bool)
    got_cert = np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:m].astype(bool)
    ok = bool((got_bad == want_bad).all() and (got_cert == ~want_bad.reshape(m, Q).any(axis=1)).all())
    h = ctypes.c_uint32()
    _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
    return {"workload": "cfg3 from pageable host buffers through nwc_verify_batch_many (H2D + verify + D2H), "
                        "no nwc_set_committee", "votes_per_s": nv / med, "ms_per_call": med * 1e3,
            "first_call_ms": first * 1e3, "reps": reps, "parity_ok": ok, "launch_keys_held": h.value}


def make_cfg3_wire(m: int, N: int = 100, Q: int = 67):
    """cfg 3 as the primary receives it: m bincode `PrimaryMessage::Certificate`s of a 100-node
    committee (stake 1, worker 0), each header with 67 parents, 67 votes by distinct members, 1 %
    of votes invalid (signed over another digest).  Fixed layout (10,100 B per certificate):
      0 u32 variant 2 | 4 str author (u64 44 + base64) | 56 u64 round | 64 u64 P = 0 |
      72 u64 Q = 67 | 80 parents 67 x 32 | 2224 id | 2256 signature | 2320 u64 V = 67 |
      2328 V x (u64 44, base64 key, 64-B signature)
    Keys and signatures come from the GPU signer; digests from hashlib (workload construction)."""
    import base64
    import torch
    from narwhal_amd import device
    cseeds = device.derive32(b"nw-committee", 0, N)
    cpk, _ = device.keygen_sign(cseeds, torch.zeros((N, 32), dtype=torch.uint8, device="cuda"))
    cpk_h = cpk.cpu().numpy()
    b64 = np.frombuffer(b"".join(base64.b64encode(k.tobytes()) for k in cpk_h), np.uint8).reshape(N, 44)
    rng = np.random.default_rng(0x4E57)
    author = rng.integers(0, N, m)
    voters = np.argsort(rng.random((m, N)), axis=1)[:, :Q]
    rounds = (np.arange(m, dtype=np.uint64) % 1000) + 1
    parents = rng.integers(0, 256, (m, Q, 32), dtype=np.uint8)
    # Header.parents is a BTreeSet<Digest>: serialised in ascending byte order (what every honest
    # encoder sends; the GPU decoder canonicalises any other order before Header::digest)
    order = np.lexsort(parents.transpose(2, 0, 1)[::-1], axis=-1)
    parents = np.take_along_axis(parents, order[:, :, None], axis=1)
    ids = np.empty((m, 32), np.uint8)
    cdig = np.empty((m, 32), np.uint8)
    for c in range(m):
        a32 = cpk_h[author[c]].tobytes()
        r8 = int(rounds[c]).to_bytes(8, "little")
        ids[c] = np.frombuffer(hashlib.sha512(a32 + r8 + parents[c].tobytes()).digest()[:32], np.uint8)
        cdig[c] = np.frombuffer(hashlib.sha512(ids[c].tobytes() + r8 + a32).digest()[:32], np.uint8)
    t_ids, t_cd = torch.from_numpy(ids).cuda(), torch.from_numpy(cdig).cuda()
    _, hsig = device.keygen_sign(cseeds[torch.from_numpy(author).cuda()].contiguous(), t_ids)
    signed = t_cd.repeat_interleave(Q, dim=0)
    bad = torch.from_numpy(rng.random(m * Q) < 0.01).cuda()
    signed[bad, 0] ^= 1
    _, vsig = device.keygen_sign(cseeds[torch.from_numpy(voters.reshape(-1)).cuda()].contiguous(), signed)
    SZ = 2328 + Q * 116
    buf = np.zeros((m, SZ), np.uint8)
    buf[:, 0:4] = np.frombuffer((2).to_bytes(4, "little"), np.uint8)
    buf[:, 4:12] = np.frombuffer((44).to_bytes(8, "little"), np.uint8)
    buf[:, 12:56] = b64[author]
    buf[:, 56:64] = rounds.view(np.uint8).reshape(m, 8)
    buf[:, 72:80] = np.frombuffer(Q.to_bytes(8, "little"), np.uint8)
    buf[:, 80:2224] = parents.reshape(m, Q * 32)
    buf[:, 2224:2256] = ids
    buf[:, 2256:2320] = hsig.cpu().numpy()
    buf[:, 2320:2328] = np.frombuffer(Q.to_bytes(8, "little"), np.uint8)
    votes = buf[:, 2328:].reshape(m, Q, 116)
    votes[:, :, 0:8] = np.frombuffer((44).to_bytes(8, "little"), np.uint8)
    votes[:, :, 8:52] = b64[voters]
    votes[:, :, 52:116] = vsig.cpu().numpy().reshape(m, Q, 64)
    exp_bad_cert = bad.view(m, Q).any(dim=1).cpu().numpy()
    return buf, cpk_h, exp_bad_cert


def bench_cfg3_wire(lib, m: int, steps: int):
    """Core::sanitize_certificate for m wire certificates (nwc_dev_sanitize_messages, bytes resident in
    HBM): decode + digests + committee checks + header signature + 67 vote leaves per certificate."""
    from narwhal_amd import _lib
    import torch
    N = 100
    buf, cpk, exp_bad = make_cfg3_wire(m, N)
    n_ = len(cpk)
    offs_c = (ctypes.c_uint32 * (n_ + 1))(*range(n_ + 1))
    cpk = np.ascontiguousarray(cpk)
    _lib.check(lib.nwc_set_committee_config(_lib.buf(cpk), (ctypes.c_uint64 * n_)(*([1] * n_)),
                                            n_, offs_c, (ctypes.c_uint32 * n_)(*([0] * n_))))
    SZ = buf.shape[1]
    data = torch.zeros(m * SZ + 64, dtype=torch.uint8, device="cuda")
    data[:m * SZ] = torch.from_numpy(buf.reshape(-1)).cuda()
    offs = torch.arange(m + 1, dtype=torch.int64, device="cuda") * SZ
    codes = torch.empty(m, dtype=torch.int32, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    run = lambda: _lib.check(lib.nwc_dev_sanitize_messages(  # noqa: E731
        ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offs.data_ptr()), m, m * SZ, 0, None,
        ctypes.c_void_p(codes.data_ptr()), None, stream))
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    got = codes.cpu().numpy()
    ok = bool(((got == 1) == exp_bad).all() and ((got == 0) == ~exp_bad).all())
    # host ABI (wire bytes in host memory, PCIe-inclusive)
    hoffs = np.arange(m + 1, dtype=np.uint64) * SZ
    hcodes = np.zeros(m, np.int32)
    flat = buf.reshape(-1)
    hts = []
    for rep in range(8):   # the first call sizes the staging arena: not timed
        t0 = time.perf_counter()
        _lib.check(lib.nwc_sanitize_messages(_lib.buf(flat), _lib.buf(hoffs), m, 0, None, _lib.buf(hcodes), None, None))
        hts.append(time.perf_counter() - t0)
    hdt = sorted(hts[1:])[len(hts[1:]) // 2]   # the median of 7 calls (host memory bandwidth varies)
    _lib.check(lib.nwc_set_committee(None, 0))
    return {"workload": "cfg3 wire: %d bincode Certificate messages (100-node committee, 67 parents, 67 votes, "
                        "1%% bad votes) -> DagError codes" % m,
            "certs_per_s": m / dt, "votes_per_s": m * 67 / dt, "ms_per_step": dt * 1e3,
            "wire_GBps": m * SZ / dt / 1e9, "parity_ok": ok and bool((hcodes == got).all()),
            "host_abi_certs_per_s": m / hdt, "failing_certs": int(exp_bad.sum())}


def bench_cfg5(lib, rank: int, world: int, total: int, steps: int, cpu_budget: float = 0.0):
    """BASELINE config 5: `total` (64M) signatures sharded in contiguous ranges of total/world over
    the ranks (strong scaling), 99 % honest-valid (cfg-2 seed scheme on the global index) and 1 %
    edge cases spread evenly over the golden edge-case classes (tests/golden/ed25519_verify.json:
    small-order / non-canonical A and R, s >= l, ...) with their expected strict verdicts.  Per-shard
    verdict words are all-gathered over RCCL (timed separately) and, as the alternative, copied
    D2H; the gather is not needed for correctness."""
    import torch
    from narwhal_amd import device
    per = total // world
    first = rank * per
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_verify.json")))["cases"]
    edge = [c for c in gold if len(c["msg"]) == 64 and not c["strict"]] + \
           [c for c in gold if len(c["msg"]) == 64 and c["strict"] and "ref" not in c["name"]][:8]
    em = torch.tensor(np.stack([np.frombuffer(bytes.fromhex(c["msg"]), np.uint8) for c in edge]), device="cuda")
    ep = torch.tensor(np.stack([np.frombuffer(bytes.fromhex(c["pk"]), np.uint8) for c in edge]), device="cuda")
    es = torch.tensor(np.stack([np.frombuffer(bytes.fromhex(c["sig"]), np.uint8) for c in edge]), device="cuda")
    exp_edge = torch.tensor([bool(c["strict"]) for c in edge], device="cuda")
    msgs = device.derive32(b"nw-msg", first, per)
    seeds = device.derive32(b"nw-seed", first, per)
    pks, sigs = device.keygen_sign(seeds, msgs)
    del seeds
    gidx = torch.arange(first, first + per, device="cuda", dtype=torch.int64)
    slot = torch.nonzero(gidx % 100 == 37).squeeze(1)
    cls = (gidx[slot] // 100) % len(edge)
    msgs[slot] = em[cls]
    pks[slot] = ep[cls]
    sigs[slot] = es[cls]
    expected = torch.ones(per, dtype=torch.bool, device="cuda")
    expected[slot] = exp_edge[cls]
    words = torch.empty(device.words_for(per), dtype=torch.int64, device="cuda")
    run = lambda: device.verify(msgs, pks, sigs, strict=True, out=words)  # noqa: E731
    run()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    barrier(world)
    dt = max_over_ranks((time.perf_counter() - t0) / steps, world)
    got = torch.from_numpy(device.unpack_bits(words, per)).cuda()
    ok = bool((got == expected).all())
    gather_ms = None
    allw = None
    if world > 1:
        import torch.distributed as dist
        allw = torch.empty(world * words.numel(), dtype=torch.int64, device="cuda")
        barrier(world)
        tg = time.perf_counter()
        dist.all_gather_into_tensor(allw, words)
        barrier(world)
        gather_ms = max_over_ranks((time.perf_counter() - tg) * 1e3, world)
    td = time.perf_counter()
    host_words = words.cpu()
    d2h_ms = max_over_ranks((time.perf_counter() - td) * 1e3, world)
    if allw is not None:
        ok = ok and bool((allw[rank * words.numel():(rank + 1) * words.numel()] == words).all())
    okt = torch.tensor([1 if ok else 0], dtype=torch.int64, device="cuda")
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    del host_words
    out = {"workload": "cfg5: %d signatures (1%% edge cases over %d golden classes) sharded %d ways, verify_strict"
                       % (total, len(edge), world),
           "verifies_per_s": total / dt, "ms_per_pass": dt * 1e3, "per_gpu": per, "scaling": "strong",
           "verdict_allgather_ms": gather_ms, "verdict_d2h_ms": d2h_ms, "allgather_needed": False,
           "edge_slots_per_gpu": int(slot.numel()), "parity_ok": bool(okt.item() == 1)}
    # the strict kernel over launches of at most NWC_VERIFY_MAX_LAUNCH (16M) equations
    out["roofline"] = roofline_extra("c5", "k_verify<true, false, false, false>", "k_verify", min(per, 16 << 20),
                                     "verify", dt * 1e3, per, 128)
    if cpu_budget > 0 and rank == 0 and world == 1:
        # the restatement's verify_strict on every CPU the box grants, on a
        # prefix of the same mixed signatures (edge cases included), verdicts checked
        from tests.oracle_lib import load_oracle
        orc = load_oracle()
        th = cpu_threads()
        k = 4096 * th
        while True:
            m_, p_, s_ = (t[:k].cpu().numpy() for t in (msgs, pks, sigs))
            t0 = time.perf_counter()
            v = orc.strict_many(m_, p_, s_, th)
            cdt = time.perf_counter() - t0
            if cdt > cpu_budget / 4 or k >= per:
                break
            k = min(per, int(k * max(2.0, cpu_budget / max(cdt, 1e-3) * 0.8)))
        out["cpu_baseline"] = {"value": k / cdt, "unit": "verifies/s", "cores": th, "kind": "port",
                               "value_per_thread": k / cdt / th,
                               "parity_ok": bool((v == expected[:k].cpu().numpy()).all()),
                               "sample": "first %d of the cfg-5 signatures (%d edge cases; C restatement of dalek "
                                         "verify_strict, %d threads, %.1f s)" % (k, int((gidx[:k] % 100 == 37).sum()), th, cdt)}
    return out


# ---- host ------------------------------------------------------------------------------------
def cpu_threads() -> int:
    """Every host CPU this process may use: the affinity mask, capped by the cgroup's CPU quota
    (on the GPU box: 16 CPUs of a 2 x 64-core host; OMP_NUM_THREADS says the same)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = cgroup_cpus()
    if q:
        n = min(n, q)
    return max(1, n)


def cgroup_cpus():
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return None


def host_info():
    """the CPU model and core counts next to every CPU baseline."""
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    phys = set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (x.strip() for x in line.split(":", 1))
                cur[k] = v
            elif cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return {"cpu_model": model, "logical_cpus": os.cpu_count(), "physical_cores": len(phys) or None,
            "affinity_cpus": aff, "cgroup_cpu_quota": cgroup_cpus(), "nproc": int(os.popen("nproc").read() or 0),
            "threads_used": cpu_threads()}


def cpu_baseline_verify(msgs, pks, sigs, budget_s: float):
    from tests.oracle_lib import load_oracle
    orc = load_oracle()
    th = cpu_threads()
    m, p, s = (t.cpu().numpy() for t in (msgs, pks, sigs))
    # calibrate on a small slice, then size the sample to ~budget_s of wall time
    k = 2048
    t0 = time.perf_counter()
    v = orc.strict_many(m[:k], p[:k], s[:k], th)
    dt = time.perf_counter() - t0
    n = int(min(len(p), max(k, k * budget_s / max(dt, 1e-6))))
    t0 = time.perf_counter()
    v = orc.strict_many(m[:n], p[:n], s[:n], th)
    dt = time.perf_counter() - t0
    assert v.all(), "oracle rejected a valid signature"
    out = {"value": n / dt, "unit": "verifies/s", "cores": th, "kind": "port", "value_per_thread": n / dt / th,
           "host": host_info(),
           "sample": "%d of the cfg-2 triples (C restatement of dalek verify_strict, %d threads = every CPU the "
                     "box grants this process, %.1f s)" % (n, th, dt)}
    try:   # a third-party point: its absence must not cost the line
        out["openssl"] = cpu_verify_openssl(m, p, s, th, budget_s / 2)
    except Exception as e:  # noqa: BLE001
        out["openssl"] = {"error": repr(e)}
    return out


def cpu_verify_openssl(m, p, s, th: int, budget_s: float):
    """SURVEY.md §8(d)'s optional third-party point: OpenSSL EVP Ed25519 single verification
    (oracle/openssl_ed25519.c) on the same cfg-2 triples and threads. Not dalek semantics (it
    accepts non-canonical and small-order encodings verify_strict rejects); on these honest
    triples both accept, which the call asserts."""
    from tests.oracle_lib import openssl_verify_many
    k = 2048
    t0 = time.perf_counter()
    openssl_verify_many(m[:k], p[:k], s[:k], th)
    dt = time.perf_counter() - t0
    n = int(min(len(p), max(k, k * budget_s / max(dt, 1e-6))))
    t0 = time.perf_counter()
    v = openssl_verify_many(m[:n], p[:n], s[:n], th)
    dt = time.perf_counter() - t0
    assert v.all(), "OpenSSL rejected a valid signature"
    return {"value": n / dt, "unit": "verifies/s", "cores": th, "kind": "third-party",
            "semantics": "not dalek semantics (OpenSSL %s EVP Ed25519)" % openssl_version(),
            "sample": "%d of the cfg-2 triples, %d threads, %.1f s" % (n, th, dt)}


def openssl_version():
    import ssl
    return ssl.OPENSSL_VERSION.split()[1] if ssl.OPENSSL_VERSION.startswith("OpenSSL") else ssl.OPENSSL_VERSION


def cpu_baseline_digest(budget_s: float, data, outs):
    """The C restatement's SHA-512 (oracle/, "port") on the host cores over the first 4 x threads
    batches of the GPU leg's own pool (copied from HBM), every CPU digest compared byte for byte
    with the GPU's digest of the same batch."""
    from tests.oracle_lib import load_oracle
    orc = load_oracle()
    th = cpu_threads()
    nb = 4 * th
    rows = data[:nb * CFG4_STRIDE].view(nb, CFG4_STRIDE)[:, :CFG4_BATCH_BYTES].cpu().numpy()
    host = np.ascontiguousarray(rows).reshape(-1)
    offs = np.arange(nb + 1, dtype=np.uint64) * CFG4_BATCH_BYTES
    gpu = outs[:nb].cpu().numpy()
    t0 = time.perf_counter()
    reps = 0
    while True:
        got = orc.digest_many(host, offs, th)
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    out = {"value": reps * host.size / dt / 1e9, "unit": "GB/s", "cores": th, "kind": "port",
           "value_per_thread": reps * host.size / dt / 1e9 / th,
           "parity_ok": bool((np.asarray(got).reshape(nb, 32) == gpu).all()),
           "sample": "%d x %d cfg-4 batches of the GPU leg's pool (C restatement SHA-512, %d threads, %.1f s); "
                     "every digest compared with the GPU's" % (reps, nb, th, dt)}
    out["openssl"] = cpu_digest_openssl(host, nb, th, budget_s / 2, gpu)
    return out


def cpu_digest_openssl(blob: np.ndarray, nb: int, th: int, budget_s: float, gpu: np.ndarray):
    """SURVEY.md §8(d)'s digest baseline: OpenSSL SHA-512 (hashlib, which releases the GIL on
    large inputs) over the same cfg-4 batches on `th` host threads, one batch per call; its digests
    compared with the GPU's."""
    from concurrent.futures import ThreadPoolExecutor
    mv = memoryview(blob)
    views = [mv[b * CFG4_BATCH_BYTES:(b + 1) * CFG4_BATCH_BYTES] for b in range(nb)]
    with ThreadPoolExecutor(th) as ex:
        t0 = time.perf_counter()
        reps = 0
        while True:
            got = list(ex.map(lambda v: hashlib.sha512(v).digest()[:32], views))
            reps += 1
            if time.perf_counter() - t0 > budget_s:
                break
        dt = time.perf_counter() - t0
    ok = all(g == gpu[b].tobytes() for b, g in enumerate(got))
    return {"value": reps * nb * CFG4_BATCH_BYTES / dt / 1e9, "unit": "GB/s", "cores": th, "kind": "openssl",
            "parity_ok": ok, "sample": "%d x %d cfg-4 batches (hashlib/OpenSSL SHA-512, %d threads, %.1f s); every "
                                       "digest compared with the GPU's" % (reps, nb, th, dt)}


def roofline_verify(vpc, n: int, kernel_ms: float, effective_tops: float, clock=None):
    """k_verify's roofline entry.  achieved = the VALU lane-instructions one launch issues (this
    build's SQ_INSTS_VALU x 64 from the committed rocprofv3 pass, profiles/<round>/summary.json)
    over the launch's duration measured live with HIP events; peak = the guide's VALU issue rate.
    frac_vop3_rate relates it to the measured 4-cycle issue of the VOP3 integer class the kernel
    consists of; effective_frac prices the dalek work model (W_strict) instead of the instructions
    actually issued (the half-size ladder issues fewer, so it can exceed the hardware fraction)."""
    out = {"bound": "valu", "unit": "T lane-ops/s", "peak": VALU_PEAK_TOPS, "kernel": "k_verify",
           "kernel_ms": kernel_ms, "verifies_per_launch": n,
           "peak_source": "MI355X_MICROARCH.md: wave64 VALU issue 2 cycles/SIMD x 4 SIMD x 256 CU x 2.4 GHz",
           "effective_frac": effective_tops / VALU_PEAK_TOPS,
           "work_model": "%d S + %d M + %d SHA-512 block per verify (dalek op model) x (%d, %d, %d) lane-ops"
                         % (W_S, W_M, W_SHA, OPS_S, OPS_M, OPS_SHA)}
    if vpc:
        ach = vpc["lane_ops_per_launch"] / (kernel_ms * 1e-3) / 1e12
        out.update({"achieved": ach, "frac": ach / VALU_PEAK_TOPS, "frac_vop3_rate": ach / VOP3_RATE_TOPS,
                    "valu_insts_per_verify": vpc["valu_insts_per_lane"],
                    "traffic": vpc["traffic"], "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
                    "traffic_per_verify": vpc["traffic"] / n, "algorithmic_bytes_per_verify": 128,
                    "traffic_over_algorithmic": vpc["traffic"] / (128.0 * n),
                    "rocprof_avg_ms": vpc["avg_ns"] * 1e-6, "pmc_source": vpc["source"]})
    else:
        out.update({"achieved": None, "frac": None, "traffic": None,
                    "pmc_source": "profiles/%s/summary.json missing" % PROFILE_ROUND})
    cyc, share = issue_cycles("k_verify")
    if cyc and out.get("frac"):
        # the true issue fraction: every wave instruction priced at its own class's issue cycles
        # (frac prices them all at 2, frac_vop3_rate all at 4); SIMD cycles at the 2.4 GHz peak
        out["frac_issue"] = out["frac"] * cyc / 2
        out["issue_census"] = {"avg_issue_cycles": cyc, "share_4cycle": share,
                               "source": os.path.relpath(CENSUS, ROOT) + " (tools/isa_census.py)"}
    if clock:
        # the shader clock this box held under the load, from the kernel's stamp build
        # (nwc_diag_verify_clock): the issue rate the clock allows, and the fraction of it reached
        out["clock_ghz"] = clock["clock_ghz"]
        out["clock"] = dict(clock, source="k_verify stamp build: median over waves of d(s_memtime)/d(s_memrealtime) "
                                          "x 100 MHz, one launch after ~2 s of back-to-back launches")
        if out.get("achieved"):
            out["frac_at_clock"] = out["achieved"] / (128 * 256 * clock["clock_ghz"] * 1e9 / 1e12)
            if out.get("frac_issue"):
                out["frac_issue_at_clock"] = out["frac_issue"] * 2.4 / clock["clock_ghz"]
    return out


# ---- main ------------------------------------------------------------------------------------
def bench_cfg4_host(group: int, pool: int = 256):
    """Config 4 from host memory through the worker's digester (`nwc_digester_*`):
    one group of `group` cfg-4 batches submitted at once, digests polled back -- from pageable
    memory (gathered into pinned stages) and from the digester's pinned receive arena (one DMA
    per group).  PCIe-inclusive; never the digest leg's value.  Every digest checked (hashlib)."""
    import numpy as np
    from narwhal_amd.processor import Digester
    host = make_cfg4_pool(pool).cpu().numpy()
    views = [host[b * CFG4_STRIDE:b * CFG4_STRIDE + CFG4_BATCH_BYTES] for b in range(pool)]
    want = [hashlib.sha512(v).digest()[:32] for v in views]
    r16 = (CFG4_BATCH_BYTES + 15) & ~15
    out = {"workload": "%d cfg-4 batches per group from host memory, nwc_digester (H2D + digest + D2H)" % group}

    def timed(dg, items):
        import gc
        ts = []
        for _ in range(3):   # the first group sizes the digester's device buffers: not counted
            gc.collect()
            gc.disable()     # a collection inside the submit loop costs tens of ms of Python time
            try:
                t0 = time.perf_counter()
                for i, v in enumerate(items):
                    dg.submit(v, i)
                t_sub = time.perf_counter() - t0
                got = []
                while len(got) < group:
                    got += dg.poll(1 << 16, 1_000_000)
                ts.append(time.perf_counter() - t0)
            finally:
                gc.enable()
            assert [t for t, _ in got] == list(range(group)) and all(d == want[t % pool] for t, d in got)
            out.setdefault("submit_ms", []).append(round(t_sub * 1e3, 2))
        return min(ts[1:])

    dg = Digester(group, 30_000_000)
    try:
        dt = timed(dg, [views[i % pool] for i in range(group)])
    finally:
        dg.close()
    out["stages_GBps"], out["stages_ms"] = group * CFG4_BATCH_BYTES / dt / 1e9, dt * 1e3
    dg = Digester(group, 30_000_000)
    try:
        arena = dg.arena(group * r16)
        items = []
        for i in range(group):
            a = arena[i * r16:i * r16 + CFG4_BATCH_BYTES]
            a[:] = views[i % pool]   # stands for the network read into the arena: not timed
            items.append(a)
        dt = timed(dg, items)
        direct = dg.direct_groups()
    finally:
        dg.close()
    out["arena_GBps"], out["arena_ms"], out["arena_direct_groups"] = group * CFG4_BATCH_BYTES / dt / 1e9, dt * 1e3, direct
    out["parity_ok"] = True
    return out


def bench_cfg2_host_abi(lib, msgs, pks, sigs, reps: int):
    """Config 2 end to end ("plus a separate end-to-end time"): the same triples
    from pageable host memory through nwc_verify_strict_many (PCIe in, chunk-pipelined, verdict
    bitmap out); never the headline value."""
    import ctypes
    import numpy as np
    from narwhal_amd import _lib
    m, p, s = (np.ascontiguousarray(t.cpu().numpy()) for t in (msgs, pks, sigs))
    n = p.shape[0]
    out = ctypes.create_string_buffer((n + 7) // 8)
    vp = ctypes.c_void_p
    call = lambda: lib.nwc_verify_strict_many(m.ctypes.data_as(vp), p.ctypes.data_as(vp), s.ctypes.data_as(vp),  # noqa: E731
                                              ctypes.c_size_t(n), out)
    _lib.check(call())
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _lib.check(call())
        ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    ok = bool(np.unpackbits(np.frombuffer(out.raw, np.uint8), bitorder="little")[:n].all())
    return {"workload": "cfg2 triples from pageable host buffers, nwc_verify_strict_many (H2D + verify + D2H)",
            "verifies_per_s": n / med, "ms_per_call": med * 1e3, "reps": reps, "verdicts_ok": ok}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--triples", "--n", dest="n", type=int, default=1 << 20,
                    help="triples per GPU (cfg 2: 1M); under torch.distributed.run spell it --triples")
    ap.add_argument("--digest-batches", type=int, default=100000, help="cfg 4: 100k batches (0 = skip)")
    ap.add_argument("--digest-pool", type=int, default=16384, help="distinct batches resident in HBM")
    ap.add_argument("--digest-steps", type=int, default=1)
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds per CPU-baseline leg (0 = skip)")
    ap.add_argument("--cfg3-certs", type=int, default=100000, help="config 3 certificates (0 = skip)")
    ap.add_argument("--cfg1-calls", type=int, default=10000, help="config 1 latency calls (0 = skip)")
    ap.add_argument("--wire-certs", type=int, default=20000, help="cfg 3 from wire bytes (0 = skip)")
    ap.add_argument("--cfg5-total", type=int, default=64 << 20, help="cfg 5 signatures over all ranks (0 = skip)")
    ap.add_argument("--host-digest-group", type=int, default=8192,
                    help="cfg 4 from host memory through nwc_digester: batches per group (0 = skip; needs --e2e-reps)")
    ap.add_argument("--clock-s", type=float, default=2.0,
                    help="seconds of back-to-back launches before the stamped clock launch (0 = skip)")
    ap.add_argument("--e2e-reps", type=int, default=3,
                    help="cfg 2 end to end through the host ABI from pageable host buffers (0 = skip)")
    args = ap.parse_args()

    import torch
    rank, world, local = dist_setup(args)
    from narwhal_amd import _lib, device
    lib = _lib.load(device_mask=1 << local)   # the library drives the same GPU as this rank

    # ---------------- verify leg (headline)
    progress("headline: config 2 verify")
    n = args.n
    msgs, pks, sigs = make_cfg2(rank, n)
    words = torch.empty(device.words_for(n), dtype=torch.int64, device="cuda")
    run = lambda: device.verify(msgs, pks, sigs, strict=True, out=words)  # noqa: E731
    for _ in range(args.warmup):
        run()
    # HIP events around every step, on the stream the library launches on (torch's current
    # stream), recorded inside the same timed loop as the wall clock
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier(world)
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        run()
        e1.record()
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    ok = bool(device.unpack_bits(words, n).all())
    kernel_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
    # verdict all-gather over RCCL (not needed for correctness; timed separately)
    gather_ms = None
    if world > 1:
        import torch.distributed as dist
        allw = torch.empty(world * words.numel(), dtype=torch.int64, device="cuda")
        barrier(world)
        tg = time.perf_counter()
        dist.all_gather_into_tensor(allw, words)
        barrier(world)
        gather_ms = max_over_ranks((time.perf_counter() - tg) * 1e3, world)
        ok = ok and bool(device.unpack_bits(allw, world * words.numel() * 64).all())
    value = world * n * args.steps / dt
    effective_tops = n / (kernel_ms * 1e-3) * ops_per_verify() / 1e12
    # the clock the chip held under this load (MI355X_MICROARCH.md DVFS item 6): ~2 s more of
    # back-to-back launches, then one launch of the kernel's stamp build (never the timed kernel)
    clock = None
    if args.clock_s > 0:
        progress("headline: in-kernel clock")
        reps = max(1, int(args.clock_s / max(kernel_ms * 1e-3, 1e-4)))
        for _ in range(reps):
            run()
        ghz, waves = device.verify_clock(msgs, pks, sigs, words)
        clock = {"clock_ghz": ghz, "waves": waves, "after_launches": reps,
                 "ok": bool(device.unpack_bits(words, n).all())}

    # reject side of the headline leg (outside the timed region): the same triples with 1 in 64
    # signatures corrupted (one bit of byte (i / 64) mod 64: R or s), verdicts equal to the construction
    bad_sigs = sigs.clone()
    ci = torch.arange(0, n, 64, device="cuda")
    bad_sigs[ci, (ci // 64) % 64] ^= 0x10
    rwords = torch.empty_like(words)
    device.verify(msgs, pks, bad_sigs, strict=True, out=rwords)
    want = np.ones(n, dtype=bool)
    want[::64] = False
    reject = {"corrupted": int(ci.numel()), "verdicts_ok": bool((device.unpack_bits(rwords, n) == want).all())}
    del bad_sigs, rwords

    # ---------------- digest leg (cfg 4)
    digest = None
    if args.digest_batches > 0:
        progress("config 4 digest")
        pool = min(args.digest_pool, args.digest_batches)
        data = make_cfg4_pool(pool)
        nb = args.digest_batches
        # message i = pool batch (i mod pool): 100k lanes in one launch, bytes read from HBM
        starts = (torch.arange(nb, dtype=torch.int64, device="cuda") % pool) * CFG4_STRIDE
        ends = starts + CFG4_BATCH_BYTES
        outs = torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
        dig = lambda: device.sha512_trunc32_ranges(data, starts, ends, out=outs)  # noqa: E731
        dig()
        devs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.digest_steps)]
        barrier(world)
        t0 = time.perf_counter()
        for e0, e1 in devs:
            e0.record()
            dig()
            e1.record()
        barrier(world)
        ddt = max_over_ranks(time.perf_counter() - t0, world)
        dk_ms = sum(e0.elapsed_time(e1) for e0, e1 in devs) / len(devs)
        dbytes = world * nb * CFG4_BATCH_BYTES * args.digest_steps
        # every one of the nb digests (outside the timed region): periodicity over the pool on the
        # device, the pool's bytes and digests against an independent host construction + hashlib
        dok, dcheck = check_cfg4_digests(data, outs, pool, nb, cpu_threads())
        dk_gbs = nb * CFG4_BATCH_BYTES / (dk_ms * 1e-3) / 1e9
        # launch_digest's choice: McNaughton-scheduled blocks above one wave per SIMD of messages
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        dkernel = "k_sha512_digest32_sched" if nb > 64 * 4 * cus else "k_sha512_digest32"
        digest = {"metric": "batch digest GB/s", "value": dbytes / ddt / 1e9, "unit": "GB/s",
                  "batches": nb, "batch_bytes": CFG4_BATCH_BYTES, "pool_distinct_batches": pool,
                  "parity_ok": dok, "parity": dcheck, "kernel": dkernel, "kernel_ms": dk_ms, "kernel_GBps": dk_gbs,
                  "hbm_frac": dk_gbs / HBM_PEAK_GBS,
                  "effective_valu_frac": dk_gbs * 1e9 / 128 * OPS_SHA / (VALU_PEAK_TOPS * 1e12)}

    extras = {}
    progress("extra configurations")
    if world == 1 and args.e2e_reps > 0:
        extras["cfg2_host_abi"] = bench_cfg2_host_abi(lib, msgs, pks, sigs, args.e2e_reps)
    if world == 1 and args.e2e_reps > 0 and args.host_digest_group > 0:
        try:   # 4.2 GB of pinned host memory: a box that refuses it still prints the line
            extras["cfg4_host"] = bench_cfg4_host(args.host_digest_group)
        except Exception as e:  # noqa: BLE001
            extras["cfg4_host"] = {"error": repr(e)}
    if args.cfg5_total > 0:
        extras["cfg5"] = bench_cfg5(lib, rank, world, args.cfg5_total, 2, args.cpu_budget / 2)
    if world == 1 and args.cfg3_certs > 0:
        extras["cfg3"] = bench_cfg3(lib, args.cfg3_certs, max(1, args.steps // 2),
                                    args.cpu_budget / 2 if rank == 0 else 0.0)
    elif args.cfg3_certs > 0:
        extras["cfg3"] = bench_cfg3_sharded(lib, rank, world, args.cfg3_certs, max(1, args.steps // 2))
    if world == 1 and args.cfg1_calls > 0:
        extras["cfg1"] = bench_cfg1(lib, args.cfg1_calls, cpu_baseline=args.cpu_budget > 0)
    if world == 1 and args.wire_certs > 0:
        extras["cfg3_wire"] = bench_cfg3_wire(lib, args.wire_certs, max(1, args.steps // 2))

    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        progress("CPU baselines")
        cpu = cpu_baseline_verify(msgs, pks, sigs, args.cpu_budget)
        if digest is not None:
            digest["cpu_baseline"] = cpu_baseline_digest(args.cpu_budget / 2, data, outs)

    vpc = profile_counters("nwc::k_verify<true, false, false, false>", "nwc::k_verify<true, false, false>",
                           "nwc::k_verify<true, false>")
    dpc = profile_counters("nwc::" + digest["kernel"]) if digest is not None else None
    if digest is not None and dpc:
        digest["traffic"] = dpc["traffic"]
        # counter fraction: this build's VALU lane-ops per launch (PMC) over the live kernel time
        digest["valu_frac"] = dpc["lane_ops_per_launch"] / (digest["kernel_ms"] * 1e-3) / (VALU_PEAK_TOPS * 1e12)
        digest["valu_frac_vop3_rate"] = digest["valu_frac"] * VALU_PEAK_TOPS / VOP3_RATE_TOPS
        dcyc, _ = issue_cycles(digest["kernel"])
        if dcyc:
            digest["valu_frac_issue"] = digest["valu_frac"] * dcyc / 2
        digest["pmc_source"] = dpc["source"]
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "verifies/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic: SHA-512-derived seeds/messages, RFC 8032 keygen+sign on the GPU (SURVEY.md §8(d) cfg 2)",
            "config": {"workload": "cfg2: %d independent (32-B msg, pk, sig) triples per GPU, all valid, "
                                   "verify_strict" % n,
                       "global_batch": world * n, "parallelism": "shard%d" % world,
                       "verdicts_ok": ok, "reject_check": reject, "verdict_allgather_ms": gather_ms,
                       "allgather_needed": False},
            "roofline": roofline_verify(vpc, n, kernel_ms, effective_tops, clock),
            "cpu_baseline": cpu,
            "digest": digest,
            "configs": extras,
            # the hash of the sources libnwc.so was compiled from (narwhal_amd/build.py source_id)
            "build_id": lib.nwc_build_id().decode(),
            "memory": _lib.memory_info(),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
