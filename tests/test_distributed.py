"""The N > 1 path's host logic with world_size-2 gloo on CPU: sharding, certificate cuts and the
verdict all-gather reproduce the single-process verdicts (oracle as the per-shard verifier)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from narwhal_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1000, 1 << 20, 64 * 1024 * 1024 + 5):
        for world in (1, 2, 4, 8):
            rs = [shard.shard_bounds(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c
            for lo, _ in rs:
                assert lo % 64 == 0 or lo == n


def test_cert_cuts_on_boundaries():
    rng = np.random.default_rng(0)
    sizes = rng.integers(0, 90, 500)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    for world in (1, 2, 3, 8):
        cuts = shard.cert_cuts(offs, world)
        assert cuts[0] == 0 and cuts[-1] == offs[-1]
        assert all(c in set(offs.tolist()) for c in cuts)
        assert cuts == sorted(cuts)


def _worker(rank, world, port, data, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.oracle_lib import load_oracle
    orc = load_oracle()
    m, p, s = data
    n = p.shape[0]
    lo, hi = shard.shard_bounds(n, world, rank)
    v = orc.strict_many(m[lo:hi], p[lo:hi], s[lo:hi], threads=1)
    words_len = (shard.shard_bounds(n, world, 0)[1] + 63) // 64
    packed = np.packbits(v.astype(np.uint8), bitorder="little")
    buf = np.zeros(words_len * 8, dtype=np.uint8)
    buf[:packed.size] = packed
    w = torch.from_numpy(buf.view(np.int64).copy())
    parts = shard.all_gather_words(w, world)
    counts = [shard.shard_bounds(n, world, r)[1] - shard.shard_bounds(n, world, r)[0] for r in range(world)]
    merged = shard.merge_words([t.numpy() for t in parts], counts)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        result_q.put((merged, float(t.item())))
    dist.destroy_process_group()


def test_two_rank_gloo_verdict_allgather(oracle):
    rng = np.random.default_rng(2)
    n = 300
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    sigs[::7, 50] ^= 1
    expect = oracle.strict_many(msgs, pks, sigs)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, (msgs, pks, sigs), q)) for r in range(2)]
    for pr in procs:
        pr.start()
    merged, mx = q.get()
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert (merged == expect).all()
    assert mx == 2.0


# ---- the library's own cut logic (nwc_shard_bounds / nwc_cert_cuts: the C++ that the host entry
# points use to split work over the devices of the init mask), against the Python twin above.
def _lib():
    from narwhal_amd import _lib as L
    return L, L.load(init=False)


def test_c_shard_bounds_match_python():
    import ctypes
    L, lib = _lib()
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    for n in (0, 1, 63, 64, 65, 4095, 4096, 4097, 1000, 1 << 20, 64 * 1024 * 1024 + 5):
        for world in (1, 2, 3, 4, 7, 8):
            prev = 0
            for r in range(world):
                assert lib.nwc_shard_bounds(n, world, r, ctypes.byref(lo), ctypes.byref(hi)) == 0
                assert (lo.value, hi.value) == shard.shard_bounds(n, world, r), (n, world, r)
                assert lo.value == prev and (lo.value % 64 == 0 or lo.value == n)   # whole verdict bytes
                prev = hi.value
            assert prev == n
    assert lib.nwc_shard_bounds(10, 0, 0, ctypes.byref(lo), ctypes.byref(hi)) == L.NWC_ERR_ARG
    assert lib.nwc_shard_bounds(10, 2, 2, ctypes.byref(lo), ctypes.byref(hi)) == L.NWC_ERR_ARG


def test_c_cert_cuts_match_python():
    L, lib = _lib()
    rng = np.random.default_rng(1)
    layouts = [np.zeros(1, np.int64),                                   # m = 0
               np.array([0, 0, 0, 0]),                                  # only empty certificates
               np.array([0, 67]),                                       # one certificate, m < devices
               np.array([0, 5, 5, 9]),                                  # m < devices, an empty one
               np.concatenate([[0], np.cumsum(rng.integers(0, 90, 500))]),
               np.concatenate([[0], np.cumsum(np.where(rng.random(300) < 0.3, 0, 67))])]
    for offs in layouts:
        m = len(offs) - 1
        o32 = np.ascontiguousarray(offs, dtype=np.uint32)
        for world in (1, 2, 3, 4, 8):
            cuts = np.zeros(world + 1, np.uint64)
            assert lib.nwc_cert_cuts(L.buf(o32), m, world, L.buf(cuts)) == 0
            assert cuts.tolist() == shard.cert_cuts(offs, world), (m, world)
            assert set(cuts.tolist()) <= set(offs.tolist())
            assert cuts[0] == 0 and cuts[-1] == offs[-1] and (np.diff(cuts.astype(np.int64)) >= 0).all()
