"""BASELINE config 4 at its full size, every digest checked (worker/src/processor.rs:38; the batch
bytes of worker/src/batch_maker.rs:81,119): the bench's own launch -- 100,000 ranges over a pool of
16,384 distinct 508,052-B batches resident in HBM, one k_sha512_digest32_sched launch -- with

  * out[i] == out[i mod pool] for all 100,000 digests (on the device), and
  * every pool batch's bytes equal to an independent numpy construction and its digest equal to
    hashlib's (OpenSSL) SHA-512[..32] (8.3 GB hashed on the host threads),

so ~98 messages per wave cross the McNaughton tape's lane hand-offs, as in the bench."""
import pytest

pytestmark = pytest.mark.gpu


def test_cfg4_full_size_every_digest():
    import torch
    import bench
    from narwhal_amd import device
    pool, nb = 16384, 100_000
    data = bench.make_cfg4_pool(pool)
    starts = (torch.arange(nb, dtype=torch.int64, device="cuda") % pool) * bench.CFG4_STRIDE
    ends = starts + bench.CFG4_BATCH_BYTES
    outs = device.sha512_trunc32_ranges(data, starts, ends)
    torch.cuda.synchronize()
    ok, detail = bench.check_cfg4_digests(data, outs, pool, nb, min(16, bench.cpu_threads()))
    assert ok, detail
    assert detail["digests_checked"] == nb and detail["pool_batches_vs_hashlib"] == pool
    # the bench's recipe equals the reference's batch layout (cfg4_host_batch: byte-wise bincode)
    for b in (0, 1, pool - 1):
        row = data[b * bench.CFG4_STRIDE:b * bench.CFG4_STRIDE + bench.CFG4_BATCH_BYTES].cpu().numpy().tobytes()
        assert row == bench.cfg4_host_batch(b), b


def test_cfg4_digest_check_catches_a_wrong_digest():
    """The checker itself: one corrupted digest (inside the pool, then outside it) is reported."""
    import torch
    import bench
    from narwhal_amd import device
    pool, nb = 64, 200
    data = bench.make_cfg4_pool(pool)
    starts = (torch.arange(nb, dtype=torch.int64, device="cuda") % pool) * bench.CFG4_STRIDE
    outs = device.sha512_trunc32_ranges(data, starts, starts + bench.CFG4_BATCH_BYTES)
    torch.cuda.synchronize()
    assert bench.check_cfg4_digests(data, outs, pool, nb, 4)[0]
    for i in (5, 150):
        o = outs.clone()
        o[i, 0] ^= 1
        ok, detail = bench.check_cfg4_digests(data, o, pool, nb, 4)
        assert not ok, (i, detail)
