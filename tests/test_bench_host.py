"""Host-side pieces of bench.py that the GPU legs' parity checks rely on (no GPU)."""
import hashlib

import numpy as np


def test_cfg4_pool_host_matches_the_bytewise_recipe():
    """The numpy pool construction (what the full-size digest check compares HBM against) equals the
    byte-wise bincode WorkerMessage::Batch of cfg4_host_batch (worker/src/batch_maker.rs:119,
    node/src/benchmark_client.rs:117-130) for first, middle and large batch indices."""
    import bench
    for b0, b1 in ((0, 3), (1000, 1002), (16382, 16384)):
        rows = bench.cfg4_pool_host(b0, b1)
        assert rows.shape == (b1 - b0, bench.CFG4_STRIDE)
        for k, b in enumerate(range(b0, b1)):
            want = bench.cfg4_host_batch(b)
            assert len(want) == bench.CFG4_BATCH_BYTES == 508_052
            assert rows[k, :bench.CFG4_BATCH_BYTES].tobytes() == want, b
            assert not rows[k, bench.CFG4_BATCH_BYTES:].any()
    # the reference fixture's digest recipe on one batch: SHA-512[..32]
    d = hashlib.sha512(bench.cfg4_pool_host(7, 8)[0, :bench.CFG4_BATCH_BYTES]).digest()[:32]
    assert d == hashlib.sha512(bench.cfg4_host_batch(7)).digest()[:32]


def test_cert_shards_balance_votes_and_keep_certificates_whole():
    """bench's config-3 sharding at world > 1: whole certificates per rank, balanced by votes."""
    import bench
    offs = np.concatenate([[0], np.cumsum(np.random.default_rng(3).integers(0, 90, 1001))]).astype(np.int64)
    for world in (1, 2, 3, 8):
        spans = [bench.cert_shard(offs, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == len(offs) - 1
        assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
        votes = [int(offs[c1] - offs[c0]) for c0, c1 in spans]
        assert sum(votes) == int(offs[-1])
        assert max(votes) - min(votes) <= 2 * 90, votes
