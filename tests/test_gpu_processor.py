"""The worker's Processor over the GPU batch digester (narwhal_amd/processor.py, nwc_digester_*):
grouped digests against hashlib (the reference's Sha512::digest(&batch)[..32],
worker/src/processor.rs:38), submission order and tags, grouping by max_group / max_wait_us, and
the Processor's store writes and WorkerPrimaryMessage bytes on the reference's own batch fixture."""
import hashlib
import json
import os
import queue
import struct
import time

import numpy as np
import pytest

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _sha32(b) -> bytes:
    return hashlib.sha512(bytes(b)).digest()[:32]


def test_digester_groups_vs_hashlib():
    from narwhal_amd.processor import Digester
    rng = np.random.default_rng(5)
    lens = [0, 1, 111, 112, 127, 128, 129, 239, 240, 255, 256] + [int(x) for x in rng.integers(0, 600_000, 60)]
    batches = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    for max_group, wait in ((1, 0), (7, 0), (64, 200_000), (4096, 1000)):
        dg = Digester(max_group, wait)
        try:
            tags = [dg.submit(b, 1000 + i) for i, b in enumerate(batches)]
            got = []
            t0 = time.time()
            while len(got) < len(batches) and time.time() - t0 < 60:
                got += dg.poll(4096, 100_000)
            assert [t for t, _ in got] == tags            # submission order, caller's tags
            for (t, d), b in zip(got, batches):
                assert d == _sha32(b), (max_group, t, len(b))
            groups, nb, nbytes = dg.stats()
            assert nb == len(batches) and nbytes == sum(lens)
            if max_group == 1:
                assert groups == len(batches)
            if max_group == 7:
                assert groups >= (len(batches) + 6) // 7
        finally:
            dg.close()


def test_digester_max_wait_gathers_a_burst():
    """Everything submitted within max_wait of the first batch goes out in one launch."""
    from narwhal_amd.processor import Digester
    rng = np.random.default_rng(6)
    batches = [rng.integers(0, 256, 5000, dtype=np.uint8).tobytes() for _ in range(50)]
    dg = Digester(1024, 500_000)
    try:
        for b in batches:
            dg.submit(b)
        got = []
        while len(got) < 50:
            got += dg.poll(64, 1_000_000)
        assert [d for _, d in got] == [_sha32(b) for b in batches]
        assert dg.stats()[0] == 1
    finally:
        dg.close()


def test_processor_reference_batch():
    """Processor::spawn over the reference worker fixture (worker/src/tests/common.rs:87-109): the
    digest, the store write under it, and bincode(WorkerPrimaryMessage::OurBatch(digest, id))."""
    from narwhal_amd.processor import Processor, worker_primary_message
    g = json.load(open(os.path.join(GOLDEN, "sha512.json")))
    ref = [c for c in g["small"] if c.get("name") == "reference-serialized_batch"]
    assert ref, "golden fixture missing"
    batch = bytes.fromhex(ref[0]["msg"])
    want = bytes.fromhex(ref[0]["digest32"])
    assert _sha32(batch) == want

    class Store(dict):
        def write(self, k, v):
            self[k] = v

    rng = np.random.default_rng(7)
    others = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 100_000, 40)]
    for own in (True, False):
        store, rx, tx = Store(), queue.Queue(), queue.Queue()
        p = Processor.spawn(3, store, rx, tx, own, max_group=16, max_wait_us=2000)
        for b in [batch] + others:
            rx.put(b)
        rx.put(None)
        p.join(60)
        msgs = [tx.get_nowait() for _ in range(len(others) + 1)]
        assert tx.empty()
        assert msgs[0] == struct.pack("<I", 0 if own else 1) + want + struct.pack("<I", 3)
        assert msgs[1:] == [worker_primary_message(_sha32(b), 3, own) for b in others]
        assert store[want] == batch and len(store) == len({_sha32(b) for b in [batch] + others})


@pytest.mark.parametrize("stages,threads", [("2", "1"), ("4", "8"), ("8", "3")])
def test_digester_stage_rotation(stages, threads):
    """A 200-MB group through the pinned stages (32 MB each) in rotation: batches straddle stage
    boundaries and every stage is refilled several times (NWC_DIGEST_STAGES / _COPY_THREADS are
    read when the digester is created)."""
    from narwhal_amd.processor import Digester
    rng = np.random.default_rng(8)
    base = rng.integers(0, 256, 600_000, dtype=np.uint8).tobytes()
    lens = [int(x) for x in rng.integers(300_000, 600_000, 400)]
    offs = [int(x) for x in rng.integers(0, 600_000 - 300_000, 400)]
    batches = [base[o:o + n] for o, n in zip(offs, lens)]
    os.environ["NWC_DIGEST_STAGES"], os.environ["NWC_DIGEST_COPY_THREADS"] = stages, threads
    try:
        dg = Digester(4096, 2_000_000)
    finally:
        del os.environ["NWC_DIGEST_STAGES"], os.environ["NWC_DIGEST_COPY_THREADS"]
    try:
        for b in batches:
            dg.submit(b)
        got = []
        t0 = time.time()
        while len(got) < len(batches) and time.time() - t0 < 60:
            got += dg.poll(4096, 1_000_000)
        assert [d for _, d in got] == [_sha32(b) for b in batches]
        assert dg.stats()[0] == 1
    finally:
        dg.close()


def test_digester_receive_arena():
    """nwc_digester_arena: batches written into the pinned arena are DMA'd into the arena's device
    mirror at their arena offsets while the group is collected (runs of adjacent batches; a gap,
    odd spacing or submission out of arena order only starts a new run), and the kernel reads them
    there; a group holding one batch from outside the arena takes the stage path.  Digests equal
    hashlib either way, in submission order."""
    from narwhal_amd.processor import Digester
    rng = np.random.default_rng(9)
    lens = [0, 1, 15, 16, 17, 127, 128, 129, 4096, 0, 333] + [int(x) for x in rng.integers(0, 400_000, 40)]
    r16 = lambda n: (n + 15) & ~15  # noqa: E731
    size = sum(r16(n) for n in lens) + (8 << 20)
    dg = Digester(4096, 2_000_000)
    try:
        arena = dg.arena(size)
        assert dg.arena(size // 2) is not None        # same arena again when it fits

        def place(gap_at=None):
            views, off = [], 0
            for i, n in enumerate(lens):
                if i == gap_at:
                    off += 3 << 20                    # a ring wrap / hole: starts a new run
                v = arena[off:off + n]
                v[:] = rng.integers(0, 256, n, dtype=np.uint8)
                views.append(v)
                off += r16(n)
            return views

        def run(views, extra=None):
            items = list(views) + ([extra] if extra is not None else [])
            want = [_sha32(v) for v in items]
            tags = [dg.submit(v) for v in items]
            got = []
            t0 = time.time()
            while len(got) < len(items) and time.time() - t0 < 60:
                got += dg.poll(4096, 200_000)
            assert [t for t, _ in got] == tags
            assert [d for _, d in got] == want

        run(place())
        d1 = dg.direct_groups()
        assert d1 >= 1
        run(place(gap_at=20))
        d2 = dg.direct_groups()
        assert d2 > d1
        run(place(), extra=rng.integers(0, 256, 1000, dtype=np.uint8).tobytes())   # one batch outside
        assert dg.direct_groups() == d2
        # random spacing: batches packed at the 16-rounded stride, shifted by odd byte counts, or
        # placed out of order -- every break starts a run; still direct, digests unchanged
        views, off = [], 0
        slots = []
        for n in lens:
            slots.append((off, n))
            off += r16(n) + int(rng.choice([0, 0, 0, 1, 7, 4096]))
        order = rng.permutation(len(slots))
        for i in order:
            o, n = slots[i]
            v = arena[o:o + n]
            v[:] = rng.integers(0, 256, n, dtype=np.uint8)
        views = [arena[o:o + n] for o, n in (slots[i] for i in order)]
        run(views)
        assert dg.direct_groups() == d2 + 1
    finally:
        dg.close()
