"""Host logic of the worker Processor mirror (narwhal_amd/processor.py) on the CPU: arrival-order
store writes and WorkerPrimaryMessage bytes (worker/src/processor.rs:35-55, primary/src/primary.rs
WorkerPrimaryMessage), the channel-close semantics, with a stand-in digester that hands digests
back in groups the way the GPU drain thread does.  The GPU digester itself is tested in
tests/test_gpu_processor.py."""
import hashlib
import queue
import struct
import threading

from narwhal_amd.processor import Processor, worker_primary_message


class GroupedDigester:
    """submit/poll/close like narwhal_amd.processor.Digester; releases digests 5 at a time."""

    def __init__(self):
        self.q, self.lock, self.closed = [], threading.Lock(), False

    def submit(self, batch, tag):
        with self.lock:
            self.q.append((tag, hashlib.sha512(bytes(batch)).digest()[:32]))

    def poll(self, max_n=4096, wait_us=0):
        import time
        time.sleep(wait_us / 4e6)
        with self.lock:
            if len(self.q) >= 5 or (self.q and self.closed):
                out, self.q = self.q[:5], self.q[5:]
                return out
        return []

    def close(self):
        self.closed = True


def test_processor_order_and_messages():
    class Store(dict):
        def write(self, k, v):
            self[k] = v

    batches = [bytes([i]) * (100 + i) for i in range(23)]
    for own in (True, False):
        store, rx, tx = Store(), queue.Queue(), queue.Queue()
        dg = GroupedDigester()
        p = Processor(9, store, rx, tx, own, digester=dg)
        for b in batches:
            rx.put(b)
        rx.put(None)
        p._feeder.join(10)
        dg.closed = True
        p.join(10)
        got = [tx.get_nowait() for _ in batches]
        want = [worker_primary_message(hashlib.sha512(b).digest()[:32], 9, own) for b in batches]
        assert got == want and tx.empty()
        assert got[0][:4] == struct.pack("<I", 0 if own else 1) and got[0][-4:] == struct.pack("<I", 9)
        assert all(store[hashlib.sha512(b).digest()[:32]] == b for b in batches)


class Store(dict):
    def write(self, k, v):
        self[k] = v


def test_submit_error_is_raised_by_join():
    """A digester whose submit raises (a bad batch type, a failed C submit): the feeder records
    the error, the collector stops instead of waiting for batches that were never queued, and
    join() raises it (_submitted was counted before submit, so join hung)."""
    class Failing(GroupedDigester):
        def submit(self, batch, tag):
            if tag == 3:
                raise TypeError("unsupported buffer type")
            super().submit(batch, tag)

    dg = Failing()
    p = Processor(1, Store(), queue.Queue(), queue.Queue(), True, digester=dg)
    for i in range(6):
        p.rx.put(bytes([i]) * 10)
    p.rx.put(None)
    try:
        p.join(10)
        raise AssertionError("join() did not raise")
    except TypeError as e:
        assert "unsupported" in str(e)
    assert p._submitted == 3 and 3 not in p._pending


def test_join_timeout_keeps_the_digester():
    """join(timeout) while the collector is still inside poll must not free the digester under
    it (use-after-free in nwc_digester_destroy): it raises TimeoutError instead."""
    class Slow(GroupedDigester):
        def poll(self, max_n=4096, wait_us=0):
            import time
            time.sleep(0.05)
            return []   # never releases anything

        def close(self):
            raise AssertionError("closed while a poller is alive")

    dg = Slow()
    p = Processor(1, Store(), queue.Queue(), queue.Queue(), True, digester=dg)
    p.rx.put(b"x" * 10)
    p.rx.put(None)
    try:
        p.join(0.3)
        raise AssertionError("join() returned")
    except TimeoutError:
        pass
    p._error = RuntimeError("test over")   # let the collector leave


def test_buf_rejects_non_contiguous_arrays():
    """A strided view would be read as nbytes contiguous bytes from its first element -- the
    wrong bytes, silently: the binding refuses it."""
    import numpy as np
    from narwhal_amd import _lib
    a = np.arange(64, dtype=np.uint8)
    assert _lib.buf(a[::2].copy()) is not None
    try:
        _lib.buf(a[::2])
        raise AssertionError("strided view accepted")
    except TypeError:
        pass


def test_buf_keeps_temporary_arrays_alive():
    """buf(x.cpu().numpy()) passes a temporary: the pointer must keep the array alive through the
    call it is an argument of (a raw address would dangle as soon as buf returned)."""
    import ctypes
    import gc
    import numpy as np
    from narwhal_amd import _lib
    p = _lib.buf(np.arange(1 << 20, dtype=np.uint8) + 7)
    gc.collect()
    junk = [np.full(1 << 20, 0xEE, np.uint8) for _ in range(16)]   # would reuse freed memory
    assert ctypes.string_at(p.value, 4) == bytes([7, 8, 9, 10])
    del junk
