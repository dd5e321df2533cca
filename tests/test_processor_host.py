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
