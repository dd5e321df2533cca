"""The worker's `Processor` (worker/src/processor.rs:20-56) over the GPU batch digester.

The reference task loops `while let Some(batch) = rx_batch.recv().await`, hashes each batch with
`Sha512::digest(&batch)[..32]` (:38), stores it under its digest (:41) and sends the bincode of
`WorkerPrimaryMessage::OurBatch(digest, id)` / `OthersBatch(digest, id)` to the primary (:44-53).
Here the loop hands every batch to a libnwc digester (`nwc_digester_*`, include/nwc.h), whose drain
thread digests whatever has queued up -- up to `max_group` batches, or what arrived within
`max_wait_us` of the first -- in one GPU launch; a collector thread then stores each batch and
sends its message, in arrival order, exactly as the reference does per batch.

There is no CPU path inside: one 500-KB batch alone costs ~30 ms on the GPU (a sequential SHA-512
chain on one lane) against ~0.36 ms on one host core, so this Processor is for workers that can
hand batches over in groups (INTEGRATION.md §4 has the measured crossover); a worker sealing one
batch at a time on a latency-critical path keeps `Sha512::digest`.

Channels are `queue.Queue`s (tokio mpsc's role); `None` on rx_batch closes it (the reference's
`recv()` returning `None`).  `store` is anything with `write(key: bytes, value: bytes)`.
"""
from __future__ import annotations

import ctypes
import queue
import struct
import threading
from typing import Dict, List, Optional, Tuple

from narwhal_amd import _lib

OUR_BATCH, OTHERS_BATCH = 0, 1   # WorkerPrimaryMessage variants (primary/src/primary.rs)


def worker_primary_message(digest: bytes, worker_id: int, own_digest: bool) -> bytes:
    """bincode::serialize(&WorkerPrimaryMessage::{Our,Others}Batch(digest, id)): u32 variant,
    the 32 digest bytes, the u32 WorkerId (processor.rs:44-50)."""
    return struct.pack("<I", OUR_BATCH if own_digest else OTHERS_BATCH) + digest + struct.pack("<I", worker_id)


class DigestGroupError(_lib.DeviceError):
    """A group of batches failed on the device (nwc_digester_poll < 0): `tags` are the batches it
    held, handed back so the caller can release or retry them."""

    def __init__(self, msg: str, tags: List[int]):
        super().__init__(msg)
        self.tags = tags


class Digester:
    """ctypes handle of one `nwc_digester` (its drain thread runs inside libnwc).  Keeps every
    submitted batch alive until its digest has been polled (the C side borrows it)."""

    def __init__(self, max_group: int = 1024, max_wait_us: int = 1000):
        self.lib = _lib.load()
        h = self.lib.nwc_digester_create(max_group, max_wait_us)
        if not h:
            raise _lib.DeviceError(self.lib.nwc_last_error().decode())
        self.h = ctypes.c_void_p(h)
        self._held: Dict[int, object] = {}
        self._next = 0
        self._lock = threading.Lock()

    def submit(self, batch, tag: Optional[int] = None) -> int:
        """Queue one batch (bytes, bytearray or a C-contiguous uint8 numpy array); returns its tag
        (a sequence number unless given).  The batch is held until its digest has been polled."""
        buf = _lib.buf(batch)   # TypeError for other types and for non-contiguous arrays
        n = batch.nbytes if hasattr(batch, "nbytes") else len(batch)
        with self._lock:
            if tag is None:
                tag = self._next
            self._next = max(self._next, tag + 1)
            self._held[tag] = (batch, buf)
        rc = self.lib.nwc_digester_submit(self.h, buf, n, tag)
        if rc < 0:
            with self._lock:
                self._held.pop(tag, None)   # not queued: the C side does not borrow it
            _lib.check(rc)
        return tag

    def arena(self, nbytes: int):
        """The digester's pinned receive arena (`nwc_digester_arena`) as a writable uint8 numpy
        array (valid until close()).  Batches written into it back to back, each at the previous
        one's offset + its length rounded up to 16, and submitted as views of it, are DMA'd straight
        into HBM (no stage fill)."""
        import numpy as np
        p = self.lib.nwc_digester_arena(self.h, nbytes)
        if not p:
            raise _lib.DeviceError(self.lib.nwc_last_error().decode())
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))

    def direct_groups(self) -> int:
        n = ctypes.c_uint64()
        _lib.check(self.lib.nwc_digester_direct_groups(self.h, ctypes.byref(n)))
        return n.value

    def poll(self, max_n: int = 4096, wait_us: int = 0) -> List[Tuple[int, bytes]]:
        tags = (ctypes.c_uint64 * max_n)()
        digs = ctypes.create_string_buffer(32 * max_n)
        n = ctypes.c_size_t(0)
        rc = self.lib.nwc_digester_poll(self.h, max_n, wait_us, tags, digs, ctypes.byref(n))
        raw = digs.raw[:32 * n.value]   # one copy: `.raw` copies the whole buffer on every access
        out = [(int(tags[i]), raw[32 * i:32 * i + 32]) for i in range(n.value)]
        with self._lock:
            for t, _ in out:
                self._held.pop(t, None)
        if rc < 0:
            # a failed group's tags (no digests), or the sticky error once nothing is left
            raise DigestGroupError("libnwc error %d: %s" % (rc, self.lib.nwc_last_error().decode()),
                                   [t for t, _ in out])
        return out

    def stats(self) -> Tuple[int, int, int]:
        g, b, by = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self.lib.nwc_digester_stats(self.h, ctypes.byref(g), ctypes.byref(b), ctypes.byref(by)))
        return g.value, b.value, by.value

    def close(self) -> None:
        if self.h:
            rc = self.lib.nwc_digester_destroy(self.h)
            self.h = None
            _lib.check(rc)


class Processor:
    """`Processor::spawn(id, store, rx_batch, tx_digest, own_digest)` (processor.rs:22-34)."""

    def __init__(self, worker_id: int, store, rx_batch: "queue.Queue", tx_digest: "queue.Queue", own_digest: bool,
                 max_group: int = 1024, max_wait_us: int = 1000, digester=None):
        self.id, self.store, self.rx, self.tx, self.own = worker_id, store, rx_batch, tx_digest, own_digest
        # `digester` (submit/poll/close) is for host-logic unit tests only; the Processor itself
        # always digests on the GPU (a missing libnwc raises here)
        self.dg = digester if digester is not None else Digester(max_group, max_wait_us)
        self._pending: Dict[int, bytes] = {}
        self._next_tag = 0
        self._submitted = 0
        self._done = 0
        self._closed = threading.Event()
        self._error: Optional[BaseException] = None
        self._feeder = threading.Thread(target=self._feed, daemon=True)
        self._collector = threading.Thread(target=self._collect, daemon=True)
        self._feeder.start()
        self._collector.start()

    @classmethod
    def spawn(cls, worker_id: int, store, rx_batch, tx_digest, own_digest: bool, **kw) -> "Processor":
        return cls(worker_id, store, rx_batch, tx_digest, own_digest, **kw)

    def _feed(self):
        try:
            while self._error is None:
                batch = self.rx.get()
                if batch is None:   # channel closed
                    break
                tag = self._next_tag
                self._pending[tag] = batch
                try:
                    self.dg.submit(batch, tag)
                except BaseException:
                    self._pending.pop(tag, None)
                    raise
                self._next_tag += 1
                self._submitted += 1   # counted only once the digester holds it
        except BaseException as e:  # noqa: BLE001 (reported by join())
            self._error = self._error or e
        finally:
            self._closed.set()

    def _collect(self):
        try:
            # stops on the feeder's error too: batches it never submitted will not come back
            while self._error is None and not (self._closed.is_set() and self._done == self._submitted):
                for tag, digest in self.dg.poll(4096, 2000):
                    batch = self._pending.pop(tag)
                    self.store.write(digest, batch)                                   # :41
                    self.tx.put(worker_primary_message(digest, self.id, self.own))    # :44-53
                    self._done += 1
        except BaseException as e:  # noqa: BLE001
            self._error = self._error or e

    def join(self, timeout: Optional[float] = None) -> None:
        """Wait until the closed channel's last batch has been stored and sent; frees the digester.
        Raises TimeoutError (and keeps the digester) if the threads are still running after
        `timeout`, and the first error of either thread otherwise."""
        self._feeder.join(timeout)
        self._collector.join(timeout)
        if self._feeder.is_alive() or self._collector.is_alive():
            # never free the digester under a thread that may be inside poll or submit
            raise TimeoutError("Processor still running after %.1f s" % timeout)
        self.dg.close()
        if self._error:
            raise self._error
