"""Device-resident entry points over torch tensors (HBM buffers + torch's current stream).

torch is plumbing here (allocation, streams, events, torch.distributed); all compute is in the
libnwc.so kernels reached through `nwc_dev_*` (include/nwc.h).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _lib


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "expected a contiguous device tensor"
    return ctypes.c_void_p(t.data_ptr())


def words_for(n: int) -> int:
    return (n + 63) // 64


def verify(msgs: torch.Tensor, pks: torch.Tensor, sigs: torch.Tensor, strict: bool = True,
           msg_index: Optional[torch.Tensor] = None, msg_stride: int = 1,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Verification equations on HBM-resident uint8 tensors msgs[*,32], pks[n,32], sigs[n,64].
    Returns int64 verdict words (bit i = equation i valid). Asynchronous on the current stream."""
    lib = _lib.load()
    n = pks.shape[0]
    assert pks.dtype == torch.uint8 and sigs.dtype == torch.uint8 and msgs.dtype == torch.uint8
    assert pks.numel() == 32 * n and sigs.numel() == 64 * n
    if msg_index is not None:
        assert msg_index.dtype == torch.int32 and msg_index.numel() == n
    elif msg_stride:
        assert msgs.numel() >= 32 * n
    if out is None:
        out = torch.empty(words_for(n), dtype=torch.int64, device=pks.device)
    _lib.check(lib.nwc_dev_verify(_ptr(msgs), _ptr(msg_index), msg_stride, _ptr(pks), _ptr(sigs), n,
                                  1 if strict else 0, _ptr(out), _stream()))
    return out


def verify_clock(msgs: torch.Tensor, pks: torch.Tensor, sigs: torch.Tensor, out: torch.Tensor) -> Tuple[float, int]:
    """nwc_diag_verify_clock: one stamped launch of the strict kernel over these inputs; returns the
    median in-kernel shader clock (GHz) over waves and the number of waves. Synchronises."""
    lib = _lib.load()
    n = pks.shape[0]
    ghz = ctypes.c_double()
    waves = ctypes.c_uint32()
    _lib.check(lib.nwc_diag_verify_clock(_ptr(msgs), 1, _ptr(pks), _ptr(sigs), n, _ptr(out), _stream(),
                                         ctypes.byref(ghz), ctypes.byref(waves)))
    return ghz.value, waves.value


def verify_batch_straus(digests: torch.Tensor, offsets: torch.Tensor, msg_index: torch.Tensor, pks: torch.Tensor,
                        sigs: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dalek's batch equation over sub-batches of ~12 votes (Straus per lane), the exact leaves for
    the sub-batches it rejects: returns leaf-style verdict words (bit per vote) for cert_reduce.
    Asynchronous."""
    lib = _lib.load()
    m = offsets.numel() - 1
    n = pks.shape[0]
    assert offsets.dtype == torch.int32 and msg_index.dtype == torch.int32 and msg_index.numel() == n
    if out is None:
        out = torch.empty(words_for(n), dtype=torch.int64, device=pks.device)
    _lib.check(lib.nwc_dev_verify_batch_straus(_ptr(digests), _ptr(offsets), _ptr(msg_index), m, n, _ptr(pks),
                                               _ptr(sigs), _ptr(out), _stream()))
    return out


def verify_batch_msm(digests: torch.Tensor, offsets: torch.Tensor, msg_index: torch.Tensor, pks: torch.Tensor,
                     sigs: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dalek's batch equation as a Pippenger MSM per group of consecutive votes (one wave per group,
    wavefront-level bucket reduction), the exact leaves for the groups it rejects: leaf-style
    verdict words (bit per vote) for cert_reduce.  Asynchronous."""
    lib = _lib.load()
    m = offsets.numel() - 1
    n = pks.shape[0]
    assert offsets.dtype == torch.int32 and msg_index.dtype == torch.int32 and msg_index.numel() == n
    if out is None:
        out = torch.empty(words_for(n), dtype=torch.int64, device=pks.device)
    _lib.check(lib.nwc_dev_verify_batch_msm(_ptr(digests), _ptr(offsets), _ptr(msg_index), m, n, _ptr(pks),
                                            _ptr(sigs), _ptr(out), _stream()))
    return out


def msm_stats():
    """nwc_msm_stats: (groups passed, groups failed, key overflows, groups skipped) of the MSM entry
    so far."""
    lib = _lib.load()
    v = [ctypes.c_uint64() for _ in range(4)]
    _lib.check(lib.nwc_msm_stats(*(ctypes.byref(x) for x in v)))
    return tuple(x.value for x in v)


def cert_reduce(leaf_words: torch.Tensor, offsets: torch.Tensor, nvotes: int,
                want_bad: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    lib = _lib.load()
    m = offsets.numel() - 1
    assert offsets.dtype == torch.int32
    cert = torch.empty(words_for(m), dtype=torch.int64, device=leaf_words.device)
    bad = torch.empty(words_for(nvotes), dtype=torch.int64, device=leaf_words.device) if want_bad else None
    _lib.check(lib.nwc_dev_cert_reduce(_ptr(leaf_words), _ptr(offsets), m, nvotes, _ptr(cert), _ptr(bad), _stream()))
    return cert, bad


def sha512_trunc32(data: torch.Tensor, offsets: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Digest32 of messages data[offsets[i]:offsets[i+1]] (offsets int64 device tensor, n+1)."""
    lib = _lib.load()
    n = offsets.numel() - 1
    assert offsets.dtype == torch.int64 and data.dtype == torch.uint8
    if out is None:
        out = torch.empty((n, 32), dtype=torch.uint8, device=data.device)
    _lib.check(lib.nwc_dev_sha512_trunc32(_ptr(data), _ptr(offsets), n, _ptr(out), _stream()))
    return out


def sha512_trunc32_ranges(data: torch.Tensor, starts: torch.Tensor, ends: torch.Tensor,
                          out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Digest32 of messages data[starts[i]:ends[i]] (int64 device tensors)."""
    lib = _lib.load()
    n = starts.numel()
    assert starts.dtype == torch.int64 and ends.dtype == torch.int64 and ends.numel() == n
    if out is None:
        out = torch.empty((n, 32), dtype=torch.uint8, device=data.device)
    _lib.check(lib.nwc_dev_sha512_trunc32_ranges(_ptr(data), _ptr(starts), _ptr(ends), n, _ptr(out), _stream()))
    return out


def derive32(tag: bytes, first: int, n: int, device="cuda") -> torch.Tensor:
    """out_i = SHA-512(tag || u64le(first + i))[..32] (SURVEY.md §8(d) seed scheme)."""
    lib = _lib.load()
    out = torch.empty((n, 32), dtype=torch.uint8, device=device)
    _lib.check(lib.nwc_dev_derive32(tag, len(tag), first, n, _ptr(out), _stream()))
    return out


def keygen_sign(seeds: torch.Tensor, msgs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    lib = _lib.load()
    n = seeds.shape[0]
    pks = torch.empty((n, 32), dtype=torch.uint8, device=seeds.device)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=seeds.device)
    _lib.check(lib.nwc_dev_keygen_sign(_ptr(seeds), _ptr(msgs), n, _ptr(pks), _ptr(sigs), _stream()))
    return pks, sigs


def keygen_sign_host(seeds: bytes, msgs: bytes, n: int) -> Tuple[bytes, bytes]:
    dev = torch.device("cuda", torch.cuda.current_device())
    s = torch.frombuffer(bytearray(seeds), dtype=torch.uint8).reshape(n, 32).to(dev)
    m = torch.frombuffer(bytearray(msgs), dtype=torch.uint8).reshape(n, 32).to(dev)
    pks, sigs = keygen_sign(s, m)
    torch.cuda.current_stream().synchronize()
    return bytes(pks.cpu().numpy().tobytes()), bytes(sigs.cpu().numpy().tobytes())


def unpack_bits(words: torch.Tensor, n: int):
    """Verdict words -> numpy bool array of length n (host)."""
    import numpy as np
    w = words.detach().cpu().numpy().view(np.uint8)
    return np.unpackbits(w, bitorder="little")[:n].astype(bool)
