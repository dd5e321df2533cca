"""Loader for the in-tree HIP library `narwhal_amd/libnwc.so` (C ABI: include/nwc.h).

There is no fallback: if the library is missing or no gfx950 device is visible, calls raise.
torch (when installed) is imported first so that the process has exactly one HIP runtime:
torch's bundled libamdhip64 carries the SONAME libamdhip64.so.7 that libnwc.so needs, and
glibc reuses an already-loaded object by SONAME, while the reverse order would load a second
runtime next to torch's.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# NWC_LIB_PATH: an alternative in-tree build of the same library (A/B experiments)
LIB_PATH = os.environ.get("NWC_LIB_PATH") or os.path.join(HERE, "libnwc.so")

NWC_OK = 0
NWC_INVALID = 1
NWC_ERR_DEVICE = -1
NWC_ERR_ARG = -2
NWC_ERR_NOT_INIT = -3
NWC_ERR_NO_DEVICE = -4

_c_u8p = ctypes.c_void_p
_SIGS = {
    "nwc_init": (ctypes.c_int, [ctypes.c_uint32]),
    "nwc_shutdown": (None, []),
    "nwc_last_error": (ctypes.c_char_p, []),
    "nwc_version": (ctypes.c_int, []),
    "nwc_device_count": (ctypes.c_int, []),
    "nwc_build_id": (ctypes.c_char_p, []),
    "nwc_memory_info": (ctypes.c_int, [ctypes.c_void_p]),
    "nwc_trim": (ctypes.c_int, []),
    "nwc_diag_set": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64]),
    "nwc_diag_verify_clock": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]),
    "nwc_verify_strict": (ctypes.c_int, [_c_u8p, _c_u8p, _c_u8p]),
    "nwc_verify_batch": (ctypes.c_int, [_c_u8p, _c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p]),
    "nwc_verify_strict_many": (ctypes.c_int, [_c_u8p, _c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p]),
    "nwc_verify_batch_many": (ctypes.c_int, [_c_u8p, _c_u8p, _c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p, _c_u8p]),
    "nwc_verify_batch_straus_many": (ctypes.c_int, [_c_u8p, _c_u8p, _c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p, _c_u8p]),
    "nwc_verify_batch_msm_many": (ctypes.c_int, [_c_u8p, _c_u8p, _c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p, _c_u8p]),
    "nwc_dev_verify_batch_msm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p]),
    "nwc_msm_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_set_committee": (ctypes.c_int, [_c_u8p, ctypes.c_size_t]),
    "nwc_cache_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_auto_cache_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_launch_keys_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_digest32": (ctypes.c_int, [_c_u8p, ctypes.c_size_t, _c_u8p]),
    "nwc_sha512_trunc32_many": (ctypes.c_int, [_c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p]),
    "nwc_dev_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "nwc_dev_cert_reduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_dev_verify_batch_straus": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                   ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p]),
    "nwc_dev_sha512_trunc32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    "nwc_dev_sha512_trunc32_ranges": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_dev_derive32": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_dev_keygen_sign": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_dev_set_device": (ctypes.c_int, [ctypes.c_int]),
    "nwc_set_committee_config": (ctypes.c_int, [_c_u8p, _c_u8p, ctypes.c_size_t, _c_u8p, _c_u8p]),
    "nwc_dev_sanitize_messages": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint64, _c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "nwc_sanitize_messages": (ctypes.c_int, [_c_u8p, _c_u8p, ctypes.c_size_t, ctypes.c_uint64, _c_u8p, _c_u8p,
                                             _c_u8p, _c_u8p]),
    "nwc_digester_create": (ctypes.c_void_p, [ctypes.c_uint32, ctypes.c_uint32]),
    "nwc_digester_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]),
    "nwc_digester_poll": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]),
    "nwc_digester_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_digester_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "nwc_digester_arena": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_size_t]),
    "nwc_digester_direct_groups": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "nwc_shard_bounds": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "nwc_cert_cuts": (ctypes.c_int, [_c_u8p, ctypes.c_size_t, ctypes.c_uint32, _c_u8p]),
}

_lib = None
_lock = threading.Lock()


class DeviceError(RuntimeError):
    """A runtime/device/argument failure of libnwc (never an 'invalid signature')."""


class Memory(ctypes.Structure):
    """nwc_memory (include/nwc.h): device bytes this process holds on one device."""
    _fields_ = [(name, ctypes.c_uint64) for name in
                ("tables", "committee", "auto_cache", "scratch", "digesters", "device_free", "device_total")]

    def as_dict(self):
        return {name: int(getattr(self, name)) for name, _ in self._fields_}


def memory_info() -> dict:
    """nwc_memory_info of the calling thread's device."""
    m = Memory()
    check(load().nwc_memory_info(ctypes.byref(m)))
    return m.as_dict()


def diag_set(name: str, value: int) -> None:
    """nwc_diag_set: a test / A-B knob ("straus_nq", "force_windows")."""
    check(load().nwc_diag_set(name.encode(), value))


def load(init: bool = True, device_mask: int = 0):
    """Load libnwc.so (and nwc_init it unless init=False). Raises if unavailable."""
    global _lib
    with _lock:
        if _lib is None:
            try:
                import torch  # noqa: F401  (one HIP runtime per process, see module docstring)
            except ImportError:
                pass
            if not os.path.exists(LIB_PATH):
                raise DeviceError("libnwc.so not built at %s: run `python -c 'import __graft_entry__ as g; g.build()'`"
                                  % LIB_PATH)
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                if os.environ.get("NWC_LIB_PATH") and not hasattr(lib, name):
                    continue   # an A/B build from before this entry point existed
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
        lib = _lib
    if init:
        rc = lib.nwc_init(device_mask)
        if rc < 0:
            raise DeviceError("nwc_init failed (%d): %s" % (rc, lib.nwc_last_error().decode()))
    return lib


def check(rc: int) -> int:
    """Raise DeviceError for rc < 0, else return rc."""
    if rc < 0:
        raise DeviceError("libnwc error %d: %s" % (rc, _lib.nwc_last_error().decode() if _lib else "?"))
    return rc


def buf(b) -> ctypes.c_void_p:
    """Pointer to a bytes-like object (bytes, bytearray, numpy array) without copying when possible."""
    if b is None:
        return None
    try:
        import numpy as np
        if isinstance(b, np.ndarray):
            # the C side reads nbytes contiguous bytes from the first element
            if not b.flags.c_contiguous:
                raise TypeError("non-contiguous array: pass np.ascontiguousarray(a)")
            # data_as keeps a reference to the array: a temporary (buf(x.cpu().numpy())) stays alive
            # for as long as the returned pointer does, i.e. through the call it is passed to
            return b.ctypes.data_as(ctypes.c_void_p)
    except ImportError:
        pass
    if isinstance(b, bytes):
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)
    if isinstance(b, bytearray):
        return ctypes.c_void_p(ctypes.addressof((ctypes.c_char * len(b)).from_buffer(b))) if len(b) else None
    raise TypeError("unsupported buffer type %r" % type(b))
