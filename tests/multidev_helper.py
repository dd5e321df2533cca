"""Subprocess body of tests/test_gpu_multidev.py: runs the host entry points with
NWC_VIRTUAL_DEVICES contexts on one GPU and writes their outputs (the parent compares them with
the oracle).  libnwc reads the variable once, in nwc_init, so it runs in its own process."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, sys.argv[3])
from narwhal_amd import _lib, device  # noqa: E402

lib = _lib.load()
d = dict(np.load(sys.argv[1]))
out = {"devices": np.array([lib.nwc_device_count()])}
m, p, s = d["m"], d["p"], d["s"]
n = p.shape[0]
bits = ctypes.create_string_buffer((n + 7) // 8)
_lib.check(lib.nwc_verify_strict_many(_lib.buf(m), _lib.buf(p), _lib.buf(s), n, bits))
out["strict"] = np.frombuffer(bits.raw, np.uint8).copy()
offs, dig = d["offs"], d["dig"]
mc = len(offs) - 1
cert = ctypes.create_string_buffer((mc + 7) // 8)
bad = ctypes.create_string_buffer((int(offs[-1]) + 7) // 8)
_lib.check(lib.nwc_verify_batch_many(_lib.buf(dig), _lib.buf(offs), _lib.buf(p), _lib.buf(s), mc, cert, bad))
out["cert"] = np.frombuffer(cert.raw, np.uint8).copy()
out["bad"] = np.frombuffer(bad.raw, np.uint8).copy()
cert2 = ctypes.create_string_buffer((mc + 7) // 8)
bad2 = ctypes.create_string_buffer((int(offs[-1]) + 7) // 8)
_lib.check(lib.nwc_verify_batch_straus_many(_lib.buf(dig), _lib.buf(offs), _lib.buf(p), _lib.buf(s), mc, cert2, bad2))
out["cert_straus"] = np.frombuffer(cert2.raw, np.uint8).copy()
out["bad_straus"] = np.frombuffer(bad2.raw, np.uint8).copy()
cert3 = ctypes.create_string_buffer((mc + 7) // 8)
bad3 = ctypes.create_string_buffer((int(offs[-1]) + 7) // 8)
_lib.check(lib.nwc_verify_batch_msm_many(_lib.buf(dig), _lib.buf(offs), _lib.buf(p), _lib.buf(s), mc, cert3, bad3))
out["cert_msm"] = np.frombuffer(cert3.raw, np.uint8).copy()
out["bad_msm"] = np.frombuffer(bad3.raw, np.uint8).copy()
blob, boffs = d["blob"], d["boffs"]
nb = len(boffs) - 1
o32 = np.zeros((nb, 32), np.uint8)
_lib.check(lib.nwc_sha512_trunc32_many(_lib.buf(blob), _lib.buf(boffs), nb, _lib.buf(o32)))
out["digests"] = o32
np.savez(sys.argv[2], **out)
