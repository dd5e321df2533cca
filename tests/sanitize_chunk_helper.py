"""Subprocess helper for tests/test_gpu_messages.py: nwc_sanitize_messages over the messages in an
.npz (wire bytes + offsets, the committee config) in one call, codes and digests written back.
The pipeline's switches (NWC_MSG_CHUNK, NWC_SIGN_DEFER, NWC_STRICT_Y) come from the environment,
which libnwc reads once per process."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, sys.argv[3])
from narwhal_amd import _lib  # noqa: E402

d = np.load(sys.argv[1])
lib = _lib.load()
keys, stakes, woffs, wids = d["keys"], d["stakes"], d["woffs"], d["wids"]
n = keys.shape[0]
_lib.check(lib.nwc_set_committee_config(_lib.buf(np.ascontiguousarray(keys)), (ctypes.c_uint64 * n)(*stakes.tolist()), n,
                                        (ctypes.c_uint32 * (n + 1))(*woffs.tolist()),
                                        (ctypes.c_uint32 * max(1, len(wids)))(*wids.tolist())))
data, offs = np.ascontiguousarray(d["data"]), np.ascontiguousarray(d["offs"])
m = offs.shape[0] - 1
codes = np.zeros(m, np.int32)
dig = np.zeros((m, 32), np.uint8)
kinds = np.zeros(m, np.uint8)
for _ in range(2):   # twice on the same stages and arena
    _lib.check(lib.nwc_sanitize_messages(_lib.buf(data), _lib.buf(offs), m, int(d["gc"]), None, _lib.buf(codes),
                                         _lib.buf(dig), _lib.buf(kinds)))
np.savez(sys.argv[2], codes=codes, dig=dig)
