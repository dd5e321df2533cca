import ctypes, sys, time
sys.path.insert(0, '.')
import numpy as np
from narwhal_amd import _lib
lib = _lib.load()
n = 300000
z = np.zeros((n, 32), np.uint8); s = np.zeros((n, 64), np.uint8)
out = ctypes.create_string_buffer((n + 7) // 8)
t = time.time(); _lib.check(lib.nwc_verify_strict_many(_lib.buf(z), _lib.buf(z), _lib.buf(s), n, out)); print("host call ok %.3f s" % (time.time() - t), flush=True)
