import time, hashlib, json, sys
sys.path.insert(0, '.')
import torch
from narwhal_amd import crypto, _lib
_lib.load()
data = bytes((i * 131 + 7) & 255 for i in range(500000))
d = crypto.digest_bytes(data)
assert d.to_vec() == hashlib.sha512(data).digest()[:32]
ts = []
for _ in range(5):
    t0 = time.perf_counter(); crypto.digest_bytes(data); ts.append(time.perf_counter() - t0)
t0 = time.perf_counter(); hashlib.sha512(data).digest(); tc = time.perf_counter() - t0
print(json.dumps({"one_batch_500000B_gpu_ms_median": sorted(ts)[2] * 1e3, "one_core_openssl_ms": tc * 1e3}))
