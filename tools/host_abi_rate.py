#!/usr/bin/env python3
"""Host-ABI throughput of nwc_verify_strict_many on config-2-sized inputs in host memory (the
PCIe-inclusive rate DESIGN.md §5 reports beside the device-resident headline).

    python tools/host_abi_rate.py [--n 1048576] [--reps 5]   -> one JSON line
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    from narwhal_amd import _lib, device
    lib = _lib.load()
    n = args.n
    msgs = device.derive32(b"abi-msg", 0, n)
    pks, sigs = device.keygen_sign(device.derive32(b"abi-seed", 0, n), msgs)
    torch.cuda.synchronize()
    m, p, s = (np.ascontiguousarray(t.cpu().numpy()) for t in (msgs, pks, sigs))
    out = ctypes.create_string_buffer((n + 7) // 8)
    vp = ctypes.c_void_p
    call = lambda: lib.nwc_verify_strict_many(m.ctypes.data_as(vp), p.ctypes.data_as(vp), s.ctypes.data_as(vp),
                                              ctypes.c_size_t(n), out)
    _lib.check(call())   # warm-up (scratch, staging)
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        _lib.check(call())
        times.append(time.perf_counter() - t0)
    ok = np.unpackbits(np.frombuffer(out.raw, np.uint8), bitorder="little")[:n].all()
    best, med = min(times), sorted(times)[len(times) // 2]
    print(json.dumps({"metric": "host-ABI verify_strict_many (pageable host buffers, PCIe + kernel)", "n": n,
                      "verifies_per_s_median": n / med, "verifies_per_s_best": n / best, "ms_median": med * 1e3,
                      "all_valid": bool(ok), "reps": args.reps}))


if __name__ == "__main__":
    main()
