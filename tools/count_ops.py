#!/usr/bin/env python3
"""Counts the VALU instructions of one fe_mul, one fe_sq and one sha512_compress in this
build's gfx950 ISA, and writes tools/op_counts.json (used by bench.py's work model).

Method: probe kernels load their operands from memory, run exactly one operation, store the
result; a baseline kernel does the same loads/stores with the operation replaced by a copy.
count(op) = VALU(op kernel) - VALU(baseline kernel).
"""
import json
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PROBE = r'''
#include "fe25519.h"
#include "sha512.h"
using namespace nwc;
__device__ __forceinline__ fe ld(const int* p) { fe r; for (int i = 0; i < 10; ++i) r.v[i] = p[i * 64 + threadIdx.x]; return r; }
__device__ __forceinline__ void st(int* p, const fe& a) { for (int i = 0; i < 10; ++i) p[i * 64 + threadIdx.x] = a.v[i]; }
extern "C" __global__ void probe_base2(const int* a, const int* b, int* o) { fe x = ld(a), y = ld(b); st(o, fe_add(x, y)); }
extern "C" __global__ void probe_mul(const int* a, const int* b, int* o) { st(o, fe_mul(ld(a), ld(b))); }
extern "C" __global__ void probe_base1(const int* a, int* o) { st(o, ld(a)); }
extern "C" __global__ void probe_sq(const int* a, int* o) { st(o, fe_sq(ld(a))); }
extern "C" __global__ void probe_shabase(const uint64_t* w, uint64_t* o) {
  uint64_t s[8], x[16];
  for (int i = 0; i < 8; ++i) s[i] = w[i * 64 + threadIdx.x];
  for (int i = 0; i < 16; ++i) x[i] = w[(8 + i) * 64 + threadIdx.x];
  for (int i = 0; i < 8; ++i) o[i * 64 + threadIdx.x] = s[i] ^ x[i] ^ x[i + 8];
}
extern "C" __global__ void probe_sha(const uint64_t* w, uint64_t* o) {
  uint64_t s[8], x[16];
  for (int i = 0; i < 8; ++i) s[i] = w[i * 64 + threadIdx.x];
  for (int i = 0; i < 16; ++i) x[i] = w[(8 + i) * 64 + threadIdx.x];
  sha512_compress(s, x);
  for (int i = 0; i < 8; ++i) o[i * 64 + threadIdx.x] = s[i];
}
'''


def valu_counts(asm: str):
    out = {}
    for m in re.finditer(r"^(probe_\w+):[^\n]*\n(.*?)^\s*s_endpgm", asm, re.S | re.M):
        body = m.group(2)
        out[m.group(1)] = sum(1 for l in body.splitlines() if re.match(r"\s+v_", l))
    return out


def main():
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "probe.hip")
        open(src, "w").write(PROBE)
        asm = os.path.join(td, "probe.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "narwhal_amd", "csrc"), "-o", asm, src], check=True)
        c = valu_counts(open(asm).read())
    res = {"fe_mul": c["probe_mul"] - c["probe_base2"], "fe_sq": c["probe_sq"] - c["probe_base1"],
           "sha512_block": c["probe_sha"] - c["probe_shabase"], "raw": c,
           "method": "VALU instructions (lane-ops per lane) of one op minus a load/store baseline; tools/count_ops.py"}
    with open(os.path.join(HERE, "op_counts.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
