#!/usr/bin/env python3
"""VALU instructions of one fe32 multiply / square / add / sub (tools/microbench/fe32.h) next to
the kernels' fe_mul / fe_sq / fe_add / fe_sub (narwhal_amd/csrc/fe25519.h), counted in the gfx950
ISA the way tools/count_ops.py counts: a probe kernel loads its operands, runs exactly one
operation and stores the result; a baseline kernel does the same loads and stores around a copy.
Prints JSON (instruction totals and the VOP3 / VOP2 / VOP1 split of each op)."""
import json
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PROBE = r'''
#include "fe25519.h"
#include "fe32.h"
using namespace nwc;
using fe32x::fe32;
__device__ __forceinline__ fe ld(const int* p) { fe r; for (int i = 0; i < 10; ++i) r.v[i] = p[i * 64 + threadIdx.x]; return r; }
__device__ __forceinline__ void st(int* p, const fe& a) { for (int i = 0; i < 10; ++i) p[i * 64 + threadIdx.x] = a.v[i]; }
__device__ __forceinline__ fe32 ld32(const unsigned* p) { fe32 r; for (int i = 0; i < 8; ++i) r.v[i] = p[i * 64 + threadIdx.x]; return r; }
__device__ __forceinline__ void st32(unsigned* p, const fe32& a) { for (int i = 0; i < 8; ++i) p[i * 64 + threadIdx.x] = a.v[i]; }
extern "C" __global__ void probe_base2(const int* a, const int* b, int* o) { fe x = ld(a), y = ld(b); fe r; for (int i = 0; i < 10; ++i) r.v[i] = x.v[i] ^ y.v[i]; st(o, r); }
extern "C" __global__ void probe_base1(const int* a, int* o) { st(o, ld(a)); }
extern "C" __global__ void probe_base2s(const int* a, const int* b, int* o) { st(o, ld(a)); st(o + 640, ld(b)); }
extern "C" __global__ void probe_mul(const int* a, const int* b, int* o) { st(o, fe_mul(ld(a), ld(b))); }
extern "C" __global__ void probe_sq(const int* a, int* o) { st(o, fe_sq(ld(a))); }
extern "C" __global__ void probe_add(const int* a, const int* b, int* o) { st(o, fe_add(ld(a), ld(b))); }
extern "C" __global__ void probe_sub(const int* a, const int* b, int* o) { st(o, fe_sub(ld(a), ld(b))); }
extern "C" __global__ void probe32_base2(const unsigned* a, const unsigned* b, unsigned* o) { fe32 x = ld32(a), y = ld32(b); fe32 r; for (int i = 0; i < 8; ++i) r.v[i] = x.v[i] ^ y.v[i]; st32(o, r); }
extern "C" __global__ void probe32_base1(const unsigned* a, unsigned* o) { st32(o, ld32(a)); }
extern "C" __global__ void probe32_base2s(const unsigned* a, const unsigned* b, unsigned* o) { st32(o, ld32(a)); st32(o + 512, ld32(b)); }
extern "C" __global__ void probe32_mul(const unsigned* a, const unsigned* b, unsigned* o) { st32(o, fe32x::fe32_mul(ld32(a), ld32(b))); }
extern "C" __global__ void probe32_sq(const unsigned* a, unsigned* o) { st32(o, fe32x::fe32_sq(ld32(a))); }
extern "C" __global__ void probe32_add(const unsigned* a, const unsigned* b, unsigned* o) { st32(o, fe32x::fe32_add(ld32(a), ld32(b))); }
extern "C" __global__ void probe32_sub(const unsigned* a, const unsigned* b, unsigned* o) { st32(o, fe32x::fe32_sub(ld32(a), ld32(b))); }
'''
VOP3_ONLY = ("v_mad_", "v_mul_hi", "v_mul_lo", "v_alignbit", "v_lshl_add_u64", "v_bitop3", "v_add3", "v_perm",
             "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64", "v_bfe", "v_bfi", "v_lshl_or", "v_and_or",
             "v_or3", "v_xad", "v_cndmask_b32_e64", "v_add_co_u32_e64", "v_addc_co_u32_e64", "v_sub_co_u32_e64",
             "v_subb_co_u32_e64", "v_subrev_co_u32_e64", "v_subbrev_co_u32_e64")


def census(asm: str):
    out = {}
    for m in re.finditer(r"^(probe\w*):[^\n]*\n(.*?)^\s*s_endpgm", asm, re.S | re.M):
        ins = [l.split()[0] for l in m.group(2).splitlines() if re.match(r"\s+v_", l)]
        vop3 = sum(1 for i in ins if i.startswith(VOP3_ONLY) or i.endswith("_e64"))
        out[m.group(1)] = {"valu": len(ins), "vop3": vop3, "mad": sum(1 for i in ins if i.startswith("v_mad_"))}
    return out


def main():
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "probe.hip")
        open(src, "w").write(PROBE)
        asm = os.path.join(td, "probe.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "narwhal_amd", "csrc"), "-I" + HERE, "-o", asm, src], check=True)
        text = open(asm).read()
        c = census(text)
    res = {}
    # add / sub against a baseline that stores both operands (the XOR baseline costs as much as an add)
    for name, base in (("mul", "base2"), ("sq", "base1"), ("add", "base2s"), ("sub", "base2s")):
        for pre, label in (("probe_", "fe10_"), ("probe32_", "fe32_")):
            op, b = c[pre + name], c[pre + base]
            res[label + name] = {k: op[k] - b[k] for k in op}
    res["method"] = ("VALU instructions of one op minus a load/store baseline in the gfx950 ISA "
                     "(tools/microbench/fe32_count.py); vop3 = VOP3-encoded (4-cycle wave64 issue), the rest VOP1/VOP2")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
