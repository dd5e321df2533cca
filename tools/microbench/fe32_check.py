#!/usr/bin/env python3
"""Big-integer check of tools/microbench/fe32's subset file (/tmp/fe32_sub.bin): for every pair
(x, y) -- uniform 256-bit values, [p, 2^255), bit 255 set, all-ones, tiny -- the fe32 multiply,
square, add and sub outputs (canonicalised on the GPU) must equal x*y, x^2, x+y, x-y mod p."""
import struct
import sys

P = 2**255 - 19


def main(path="/tmp/fe32_sub.bin"):
    blob = open(path, "rb").read()
    n = struct.unpack_from("<Q", blob)[0]
    off = 8
    xs = blob[off:off + 32 * n]
    ys = blob[off + 32 * n:off + 64 * n]
    outs = blob[off + 64 * n:off + 64 * n + 128 * n]
    bad = 0
    high = 0
    for i in range(n):
        x = int.from_bytes(xs[32 * i:32 * i + 32], "little")
        y = int.from_bytes(ys[32 * i:32 * i + 32], "little")
        high += (x >> 255) | (y >> 255)
        want = ((x * y) % P, (x * x) % P, (x + y) % P, (x - y) % P)
        got = tuple(int.from_bytes(outs[128 * i + 32 * k:128 * i + 32 * k + 32], "little") for k in range(4))
        if got != want:
            bad += 1
            if bad < 5:
                print("mismatch", i, hex(x), hex(y), [hex(g) for g in got], [hex(w) for w in want])
    print('{"subset": %d, "with_bit255": %d, "bigint_mismatches": %d}' % (n, high, bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
