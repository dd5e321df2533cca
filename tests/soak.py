#!/usr/bin/env python3
"""Differential soak: N synthetic (msg, pk, sig) triples, mutated into every input class the path
has (bit flips in R / s / A / msg, s + l, small-order and non-canonical R and A encodings, random R
and A bytes, the golden edge cases tiled in), verified on the GPU in strict and batch-leaf mode
and compared verdict by verdict with the CPU restatement (oracle/, multithreaded).

    python tests/soak.py [--n 8388608] [--chunk 1048576] [--committee K] [--call C] [--straus] [--out gpurun_out/soak.json]

--launch-keys K draws the signers from K keys WITHOUT registering them: every chunk's batch-leaf
launch (>= 65,536 equations) detects its repeated keys itself (launch keys) -- the
committee's, the small-order encodings and the golden cases' keys mutate() tiles in -- and decides
their votes with the comb kernel, the rest with the ladder.

--call C verifies each chunk in device calls of at most C equations (C <= 1024 without a
committee: the cold kernel, k_verify_cold, one block per equation).
--dalek runs every chunk, cut into ragged certificates as --host-batch does, through the MSM
entry with dalek's batch semantics (nwc_dev_verify_batch_msm: with launch keys, the comb leaves and
dalek's equation per certificate over their failing votes, resolve.h) with the z seed fixed, and
compares every certificate bit with the oracle's evaluation of dalek's equation for the same z_i
(orc_batch_z8) and the bad-vote bits with the leaves of the failing certificates.
--straus also runs every chunk through dalek's batch equation over sub-batches
(nwc_dev_verify_batch_straus, each triple its own certificate, so sub-batches mix every class):
its per-vote bits must equal the oracle leaf on every vote outside dalek's randomized domain
(orc_vote_class 1), where either outcome is dalek's.

Test infrastructure (it runs the oracle), kept under tests/ like the oracle helpers; not part of
the default pytest run (minutes of CPU oracle time).

Prints one JSON object: per class counts, valid counts and mismatches (must be 0)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from narwhal_amd import _lib, device  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402

P = (1 << 255) - 19
L = (1 << 252) + 27742317777372353535851937790883648493
Y8 = 0x05fc536d880238b13933c6d305acdfd5f098eff289f4c345b027b2c28f95e826   # y of the order-8 points


def enc(y: int, sign: int) -> bytes:
    return (y | (sign << 255)).to_bytes(32, "little")


SMALL = [enc(y, s) for y in (0, 1, P - 1, Y8, P - Y8) for s in (0, 1)] + \
        [enc(y + P, s) for y in (0, 1) for s in (0, 1)]   # non-canonical aliases y + p < 2^255
CLASSES = ["valid", "flip_R", "flip_s", "flip_A", "flip_msg", "s_plus_l", "small_R", "small_A",
           "random_R", "random_A", "noncanon_R", "golden"]


def mutate(rng, m, p, s, golden, valid_frac=0.30):
    n = len(p)
    rest = np.array([0.07, 0.07, 0.07, 0.07, 0.06, 0.06, 0.06, 0.06, 0.06, 0.06, 0.06])
    kind = rng.choice(len(CLASSES), n, p=np.concatenate([[valid_frac], rest / rest.sum() * (1 - valid_frac)]))
    idx = lambda k: np.nonzero(kind == k)[0]  # noqa: E731
    i = idx(1); s[i, rng.integers(0, 32, len(i))] ^= (1 << rng.integers(0, 8, len(i))).astype(np.uint8)
    i = idx(2); s[i, 32 + rng.integers(0, 32, len(i))] ^= (1 << rng.integers(0, 8, len(i))).astype(np.uint8)
    i = idx(3); p[i, rng.integers(0, 32, len(i))] ^= (1 << rng.integers(0, 8, len(i))).astype(np.uint8)
    i = idx(4); m[i, rng.integers(0, 32, len(i))] ^= (1 << rng.integers(0, 8, len(i))).astype(np.uint8)
    for j in idx(5):
        sv = int.from_bytes(s[j, 32:].tobytes(), "little") + L
        if sv < (1 << 256):
            s[j, 32:] = np.frombuffer(sv.to_bytes(32, "little"), np.uint8)
    small = np.frombuffer(b"".join(SMALL), np.uint8).reshape(-1, 32)
    i = idx(6); s[i, :32] = small[rng.integers(0, len(small), len(i))]
    i = idx(7); p[i] = small[rng.integers(0, len(small), len(i))]
    i = idx(8); s[i, :32] = rng.integers(0, 256, (len(i), 32), dtype=np.uint8)
    i = idx(9); p[i] = rng.integers(0, 256, (len(i), 32), dtype=np.uint8)
    for j in idx(10):   # same R point, non-canonical encoding when y + p fits (rare for random y)
        y = int.from_bytes(s[j, :32].tobytes(), "little")
        yy, sign = y & ((1 << 255) - 1), y >> 255
        if yy + P < (1 << 255):
            s[j, :32] = np.frombuffer(enc(yy + P, sign), np.uint8)
        else:
            s[j, 31] ^= 0x80   # else flip the sign bit
    gm, gp, gs = golden
    i = idx(11); g = rng.integers(0, len(gm), len(i)); m[i], p[i], s[i] = gm[g], gp[g], gs[g]
    return kind


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8 << 20)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "soak.json"))
    ap.add_argument("--committee", type=int, default=0,
                    help="K > 0: signers drawn from K keys registered with nwc_set_committee (comb path, "
                         "cached ladder and the uncached list for mutated keys)")
    ap.add_argument("--launch-keys", type=int, default=0,
                    help="K > 0: signers drawn from K keys that are NOT registered (launch keys)")
    ap.add_argument("--call", type=int, default=0, help="C > 0: device calls of at most C equations")
    ap.add_argument("--straus", action="store_true", help="also the Straus sub-batch path (per-vote bits vs the oracle)")
    ap.add_argument("--host-batch", action="store_true",
                    help="also nwc_verify_batch_many from host memory: each chunk's triples in ragged certificates "
                         "(0..130 votes, votes signing their certificate's digest before mutation), certificate and "
                         "bad-vote bits vs the oracle's batch_many on the same inputs")
    ap.add_argument("--dalek", action="store_true",
                    help="also the per-certificate dalek equation (fixed seed) on ragged certificates vs orc_batch_z8")
    ap.add_argument("--valid-frac", type=float, default=0.30,
                    help="share of unmutated triples (0.99: most Straus sub-batches pass, the rest exercise the leaves)")
    args = ap.parse_args()
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    if args.launch_keys:
        lseeds = device.derive32(b"soak-lk-seed", 0, args.launch_keys)
    if args.committee:
        cseeds = device.derive32(b"soak-seed", 0, args.committee)
        cpks, _ = device.keygen_sign(cseeds, cseeds)
        torch.cuda.synchronize()
        ck = cpks.cpu().numpy().copy()
        _lib.check(lib.nwc_set_committee(_lib.buf(ck), args.committee))
    orc = load_oracle()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_verify.json")))
    cases = [c for c in gold["cases"] if len(c["msg"]) == 64]
    golden = tuple(np.stack([np.frombuffer(bytes.fromhex(c[k]), np.uint8) for c in cases]) for k in ("msg", "pk", "sig"))
    rng = np.random.default_rng(20261016)
    stats = {c: {"n": 0, "strict_valid": 0, "leaf_valid": 0, "strict_mismatch": 0, "leaf_mismatch": 0,
                 "straus_mismatch": 0, "randomized": 0, "straus_randomized_pass": 0} for c in CLASSES}
    host_batch = {"votes": 0, "certificates": 0, "bad_votes": 0, "failing_certificates": 0, "mismatch": 0}
    dalek = {"votes": 0, "certificates": 0, "failing_certificates": 0, "certificates_with_randomized_votes": 0,
             "randomized_certificates_passed": 0, "cert_mismatch": 0, "bad_vote_mismatch": 0, "mismatch": 0}
    t0 = time.time()
    done = 0
    mism = []
    while done < args.n:
        n = min(args.chunk, args.n - done)
        if args.committee:
            who = torch.from_numpy(rng.integers(0, args.committee, n)).cuda()
            seeds = cseeds[who]
        elif args.launch_keys:
            who = torch.from_numpy(rng.integers(0, args.launch_keys, n)).cuda()
            seeds = lseeds[who]
        else:
            seeds = device.derive32(b"soak-seed", done, n)
        if args.host_batch or args.dalek:
            # ragged certificates over this chunk's triples; vote v signs its certificate's digest
            counts = []
            while sum(counts) < n:
                counts.append(int(rng.integers(0, 131)))
            counts[-1] -= sum(counts) - n
            offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
            ncert = len(counts)
            cdig = device.derive32(b"soak-cert", done, ncert).cpu().numpy().copy()
            vote_cert = np.repeat(np.arange(ncert), counts)
            msgs = torch.from_numpy(np.ascontiguousarray(cdig[vote_cert])).cuda()
        else:
            msgs = device.derive32(b"soak-msg", done, n)
        pks, sigs = device.keygen_sign(seeds, msgs)
        torch.cuda.synchronize()
        m, p, s = (t.cpu().numpy().copy() for t in (msgs, pks, sigs))
        kind = mutate(rng, m, p, s, golden, args.valid_frac)
        tm, tp, ts = (torch.from_numpy(x).cuda() for x in (m, p, s))
        def run(strict):
            step = args.call or n
            return np.concatenate([device.unpack_bits(device.verify(tm[a:a + step], tp[a:a + step], ts[a:a + step],
                                                                    strict=strict), min(step, n - a))
                                   for a in range(0, n, step)])
        gs, gl = run(True), run(False)
        os_ = orc.strict_many(m, p, s, threads=threads)
        ol = orc.leaf_many(m, p, s, threads=threads)
        if args.straus:
            ar = torch.arange(n + 1, dtype=torch.int32, device="cuda")
            gb = device.unpack_bits(device.verify_batch_straus(tm, ar, ar[:n], tp, ts), n)
            cls = orc.vote_class_many(m, p, s, threads=threads)
            rnd = cls == 1
            smis = (gb != ol) & ~rnd
        else:
            gb = np.zeros(n, bool)
            rnd = smis = np.zeros(n, bool)
        hb_mis = 0
        if args.host_batch:
            import ctypes
            cert = ctypes.create_string_buffer((ncert + 7) // 8)
            badb = ctypes.create_string_buffer((n + 7) // 8)
            _lib.check(lib.nwc_verify_batch_many(_lib.buf(cdig), _lib.buf(offs), _lib.buf(p), _lib.buf(s), ncert,
                                                 cert, badb))
            ocert, obad = orc.batch_many(cdig, offs, p, s, threads=threads)
            hbad = np.unpackbits(np.frombuffer(badb.raw, np.uint8), bitorder="little")[:n].astype(bool)
            hcert = np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:ncert].astype(bool)
            hb_mis = int((hbad != obad.astype(bool)).sum()) + int((hcert != ocert.astype(bool)).sum())
            host_batch["votes"] += n
            host_batch["certificates"] += ncert
            host_batch["bad_votes"] += int(obad.sum())
            host_batch["failing_certificates"] += int((~ocert.astype(bool)).sum())
            host_batch["mismatch"] += hb_mis
        if args.dalek:
            import hashlib
            from concurrent.futures import ThreadPoolExecutor
            seed = 0x5EED0000 + done // args.chunk
            _lib.diag_set("dalek_seed", seed)
            try:
                do = torch.from_numpy(offs.astype(np.int32)).cuda()
                dmi = torch.from_numpy(vote_cert.astype(np.int32)).cuda()
                leafw = device.verify_batch_msm(torch.from_numpy(cdig).cuda(), do, dmi, tp, ts)
                cw, bw = device.cert_reduce(leafw, do, n)
                torch.cuda.synchronize()
            finally:
                _lib.diag_set("dalek_seed", 0)
            gcert, gbad = device.unpack_bits(cw, ncert), device.unpack_bits(bw, n)
            sb = seed.to_bytes(4, "little") + bytes(28)
            zs = np.frombuffer(b"".join(hashlib.sha512(sb + v.to_bytes(8, "little")).digest()[:16] for v in range(n)),
                               np.uint8).reshape(n, 16)
            parts = np.array_split(np.arange(ncert), threads)

            def z8(part):
                if len(part) == 0:
                    return np.zeros(0, bool)
                c0, c1 = int(part[0]), int(part[-1]) + 1
                v0, v1 = int(offs[c0]), int(offs[c1])
                return orc.batch_z_many(cdig[c0:c1], (offs[c0:c1 + 1] - v0).astype(np.uint32), p[v0:v1], s[v0:v1],
                                        zs[v0:v1], z8=True)
            with ThreadPoolExecutor(threads) as ex:
                ocert = np.concatenate(list(ex.map(z8, parts)))
            # the votes' leaves against their certificate's digest (the mutations changed m, which
            # the certificate path never reads): the bad set of a rejected certificate
            olc = orc.leaf_many(np.ascontiguousarray(cdig[vote_cert]), p, s, threads=threads).astype(bool)
            obad = ~olc & ~np.repeat(ocert, counts)
            dalek["cert_mismatch"] += int((gcert != ocert).sum())
            dalek["bad_vote_mismatch"] += int((gbad != obad).sum())
            dmis = int((gcert != ocert).sum()) + int((gbad != obad).sum())
            cls = orc.vote_class_many(m, p, s, threads=threads)
            csum = np.concatenate([[0], np.cumsum(cls == 1)])
            rcert = (csum[offs[1:].astype(np.int64)] - csum[offs[:-1].astype(np.int64)]) > 0
            dalek["votes"] += n
            dalek["certificates"] += ncert
            dalek["failing_certificates"] += int((~ocert).sum())
            dalek["certificates_with_randomized_votes"] += int(rcert.sum())
            dalek["randomized_certificates_passed"] += int((rcert & ocert).sum())
            dalek["mismatch"] += dmis
        for j in np.nonzero((gs != os_) | (gl != ol) | smis)[0][:20]:
            mism.append({"class": CLASSES[kind[j]], "index": int(done + j), "msg": m[j].tobytes().hex(),
                         "pk": p[j].tobytes().hex(), "sig": s[j].tobytes().hex(), "gpu_strict": bool(gs[j]),
                         "oracle_strict": bool(os_[j]), "gpu_leaf": bool(gl[j]), "oracle_leaf": bool(ol[j]),
                         "gpu_straus": bool(gb[j]) if args.straus else None})
        for k, name in enumerate(CLASSES):
            sel = kind == k
            st = stats[name]
            st["n"] += int(sel.sum())
            st["strict_valid"] += int(os_[sel].sum())
            st["leaf_valid"] += int(ol[sel].sum())
            st["strict_mismatch"] += int((gs[sel] != os_[sel]).sum())
            st["leaf_mismatch"] += int((gl[sel] != ol[sel]).sum())
            st["straus_mismatch"] += int(smis[sel].sum())
            st["randomized"] += int(rnd[sel].sum())
            st["straus_randomized_pass"] += int((rnd & (gb != 0))[sel].sum())
        done += n
        print("soak %d / %d  %.0f s" % (done, args.n, time.time() - t0), file=sys.stderr, flush=True)
    total = {k: sum(v[k] for v in stats.values()) for k in ("n", "strict_mismatch", "leaf_mismatch", "straus_mismatch",
                                                             "randomized", "straus_randomized_pass")}
    held = None
    if args.launch_keys:
        import ctypes
        h = ctypes.c_uint32()
        _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
        held = h.value
    out = {"triples": args.n, "committee": args.committee, "launch_keys": args.launch_keys, "launch_keys_held": held,
           "call": args.call, "straus": args.straus, "host_batch": host_batch if args.host_batch else None,
           "dalek": dalek if args.dalek else None,
           "valid_frac": args.valid_frac, "oracle_threads": threads, "seconds": time.time() - t0, "classes": stats, "total": total,
           "mismatches": mism}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(dict(total, host_batch_mismatch=host_batch["mismatch"], dalek_mismatch=dalek["mismatch"])))
    return 0 if (total["strict_mismatch"] == 0 and total["leaf_mismatch"] == 0 and total["straus_mismatch"] == 0
                 and host_batch["mismatch"] == 0 and dalek["mismatch"] == 0) else 1


if __name__ == "__main__":
    sys.exit(main())
