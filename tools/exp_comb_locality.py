#!/usr/bin/env python3
"""Experiment: does the committee comb kernel (k_verify_comb) run faster when the votes of one key
are contiguous in the launch?  Config-3 votes (100 keys, 1 % bad) with the committee cache, timed
in the caller's order (every certificate's 67 voters interleaved), grouped by key (a permutation
of the same votes), and with a single-key committee (the locality limit).

    python tools/exp_comb_locality.py [--certs 100000] [--steps 5]   -> one JSON line
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--certs", type=int, default=100000)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from narwhal_amd import _lib, device
    lib = _lib.load()
    m, N, Q = args.certs, 100, 67
    nv = m * Q
    cseeds = device.derive32(b"nw-committee", 0, N)
    cdig = device.derive32(b"nw-cert", 0, m)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x4E57)
    voters = torch.rand((m, N), device="cuda", generator=g).argsort(dim=1)[:, :Q].reshape(-1)
    bad = torch.rand(nv, device="cuda", generator=g) < 0.01
    msg_index = torch.arange(m, device="cuda", dtype=torch.int32).repeat_interleave(Q)
    signed = cdig[msg_index.long()].clone()
    signed[bad, 0] ^= 1
    pks, sigs = device.keygen_sign(cseeds[voters], signed)
    committee_pks, _ = device.keygen_sign(cseeds, cdig[:N])
    torch.cuda.synchronize()
    cpk = committee_pks.cpu().numpy()   # kept alive across the call (_lib.buf holds a raw pointer)
    _lib.check(lib.nwc_set_committee(_lib.buf(cpk), N))
    perm = torch.argsort(voters, stable=True)
    cases = {
        "caller_order": (pks, sigs, msg_index, bad),
        "grouped_by_key": (pks[perm].contiguous(), sigs[perm].contiguous(), msg_index[perm].contiguous(), bad[perm]),
    }
    out = {}
    for tag, (P, S, MI, want_bad) in cases.items():
        words = torch.empty(device.words_for(nv), dtype=torch.int64, device="cuda")
        run = lambda: device.verify(cdig, P, S, strict=False, msg_index=MI, out=words)  # noqa: E731
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            w = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        got_bad = ~torch.from_numpy(device.unpack_bits(w, nv)).cuda()
        out[tag] = {"votes_per_s": nv / dt, "ms": dt * 1e3, "verdicts_ok": bool((got_bad == want_bad).all())}
    # one key: every vote by committee member 0 (its own signatures); the same 100-key committee
    one = torch.zeros_like(voters)
    P1, S1 = device.keygen_sign(cseeds[one], signed)
    torch.cuda.synchronize()
    words = torch.empty(device.words_for(nv), dtype=torch.int64, device="cuda")
    run = lambda: device.verify(cdig, P1, S1, strict=False, msg_index=msg_index, out=words)  # noqa: E731
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        w = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    got_bad = ~torch.from_numpy(device.unpack_bits(w, nv)).cuda()
    out["one_key"] = {"votes_per_s": nv / dt, "ms": dt * 1e3, "verdicts_ok": bool((got_bad == bad).all())}
    _lib.check(lib.nwc_set_committee(None, 0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
