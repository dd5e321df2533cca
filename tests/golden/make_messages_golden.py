#!/usr/bin/env python3
"""Generates tests/golden/messages.json: wire-format PrimaryMessages with their expected
sanitize codes and digests.

Positive cases are the reference's own primary test fixtures (primary/src/tests/common.rs:
keys() = StdRng::from_seed([0; 32]) keypairs, committee() = 4 authorities of stake 1 running worker
0, header(), headers(), votes(header), certificate(header), Certificate::genesis), which the
reference's core tests accept (primary/src/tests/core_tests.rs:11-89 process_header, :212-283
process_votes, :286-361 process_certificates).  Negative cases mutate them; their expected codes
come from the CPU restatement (oracle/messages_ref.py) with the Python restatement of dalek
(oracle/ed25519_ref.py) for signatures -- parity-unpinned by the reference's tests, which hold no
negative message fixtures.

    python tests/golden/make_messages_golden.py
"""
from __future__ import annotations

import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import ed25519_ref as ed  # noqa: E402
import messages_ref as mr  # noqa: E402


class PySig:
    def strict(self, m, pk, s):
        return ed.verify_strict(m, pk, s)

    def leaf(self, m, pk, s):
        return ed.leaf_ok(m, pk, s)


def main():
    gold = json.load(open(os.path.join(HERE, "ed25519_verify.json")))
    seeds = [bytes.fromhex(s) for s in gold["reference_keys"]["seeds"]]
    pks = [bytes.fromhex(p) for p in gold["reference_keys"]["pks"]]
    assert [ed.public_key(s) for s in seeds] == pks
    outsider_seed = bytes(range(32))
    outsider = ed.public_key(outsider_seed)
    committee = mr.RefCommittee({pk: (1, [0]) for pk in pks})
    sig = PySig()
    cases = []

    def add(name, msg, source, gc_round=0, target=None):
        code, kind, dig = mr.sanitize(msg, committee, sig, gc_round, target)
        cases.append({"name": name, "msg": msg.hex(), "code": code, "code_name": mr.NAMES[code],
                      "kind": kind if kind is not None else -1, "digest": dig.hex(), "gc_round": gc_round,
                      "target": None if target is None else [target[0].hex(), target[1], target[2].hex()],
                      "source": source})
        return code

    genesis = [mr.digest72(bytes(32), 0, pk) for pk in pks]

    def make_header(k, round_=1, payload=(), parents=None, seed=None, author=None):
        author = author if author is not None else pks[k]
        seed = seed if seed is not None else seeds[k]
        parents = genesis if parents is None else parents
        hid = mr.header_id(author, round_, list(payload), list(parents))
        return author, round_, list(payload), list(parents), hid, ed.sign(seed, hid)

    def hdr_bytes(h):
        return mr.enc_header(*h)

    def vote_sig(h, k):
        return ed.sign(seeds[k], mr.digest72(h[4], h[1], h[0]))

    REF = "reference fixture (primary/src/tests/common.rs), accepted by core_tests"
    RES = "restatement (oracle/messages_ref.py), parity-unpinned"
    # keys().pop() is the last key: header() is by key 3
    h3 = make_header(3)
    assert add("ref-header", mr.msg_header(hdr_bytes(h3)), REF) == 0
    for k in range(4):
        assert add("ref-headers-%d" % k, mr.msg_header(hdr_bytes(make_header(k))), REF) == 0
    target = (h3[4], h3[1], h3[0])
    for k in range(4):
        m = mr.msg_vote(h3[4], 1, h3[0], pks[k], vote_sig(h3, k))
        assert add("ref-vote-%d" % k, m, REF, target=target) == 0
    votes3 = [(pks[k], vote_sig(h3, k)) for k in range(4)]
    assert add("ref-certificate", mr.msg_certificate(hdr_bytes(h3), votes3), REF) == 0
    for k in range(4):
        hk = make_header(k)
        assert add("ref-certificates-%d" % k,
                   mr.msg_certificate(hdr_bytes(hk), [(pks[j], vote_sig(hk, j)) for j in range(4)]), REF) == 0
    for k in range(4):
        g = (pks[k], 0, [], [], bytes(32), bytes(64))
        assert add("ref-genesis-%d" % k, mr.msg_certificate(hdr_bytes(g), []), REF) == 0

    # ---- negative / edge cases (restatement) --------------------------------------------------
    bad_id = list(h3)
    bad_id[4] = bytes([h3[4][0] ^ 1]) + h3[4][1:]
    add("header-bad-id", mr.msg_header(hdr_bytes(bad_id)), RES)
    add("header-outsider", mr.msg_header(hdr_bytes(make_header(0, seed=outsider_seed, author=outsider))), RES)
    add("header-unknown-worker", mr.msg_header(hdr_bytes(make_header(2, payload=[(bytes([7] * 32), 1)]))), RES)
    add("header-known-worker", mr.msg_header(hdr_bytes(make_header(2, payload=[(bytes([7] * 32), 0),
                                                                             (bytes([3] * 32), 0)]))), RES)
    bad_sig = list(h3)
    bad_sig[5] = h3[5][:40] + bytes([h3[5][40] ^ 4]) + h3[5][41:]
    add("header-bad-signature", mr.msg_header(hdr_bytes(bad_sig)), RES)
    add("header-too-old", mr.msg_header(hdr_bytes(h3)), RES, gc_round=2)
    add("header-gc-equal", mr.msg_header(hdr_bytes(h3)), RES, gc_round=1)
    add("header-trailing-bytes", mr.msg_header(hdr_bytes(h3)) + b"\x01\x02\x03", RES)
    add("header-many-parents", mr.msg_header(hdr_bytes(make_header(
        1, round_=5, parents=[bytes([i] * 32) for i in range(40)],
        payload=[(bytes([i + 100] * 32), 0) for i in range(9)]))), RES)

    C = mr.msg_certificate
    add("cert-two-votes-no-quorum", C(hdr_bytes(h3), votes3[:2]), RES)
    add("cert-three-votes", C(hdr_bytes(h3), votes3[:3]), RES)
    add("cert-reuse", C(hdr_bytes(h3), votes3[:2] + [votes3[1]] + votes3[2:]), RES)
    out_vote = (outsider, ed.sign(outsider_seed, mr.digest72(h3[4], 1, h3[0])))
    add("cert-outsider-then-reuse", C(hdr_bytes(h3), [votes3[0], out_vote, votes3[0]] + votes3[1:]), RES)
    add("cert-reuse-then-outsider", C(hdr_bytes(h3), [votes3[0], votes3[0], out_vote] + votes3[1:]), RES)
    badv = list(votes3)
    badv[2] = (pks[2], badv[2][1][:50] + bytes([badv[2][1][50] ^ 1]) + badv[2][1][51:])
    add("cert-bad-vote-signature", C(hdr_bytes(h3), badv), RES)
    zero = list(votes3)
    zero[1] = (pks[1], bytes(64))          # crypto_tests.rs:96-115 verify_invalid_batch analogue
    add("cert-zero-signature-vote", C(hdr_bytes(h3), zero), RES)
    add("cert-bad-header-signature", C(hdr_bytes(bad_sig), votes3), RES)
    add("cert-bad-header-id", C(hdr_bytes(bad_id), votes3), RES)
    add("cert-too-old", C(hdr_bytes(h3), votes3), RES, gc_round=3)
    g0 = (pks[0], 0, [], [], bytes(32), bytes(64))
    add("genesis-too-old", C(hdr_bytes(g0), []), RES, gc_round=1)
    g_out = (outsider, 0, [], [], bytes(32), bytes(64))
    add("genesis-outsider", C(hdr_bytes(g_out), []), RES)
    g_r1 = (pks[0], 1, [], [], bytes(32), bytes(64))
    add("genesis-round-1", C(hdr_bytes(g_r1), []), RES)
    add("genesis-with-votes", C(hdr_bytes(g0), votes3[:1]), RES)
    add("cert-outsider-author", C(hdr_bytes(make_header(0, seed=outsider_seed, author=outsider)), votes3), RES)

    V = mr.msg_vote
    add("vote-no-target-check", V(h3[4], 1, h3[0], pks[1], vote_sig(h3, 1)), RES)
    add("vote-unexpected-id", V(bad_id[4], 1, h3[0], pks[1], vote_sig(h3, 1)), RES, target=target)
    add("vote-too-old", V(h3[4], 0, h3[0], pks[1], vote_sig(h3, 1)), RES, target=target)
    add("vote-outsider", V(h3[4], 1, h3[0], outsider, ed.sign(outsider_seed, mr.digest72(h3[4], 1, h3[0]))), RES,
        target=target)
    add("vote-bad-signature", V(h3[4], 1, h3[0], pks[1], vote_sig(h3, 2)), RES, target=target)

    # ---- wire-format errors -----------------------------------------------------------------
    good = mr.msg_header(hdr_bytes(h3))
    for cut in (0, 3, 4, 10, 40, 56, 70, len(good) - 65, len(good) - 1):
        add("truncated-header-%d" % cut, good[:cut], RES)
    goodc = C(hdr_bytes(h3), votes3)
    for cut in (len(goodc) - 1, len(goodc) - 64, len(goodc) - 116, len(goodc) - 117):
        add("truncated-cert-%d" % cut, goodc[:cut], RES)
    add("variant-3-certificates-request", struct.pack("<I", 3) + struct.pack("<Q", 0) + mr.enc_key(pks[0]), RES)
    add("variant-7", struct.pack("<I", 7) + good[4:], RES)
    bad_char = bytearray(good)
    bad_char[4 + 8 + 5] = ord("*")
    add("base64-bad-char", bytes(bad_char), RES)
    bits = bytearray(good)
    s42 = bits[4 + 8 + 42]
    bits[4 + 8 + 42] = ord(mr.B64[mr.B64.index(chr(s42)) ^ 1])
    add("base64-trailing-bits", bytes(bits), RES)
    nopad = bytearray(good)
    nopad[4 + 8 + 43] = ord("A")
    add("base64-no-padding-char", bytes(nopad), RES)
    short = struct.pack("<I", 0) + struct.pack("<Q", 43) + good[12:12 + 43] + good[4 + 8 + 44:]
    add("base64-length-43", short, RES)
    huge = bytearray(goodc)
    off = len(goodc) - 4 * 116 - 8
    huge[off:off + 8] = struct.pack("<Q", 1 << 40)
    add("cert-huge-vote-count", bytes(huge), RES)

    out = {"committee": {"keys": [p.hex() for p in pks], "stakes": [1] * 4, "workers": [[0]] * 4,
                         "source": "primary/src/tests/common.rs committee()"},
           "outsider": outsider.hex(), "cases": cases}
    json.dump(out, open(os.path.join(HERE, "messages.json"), "w"), indent=1)
    from collections import Counter
    print(len(cases), "cases", Counter(c["code_name"] for c in cases))


if __name__ == "__main__":
    main()
