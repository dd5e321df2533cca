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

    # ---- round 2: BTreeMap / BTreeSet canonicalisation (primary/src/messages.rs:17-18, 75-81) ------
    CAN = "restatement: serde builds the BTreeMap/BTreeSet (sorted, deduplicated, last value wins)"

    def wire_header(k, parents, payload, id_over_wire=False, round_=2):
        """Header of key k sent with entries in the given (wire) order; its id is Header::digest of
        the canonical form, or (id_over_wire) of the wire order as a confused peer might compute."""
        if id_over_wire:
            b = pks[k] + struct.pack("<Q", round_)
            for d, w in payload:
                b += d + struct.pack("<I", w)
            hid = mr.sha512_32(b + b"".join(parents))
        else:
            hid = mr.header_id(pks[k], round_, payload, parents)
        return mr.enc_header(pks[k], round_, payload, parents, hid, ed.sign(seeds[k], hid), wire_order=True), hid

    P = [bytes([v] * 32) for v in (200, 13, 150, 7, 99, 42)]              # distinct digests, not sorted
    assert sorted(P) != P
    for name, parents, payload, over_wire in [
            ("header-unsorted-parents", P, [], False),
            ("header-duplicate-parents", P[:3] + P[:2] + P[3:], [], False),
            ("header-unsorted-parents-id-over-wire-order", P, [], True),
            ("header-duplicate-parents-id-over-wire-order", P[:3] + [P[0]] + P[3:], [], True),
            ("header-unsorted-payload", [], [(P[4], 0), (P[1], 0), (P[2], 0)], False),
            ("header-duplicate-payload-bad-then-good", P[:2], [(P[3], 1), (P[1], 0), (P[3], 0)], False),
            ("header-duplicate-payload-good-then-bad", P[:2], [(P[3], 0), (P[1], 0), (P[3], 1)], False),
            ("header-duplicate-payload-same", P[:2], [(P[3], 0), (P[3], 0), (P[0], 0)], False),
            ("header-many-unsorted", [bytes([(i * 101 + 7) % 256] * 32) for i in range(150)] +
             [bytes([(i * 101 + 7) % 256] * 32) for i in range(0, 150, 7)],
             [(bytes([(i * 53 + 1) % 256] * 32), 0) for i in range(70)] + [(bytes([54] * 32), 0)], False)]:
        hb, hid = wire_header(1, parents, payload, over_wire)
        add(name, mr.msg_header(hb), CAN)
        # the same header inside a certificate with the committee's votes on it
        vs = [(pks[j], ed.sign(seeds[j], mr.digest72(hid, 2, pks[1]))) for j in range(4)]
        add(name.replace("header-", "cert-", 1), C(hb, vs), CAN)

    # ---- round 2: base64 0.13 key forms (crypto/src/lib.rs:73-79) ---------------------------------
    B64R = "restatement of base64 0.13 decode + bytes[..32] (crypto/src/lib.rs:73-79)"
    import base64 as _b64

    def forms_of(pk):
        k = _b64.b64encode(pk)
        return {
            "unpadded-43": k[:43],
            "long-88": _b64.b64encode(pk + bytes(range(32))),            # first 32 bytes are the key
            "long-45-unpadded": _b64.b64encode(pk + b"\x07\x09").rstrip(b"="),
            "long-48": _b64.b64encode(pk + b"\x01\x02\x03\x04"),
            "short-31-bytes": _b64.b64encode(pk[:31]),                   # decodes to 31 bytes: panic
            "empty": b"",                                                # 0 bytes: panic
            "short-40-chars": k[:40],                                    # 30 bytes: panic
            "pad-at-42": k[:42] + b"==",                                 # '=' at chunk position 2, too early
            "len-45": k + b"A",                                          # 45 % 8 == 5: InvalidLength
            "len-41": k[:41],                                            # 41 % 8 == 1
            "pad-then-symbol": k[:43] + b"=A==",
            "non-utf8": k[:20] + b"\xff" + k[21:],
            "space": k[:43] + b" ",
            "nonzero-trailing-unpadded": k[:42] + mr.B64[mr.B64.index(chr(k[42])) | 1].encode(),
        }

    f1 = forms_of(pks[1])
    for fname, text in f1.items():
        hid = mr.header_id(pks[1], 3, [], [])
        hb = mr.enc_header(pks[1], 3, [], [], hid, ed.sign(seeds[1], hid), author_text=text)
        add("b64-header-author-" + fname, mr.msg_header(hb), B64R)
        add("b64-cert-vote1-" + fname, C(hdr_bytes(h3), votes3, key_texts=[None, text, None, None]), B64R)
        add("b64-vote-author-" + fname,
            struct.pack("<I", 1) + h3[4] + struct.pack("<Q", 1) + mr.enc_key(h3[0]) + mr.enc_key(pks[1], text) +
            vote_sig(h3, 1), B64R, target=target)
    add("b64-vote-origin-unpadded", struct.pack("<I", 1) + h3[4] + struct.pack("<Q", 1) +
        mr.enc_key(h3[0], forms_of(h3[0])["unpadded-43"]) + mr.enc_key(pks[1]) + vote_sig(h3, 1), B64R, target=target)
    # the first failing vote decides: a panicking key before an invalid one, and after it
    f2 = forms_of(pks[2])
    add("b64-cert-panic-then-error", C(hdr_bytes(h3), votes3, key_texts=[None, f1["empty"], f2["len-45"], None]), B64R)
    add("b64-cert-error-then-panic", C(hdr_bytes(h3), votes3, key_texts=[None, f1["len-45"], f2["empty"], None]), B64R)
    full = C(hdr_bytes(h3), votes3, key_texts=[None, None, None, forms_of(pks[3])["short-31-bytes"]])
    add("b64-cert-panic-in-truncated-last-vote", full[:-10], B64R)
    add("b64-cert-truncated-in-key-of-panic-vote", full[:-64 - 3], B64R)
    mixed = [None, f1["unpadded-43"], f2["long-88"], forms_of(pks[3])["long-48"]]
    add("b64-cert-mixed-key-lengths", C(hdr_bytes(h3), votes3, key_texts=mixed), B64R)
    add("b64-cert-mixed-key-lengths-reuse", C(hdr_bytes(h3), votes3 + [votes3[1]], key_texts=mixed + [f1["long-48"]]),
        B64R)
    add("b64-cert-mixed-key-lengths-bad-sig", C(hdr_bytes(h3), badv, key_texts=mixed), B64R)
    add("b64-cert-mixed-key-lengths-unsorted-header",
        C(wire_header(1, P, [], False, round_=2)[0],
          [(pks[j], ed.sign(seeds[j], mr.digest72(wire_header(1, P, [], False, round_=2)[1], 2, pks[1])))
           for j in range(4)], key_texts=[f1 and forms_of(pks[0])["long-88"], f1["unpadded-43"], None, None]), B64R)

    out = {"committee": {"keys": [p.hex() for p in pks], "stakes": [1] * 4, "workers": [[0]] * 4,
                         "source": "primary/src/tests/common.rs committee()"},
           "outsider": outsider.hex(), "cases": cases}
    json.dump(out, open(os.path.join(HERE, "messages.json"), "w"), indent=1)
    from collections import Counter
    print(len(cases), "cases", Counter(c["code_name"] for c in cases))


if __name__ == "__main__":
    main()
