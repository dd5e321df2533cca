"""GPU message pipeline (nwc_sanitize_messages): wire bytes in, DagError codes and message digests
out -- against the golden fixtures (the reference's primary test fixtures + restated negatives)
and, on larger randomized batches, against the CPU restatement (oracle/messages_ref.py with the C
restatement of dalek for signatures)."""
import ctypes
import json
import os
import struct
import sys

import numpy as np
import pytest

from tests.conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "oracle"))


@pytest.fixture(scope="module")
def lib():
    from narwhal_amd import _lib
    return _lib.load()


class _CSig:
    def __init__(self, oracle):
        self.o = oracle

    def strict(self, m, pk, s):
        return self.o.verify_strict(m, pk, s)

    def leaf(self, m, pk, s):
        return self.o.leaf(m, pk, s)


def _install(lib, keys, stakes, workers):
    from narwhal_amd import _lib
    n = len(keys)
    offs, ids = [0], []
    for w in workers:
        ids.extend(w)
        offs.append(len(ids))
    kb = b"".join(keys)
    _lib.check(lib.nwc_set_committee_config(_lib.buf(kb), (ctypes.c_uint64 * n)(*stakes), n,
                                            (ctypes.c_uint32 * (n + 1))(*offs), (ctypes.c_uint32 * max(1, len(ids)))(*ids)))


def _sanitize(lib, msgs, gc_round=0, target=None):
    from narwhal_amd import _lib
    m = len(msgs)
    offs = np.zeros(m + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in msgs])
    data = b"".join(msgs) or b"\0"
    codes = np.zeros(m, np.int32)
    dig = np.zeros((m, 32), np.uint8)
    kinds = np.zeros(m, np.uint8)
    tb = None
    if target is not None:
        tb = target[0] + struct.pack("<Q", target[1]) + target[2]
    _lib.check(lib.nwc_sanitize_messages(_lib.buf(data), _lib.buf(offs), m, gc_round, _lib.buf(tb) if tb else None,
                                         _lib.buf(codes), _lib.buf(dig), _lib.buf(kinds)))
    return codes, dig, kinds


def test_golden_messages(lib):
    g = json.load(open(os.path.join(GOLDEN, "messages.json")))
    c = g["committee"]
    _install(lib, [bytes.fromhex(k) for k in c["keys"]], c["stakes"], c["workers"])
    groups = {}
    for case in g["cases"]:
        key = (case["gc_round"], json.dumps(case["target"]))
        groups.setdefault(key, []).append(case)
    try:
        for (gc, tj), cases in groups.items():
            t = json.loads(tj)
            target = None if t is None else (bytes.fromhex(t[0]), t[1], bytes.fromhex(t[2]))
            codes, dig, kinds = _sanitize(lib, [bytes.fromhex(x["msg"]) for x in cases], gc, target)
            for i, case in enumerate(cases):
                assert codes[i] == case["code"], (case["name"], int(codes[i]), case["code_name"])
                if case["kind"] >= 0 and case["kind"] != 3:
                    assert dig[i].tobytes().hex() == case["digest"], case["name"]
                    assert kinds[i] == case["kind"], case["name"]
    finally:
        lib.nwc_set_committee(None, 0)


def _random_batch(oracle, rng, N=100, ncert=300, nhdr=100, nvote=200):
    """Committee of N (stakes 1..3, 1-2 workers); certificates with quorum-sized vote sets, headers
    and votes, each mutated with small probability in one of the ways the checks distinguish."""
    import messages_ref as mr
    seeds = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(N + 5)]
    pks = [oracle.public_key(s) for s in seeds]
    stakes = [int(x) for x in rng.integers(1, 4, N)]
    workers = [[0] if rng.random() < 0.5 else [0, 1] for _ in range(N)]
    committee = mr.RefCommittee({pks[k]: (stakes[k], workers[k]) for k in range(N)})
    quorum = committee.quorum_threshold()

    def header(k, rnd):
        parents = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(int(rng.integers(0, 8)))]
        payload = [(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), int(rng.integers(0, 2)))
                   for _ in range(int(rng.integers(0, 3)))]
        payload = [(d, w if w in workers[k % N] or rng.random() < 0.3 else 0) for d, w in payload]
        if rng.random() < 0.15 and parents:      # Byzantine wire order: duplicates, unsorted
            parents = parents + [parents[int(rng.integers(0, len(parents)))]]
        if rng.random() < 0.15 and payload:
            d0, _ = payload[int(rng.integers(0, len(payload)))]
            payload = payload + [(d0, int(rng.integers(0, 2)))]
        if rng.random() < 0.1:
            parents.reverse()
            payload.reverse()
        hid = mr.header_id(pks[k], rnd, payload, parents)
        return [pks[k], rnd, payload, parents, hid, oracle.sign(seeds[k], hid)]

    import base64

    def key_text(pk, p=0.1):
        """base64 0.13 accepts more than base64::encode emits (crypto/src/lib.rs:73-79)."""
        if rng.random() >= p:
            return None
        u = 0.9 + 0.1 * rng.random()
        if u < 0.94:
            return base64.b64encode(pk)[:43]                        # unpadded
        if u < 0.97:
            return base64.b64encode(pk + bytes(int(rng.integers(1, 40))))   # longer decode
        return base64.b64encode(pk[:int(rng.integers(0, 32))])       # < 32 bytes: panic

    msgs = []
    for _ in range(ncert):
        k = int(rng.integers(0, N + 5 if rng.random() < 0.03 else N))
        rnd = int(rng.integers(1, 50))
        h = header(k, rnd)
        if rng.random() < 0.03:
            h[4] = bytes([h[4][0] ^ 1]) + h[4][1:]
        if rng.random() < 0.03:
            h[5] = h[5][:33] + bytes([h[5][33] ^ 2]) + h[5][34:]
        cd = mr.digest72(h[4], h[1], h[0])
        order = list(rng.permutation(N))
        voters, w = [], 0
        for v in order:
            voters.append(int(v))
            w += stakes[v]
            if w >= quorum:
                break
        if rng.random() < 0.05:
            voters = voters[:-1]
        if rng.random() < 0.03:
            voters.insert(int(rng.integers(0, len(voters))), voters[0])
        if rng.random() < 0.03:
            voters.insert(int(rng.integers(0, len(voters))), N + 1)
        votes = [(pks[v], oracle.sign(seeds[v], cd)) for v in voters]
        if rng.random() < 0.04:
            j = int(rng.integers(0, len(votes)))
            s = votes[j][1]
            votes[j] = (votes[j][0], s[:45] + bytes([s[45] ^ 8]) + s[46:])
        m = mr.msg_certificate(mr.enc_header(*h, wire_order=True, author_text=key_text(h[0])), votes,
                               key_texts=[key_text(kk, 0.005) for kk, _ in votes])
        if rng.random() < 0.02:
            m = m[:int(rng.integers(0, len(m)))]
        msgs.append(m)
    for _ in range(nhdr):
        k = int(rng.integers(0, N + 5 if rng.random() < 0.05 else N))
        h = header(k, int(rng.integers(0, 50)))
        if rng.random() < 0.05:
            h[5] = bytes(64)
        msgs.append(mr.msg_header(mr.enc_header(*h, wire_order=True, author_text=key_text(h[0]))))
    for _ in range(nvote):
        k = int(rng.integers(0, N + 5 if rng.random() < 0.05 else N))
        hid = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        origin = pks[int(rng.integers(0, N))]
        rnd = int(rng.integers(0, 50))
        s = oracle.sign(seeds[k], mr.digest72(hid, rnd, origin))
        if rng.random() < 0.05:
            s = s[:10] + bytes([s[10] ^ 1]) + s[11:]
        msgs.append(struct.pack("<I", 1) + hid + struct.pack("<Q", rnd) + mr.enc_key(origin, key_text(origin)) +
                    mr.enc_key(pks[k], key_text(pks[k])) + s)
    order = rng.permutation(len(msgs))
    return committee, pks[:N], stakes, workers, [msgs[i] for i in order]


def test_random_batches_vs_oracle(lib, oracle):
    import messages_ref as mr
    rng = np.random.default_rng(2024)
    committee, pks, stakes, workers, msgs = _random_batch(oracle, rng)
    _install(lib, pks, stakes, workers)
    sig = _CSig(oracle)
    try:
        for gc in (0, 20):
            codes, dig, kinds = _sanitize(lib, msgs, gc)
            for i, m in enumerate(msgs):
                code, kind, d = mr.sanitize(m, committee, sig, gc)
                assert codes[i] == code, (i, int(codes[i]), mr.NAMES[code])
                if kind in (0, 1, 2):
                    assert dig[i].tobytes() == d, i
        counts = np.bincount(codes, minlength=12)
        assert counts[0] > 100 and counts[1] > 5 and counts[6] > 3 and counts[11] > 3   # the mix exercises the paths
    finally:
        lib.nwc_set_committee(None, 0)


def test_mirror_objects(lib):
    """narwhal_amd.messages: Header::new / Vote::new / Certificate through verify(), DagError."""
    from narwhal_amd.crypto import Digest, PublicKey, SecretKey
    from narwhal_amd.messages import Authority, Certificate, Committee, DagError, Header, Vote, sanitize_many
    g = json.load(open(os.path.join(GOLDEN, "ed25519_verify.json")))
    seeds = [bytes.fromhex(s) for s in g["reference_keys"]["seeds"]]
    keys = [(PublicKey(bytes.fromhex(p)), SecretKey(s + bytes.fromhex(p)))
            for s, p in zip(seeds, g["reference_keys"]["pks"])]
    committee = Committee({pk: Authority(1, [0]) for pk, _ in keys})
    try:
        parents = {c.digest() for c in Certificate.genesis(committee)}
        author, secret = keys[3]
        h = Header.new(author, 1, {}, parents, secret)
        h.verify(committee)
        votes = [Vote.new(h, pk, sk) for pk, sk in keys]
        for v in votes:
            v.verify(committee)
        cert = Certificate(h, [(v.author, v.signature) for v in votes])
        cert.verify(committee)
        digs = []
        errs = sanitize_many([h.to_bytes(), cert.to_bytes()] + [v.to_bytes() for v in votes], committee,
                             current_header=h, digests=digs)
        assert errs == [None] * 6
        assert digs[0] == h.id and digs[1] == cert.digest() and digs[2] == votes[0].digest()
        short = Certificate(h, cert.votes[:2])
        with pytest.raises(DagError) as e:
            short.verify(committee)
        assert e.value.name == "CertificateRequiresQuorum"
        bad = Header(h.author, h.round, {Digest(bytes(32)): 5}, h.parents, h.id, h.signature)
        with pytest.raises(DagError) as e:
            bad.verify(committee)
        assert e.value.name == "InvalidHeaderId"
    finally:
        lib.nwc_set_committee(None, 0)


def test_large_unsorted_headers(lib, oracle):
    """Byzantine headers whose payload map / parent set arrive unsorted, reversed and with duplicates,
    from small to a near-maximum frame (200k parents = 6.4 MB of the LengthDelimitedCodec's 8 MiB):
    codes and digests against the restatement, and the big one bounded in time (the bitonic path of
    messages.h canon_entries; the rank method needed cnt^2 loads)."""
    import time
    import messages_ref as mr
    rng = np.random.default_rng(77)
    seeds = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(4)]
    pks = [oracle.public_key(s) for s in seeds]
    committee = mr.RefCommittee({pk: (1, [0, 1]) for pk in pks})
    _install(lib, pks, [1] * 4, [[0, 1]] * 4)
    sig = _CSig(oracle)

    def header(nparents, npayload, ids_on_wire=False):
        parents = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(nparents)]
        parents = sorted(parents, reverse=True)
        parents += [parents[int(i)] for i in rng.integers(0, nparents, max(1, nparents // 10))]
        parents = [parents[int(i)] for i in rng.permutation(len(parents))] if rng.random() < 0.5 else parents
        payload = [(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), int(rng.integers(0, 2))) for _ in range(npayload)]
        payload += [(payload[int(i)][0], int(rng.integers(0, 3))) for i in rng.integers(0, max(1, npayload), npayload // 8)]
        payload.reverse()
        if ids_on_wire:   # id over the wire order: InvalidHeaderId
            b = pks[0] + struct.pack("<Q", 5)
            b += b"".join(d + struct.pack("<I", w) for d, w in payload) + b"".join(parents)
            hid = mr.sha512_32(b)
        else:
            hid = mr.header_id(pks[0], 5, payload, parents)
        return mr.msg_header(mr.enc_header(pks[0], 5, payload, parents, hid, oracle.sign(seeds[0], hid),
                                           wire_order=True))

    try:
        msgs = [header(n, p, w) for n, p in ((600, 40), (700, 600), (5000, 3000), (20000, 0)) for w in (False, True)]
        codes, dig, _ = _sanitize(lib, msgs)
        for i, m in enumerate(msgs):
            code, kind, d = mr.sanitize(m, committee, sig)
            assert codes[i] == code, (i, int(codes[i]), mr.NAMES[code])
            assert dig[i].tobytes() == d, i
        big = header(200000, 0)
        assert len(big) < 8 << 20
        _sanitize(lib, [big])                  # warm-up (allocations)
        t0 = time.perf_counter()
        codes, dig, _ = _sanitize(lib, [big])
        dt = time.perf_counter() - t0
        code, _, d = mr.sanitize(big, committee, sig)
        assert codes[0] == code and dig[0].tobytes() == d
        print("200k unsorted parents: %.1f ms" % (dt * 1e3))
        assert dt < 2.0, dt
    finally:
        lib.nwc_set_committee(None, 0)


@pytest.mark.parametrize("env", [{}, {"NWC_STRICT_Y": "0"}, {"NWC_SIGN_DEFER": "0"}])
def test_random_batches_chunked_vs_oracle(oracle, tmp_path, env):
    """The random batch (outsiders, bad header and vote signatures, quorum failures, base64 key
    forms, truncations) tiled to ~10 MB and sent through the chunked host pipeline in 1-MB chunks
    (a child process: libnwc reads NWC_MSG_CHUNK once): every code and digest equals the
    restatement's.  Covers the strict equations without the uncached list on the parse stream
    (outsiders' messages end in UnknownAuthority first), the list path and k_verify_comb."""
    import subprocess
    import messages_ref as mr
    rng = np.random.default_rng(2026)
    committee, pks, stakes, workers, msgs = _random_batch(oracle, rng)
    sig = _CSig(oracle)
    exp = [mr.sanitize(m, committee, sig, 0) for m in msgs]
    reps = 1 + (10 << 20) // sum(len(m) for m in msgs)
    tiled = msgs * reps
    offs = np.zeros(len(tiled) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in tiled])
    woffs, wids = [0], []
    for w in workers:
        wids.extend(w)
        woffs.append(len(wids))
    inp, out = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    np.savez(inp, data=np.frombuffer(b"".join(tiled), np.uint8), offs=offs,
             keys=np.frombuffer(b"".join(pks), np.uint8).reshape(len(pks), 32), stakes=np.array(stakes, np.uint64),
             woffs=np.array(woffs, np.uint32), wids=np.array(wids, np.uint32), gc=0)
    e = dict(os.environ, NWC_MSG_CHUNK=str(1 << 20), **env)
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize_chunk_helper.py"), inp, out, ROOT], env=e,
                   check=True, timeout=300)
    r = np.load(out)
    for i in range(len(tiled)):
        code, kind, d = exp[i % len(msgs)]
        assert r["codes"][i] == code, (env, i, int(r["codes"][i]), mr.NAMES[code])
        if kind in (0, 1, 2):
            assert r["dig"][i].tobytes() == d, (env, i)
    counts = np.bincount(r["codes"], minlength=12)
    assert counts[0] > 100 and counts[1] > 5 and counts[4] > 5
