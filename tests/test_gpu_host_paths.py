"""Large host calls (the Rust shim's situation: pageable host buffers in, bitmaps out) against the
oracle: nwc_verify_strict_many and nwc_verify_batch_many over several pipelined chunks, whose
inputs travel through the device's pinned stages (copy_pool.h HostStager) -- chunk boundaries,
stage boundaries (32 MB) and the verdict merge all crossed -- and, for the certificates, launch
keys picking the committee up inside the chunks (crypto/src/lib.rs:200-219)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(buf, n):
    return np.unpackbits(np.frombuffer(buf.raw, np.uint8), bitorder="little")[:n].astype(bool)


def test_strict_many_host_chunks(oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(81)
    n = 400_000   # chunks of 131,072 then x3: two chunks, the second across stage boundaries
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    bad = rng.random(n) < 0.02
    bad[[0, 63, 64, 131071, 131072, 131073, n - 1]] = True
    sigs[bad, 45] ^= 4
    out = ctypes.create_string_buffer((n + 7) // 8)
    _lib.check(lib.nwc_verify_strict_many(_lib.buf(msgs), _lib.buf(pks), _lib.buf(sigs), n, out))
    got = _bits(out, n)
    exp = oracle.strict_many(msgs, pks, sigs)
    assert (exp == ~bad).all()
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


def test_strict_many_host_ragged(oracle):
    """The paired host pipeline (strict calls, no committee cache) at sizes that end inside a
    64-equation wave and off every chunk boundary, twice in a row on the same stages and arena:
    verdicts equal the oracle's."""
    from narwhal_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(83)
    for n in (262_144 + 16_384 * 3 + 17, 300_001):
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        pks, sigs = oracle.keygen_sign_many(seeds, msgs)
        bad = rng.random(n) < 0.01
        bad[[16_383, 16_384, n - 1]] = True
        sigs[bad, 2] ^= 8
        out = ctypes.create_string_buffer((n + 7) // 8)
        _lib.check(lib.nwc_verify_strict_many(_lib.buf(msgs), _lib.buf(pks), _lib.buf(sigs), n, out))
        got = _bits(out, n)
        exp = oracle.strict_many(msgs, pks, sigs)
        assert (got == exp).all(), (n, np.nonzero(got != exp)[0][:10])
        assert (exp == ~bad).all()


@pytest.mark.parametrize("env", [{"NWC_HOST_PAIR_FIRST": "4096", "NWC_HOST_PAIR_GROWTH": "2"},
                                 {"NWC_HOST_PAIR_FIRST": "8192", "NWC_HOST_PAIR_GROWTH": "1",
                                  "NWC_FORCE_FALLBACK_EVERY": "3"},
                                 {"NWC_HOST_PAIR": "0"}])
def test_strict_many_host_pipelines(env, oracle, tmp_path):
    """Strict host calls through the paired pipeline cut into many alternating chunks (each chunk
    on its own half of the table slots and its own fallback list; one case sends every third
    equation of each chunk through the fallback kernel) and through the single-stream chunks:
    verdicts equal the oracle's, on two calls in a row.  Each case in its own process (libnwc
    reads the switches once)."""
    import os
    import subprocess
    import sys
    from tests.conftest import ROOT
    rng = np.random.default_rng(84)
    n = 150_001
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    bad = rng.random(n) < 0.01
    bad[[4095, 4096, 8191, 8192, 12287, 12288, n - 1]] = True
    sigs[bad, 9] ^= 2
    exp = oracle.strict_many(msgs, pks, sigs)
    assert (exp == ~bad).all()
    inp, out = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    np.savez(inp, m=msgs, p=pks, s=sigs)
    e = dict(os.environ)
    e.update(env)
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "host_pair_helper.py"), inp, out, ROOT], env=e,
                   check=True, timeout=300)
    r = np.load(out)
    for k in ("first", "second"):
        assert (r[k] == exp).all(), (env, k, np.nonzero(r[k] != exp)[0][:10])


def test_batch_many_host_chunks(oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    rng = np.random.default_rng(82)
    m, Q, N = 6000, 67, 100
    cseeds = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    voters = np.argsort(rng.random((m, N)), axis=1)[:, :Q].reshape(-1)
    signed = np.repeat(dig, Q, axis=0)
    bad = rng.random(m * Q) < 0.01
    signed[bad, 3] ^= 1
    pks, sigs = oracle.keygen_sign_many(cseeds[voters], signed)
    offs = (np.arange(m + 1) * Q).astype(np.uint32)
    cert = ctypes.create_string_buffer((m + 7) // 8)
    badb = ctypes.create_string_buffer((m * Q + 7) // 8)
    for _ in range(2):   # first call: the launch keys join; second: steady state
        _lib.check(lib.nwc_verify_batch_many(_lib.buf(dig), _lib.buf(offs), _lib.buf(pks), _lib.buf(sigs), m, cert, badb))
        assert (_bits(badb, m * Q) == bad).all()
        assert (_bits(cert, m) == ~bad.reshape(m, Q).any(axis=1)).all()
    ocert, obad = oracle.batch_many(dig, offs, pks, sigs)
    assert (obad == bad).all() and (ocert == ~bad.reshape(m, Q).any(axis=1)).all()
    h = ctypes.c_uint32()
    _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
    assert h.value == N
    _lib.check(lib.nwc_set_committee(None, 0))


def test_batch_many_ragged_device_index(oracle):
    """Certificates of 0..130 votes (empty ones first, last and inside) at the three host-call sizes:
    packed into pinned memory, one copy (non-pipelined) and pipelined chunks.  The two larger ones
    build the vote -> certificate index on the device (k_cert_index) from the offsets; the Straus
    entry the same way.  Votes reuse a table of 100 keys x 40 digests, so any vote is cheap to make."""
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    rng = np.random.default_rng(83)
    N, D = 100, 40
    seeds = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (D, 32), dtype=np.uint8)
    pk_t, sig_t = oracle.keygen_sign_many(np.repeat(seeds, D, axis=0), np.tile(dig, (N, 1)))   # row k * D + d
    for target in (3000, 100_000, 300_000):
        m = target // 65 + 1
        counts = rng.integers(0, 131, m)
        counts[[0, m // 2, m - 1]] = 0
        offs = np.zeros(m + 1, np.uint32)
        offs[1:] = np.cumsum(counts)
        nv = int(offs[-1])
        dc = rng.integers(0, D, m)
        vote_cert = np.repeat(np.arange(m), counts)
        rows = rng.integers(0, N, nv) * D + dc[vote_cert]
        pks, sigs = pk_t[rows], sig_t[rows].copy()
        bad = rng.random(nv) < 0.01
        sigs[bad, 7] ^= 0x10
        digs = np.ascontiguousarray(dig[dc])
        exp_cert = np.bincount(vote_cert[bad], minlength=m) == 0
        if target == 3000:
            ocert, obad = oracle.batch_many(digs, offs, pks, sigs)
            assert (obad == bad).all() and (ocert == exp_cert).all()
        entries = [lib.nwc_verify_batch_many] + ([lib.nwc_verify_batch_straus_many] if target < 300_000 else [])
        for fn in entries:
            cert = ctypes.create_string_buffer((m + 7) // 8)
            badb = ctypes.create_string_buffer((nv + 7) // 8)
            _lib.check(fn(_lib.buf(digs), _lib.buf(offs), _lib.buf(pks), _lib.buf(sigs), m, cert, badb))
            assert (_bits(badb, nv) == bad).all(), (target, fn.__name__, np.nonzero(_bits(badb, nv) != bad)[0][:10])
            assert (_bits(cert, m) == exp_cert).all(), (target, fn.__name__, np.nonzero(_bits(cert, m) != exp_cert)[0][:10])
    _lib.check(lib.nwc_set_committee(None, 0))


def test_sanitize_messages_host_staged():
    """nwc_sanitize_messages on a batch above the staging threshold (4 MB of wire bytes, through the
    pinned stages): the golden wire fixtures tiled ~500 times, every code and digest as the fixture
    says (primary/src/core.rs:306-346 via the restatement, tests/golden/messages.json)."""
    _sanitize_tiled_golden()


@pytest.mark.parametrize("env", [{}, {"NWC_SIGN_DEFER": "0"}, {"NWC_STRICT_Y": "0"}])
def test_sanitize_messages_host_chunks(env):
    """The same batch in 1-MB pipelined chunks (NWC_MSG_CHUNK, read once per process: a child
    process) -- the production pipeline forced to ~8 chunks cut on 64-message boundaries, sharing
    one 64-aligned vote counter, each parsed while the previous one's leaves run on the side stream,
    with the leaves' sign tests deferred (k_verify_comb_y / k_verify_comb_y_sign / k_comb_sign) or
    decided in k_verify_comb (NWC_SIGN_DEFER=0), and the strict equations list-free on the parse
    stream (the default: an uncached author is a non-member, UnknownAuthority first) or through
    the comb path's lists on the leaf stream (NWC_STRICT_Y=0) -- codes and digests unchanged.  (Round 6 removed
    the pipeline's A/B switches that lost or tied: profiles/r05/wire_host.md.)"""
    import os
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from tests.test_gpu_host_paths import _sanitize_tiled_golden\n"
            "_sanitize_tiled_golden()\n"
            "print('done', flush=True)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, NWC_MSG_CHUNK=str(1 << 20), NWC_HOST_TIMING="1", **env))
    assert r.returncode == 0 and "done" in r.stdout, (r.returncode, r.stdout[-500:], r.stderr[-3000:])
    steps = [l for l in r.stderr.splitlines() if l.startswith("nwc sanitize steps:")]
    assert steps and all(l.count("parse queued") >= 4 for l in steps), r.stderr[-2000:]   # several chunks


def _sanitize_tiled_golden():
    import json
    import os
    from narwhal_amd import _lib
    from tests.conftest import GOLDEN
    lib = _lib.load()
    g = json.load(open(os.path.join(GOLDEN, "messages.json")))
    c = g["committee"]
    n = len(c["keys"])
    offs_w, ids = [0], []
    for w in c["workers"]:
        ids.extend(w)
        offs_w.append(len(ids))
    kb = b"".join(bytes.fromhex(k) for k in c["keys"])
    _lib.check(lib.nwc_set_committee_config(_lib.buf(kb), (ctypes.c_uint64 * n)(*c["stakes"]), n,
                                            (ctypes.c_uint32 * (n + 1))(*offs_w), (ctypes.c_uint32 * max(1, len(ids)))(*ids)))
    try:
        cases = [x for x in g["cases"] if x["gc_round"] == 0 and x["target"] is None]
        reps = 1 + (8 << 20) // sum(len(x["msg"]) // 2 for x in cases)
        tiled = cases * reps
        msgs = [bytes.fromhex(x["msg"]) for x in tiled]
        offs = np.zeros(len(msgs) + 1, np.uint64)
        offs[1:] = np.cumsum([len(b) for b in msgs])
        assert offs[-1] >= (4 << 20)
        data = b"".join(msgs)
        codes = np.zeros(len(msgs), np.int32)
        dig = np.zeros((len(msgs), 32), np.uint8)
        kinds = np.zeros(len(msgs), np.uint8)
        _lib.check(lib.nwc_sanitize_messages(_lib.buf(data), _lib.buf(offs), len(msgs), 0, None, _lib.buf(codes),
                                             _lib.buf(dig), _lib.buf(kinds)))
        for i, x in enumerate(tiled):
            assert codes[i] == x["code"], (i, x["name"], int(codes[i]))
            if x["kind"] >= 0 and x["kind"] != 3:
                assert dig[i].tobytes().hex() == x["digest"] and kinds[i] == x["kind"], (i, x["name"])
    finally:
        lib.nwc_set_committee(None, 0)


def test_process_exits_after_staged_calls():
    """A process that made staged host calls and never called nwc_shutdown (a Python or Rust caller
    that just exits) must exit cleanly: the stager's copy threads are stopped at teardown (a
    joinable std::thread destroyed at exit would call std::terminate)."""
    import os
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = ("import ctypes, sys; sys.path.insert(0, %r)\n"
            "import numpy as np\n"
            "from narwhal_amd import _lib\n"
            "lib = _lib.load()\n"
            "n = 300000\n"
            "z = np.zeros((n, 32), np.uint8); s = np.zeros((n, 64), np.uint8)\n"
            "out = ctypes.create_string_buffer((n + 7) // 8)\n"
            "_lib.check(lib.nwc_verify_strict_many(_lib.buf(z), _lib.buf(z), _lib.buf(s), n, out))\n"
            "print('done', flush=True)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, cwd=ROOT,
                       env=dict(os.environ))
    assert r.returncode == 0 and "done" in r.stdout, (r.returncode, r.stdout[-500:], r.stderr[-2000:])
