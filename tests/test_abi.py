"""The C-ABI library loads and exports every symbol include/nwc.h declares (CPU only: no
device compute is called here)."""
import ctypes
import os
import re
import subprocess

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "nwc.h")
LIB = os.path.join(ROOT, "narwhal_amd", "libnwc.so")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(nwc_[a-z0-9_]+)\s*\(", text)))


def test_library_built():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 18
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_ctypes_bindings_cover_header():
    from narwhal_amd import _lib
    assert set(declared_symbols()) == set(_lib._SIGS), set(declared_symbols()) ^ set(_lib._SIGS)


def test_calls_without_init_fail_loudly():
    """Before nwc_init every entry point returns NWC_ERR_NOT_INIT (< 0) -- never a verdict."""
    from narwhal_amd import _lib
    lib = _lib.load(init=False)
    assert lib.nwc_version() >> 16 == 1
    if lib.nwc_device_count() == 0:
        z = bytes(64)
        p = _lib.buf(z)
        assert lib.nwc_verify_strict(p, p, p) == _lib.NWC_ERR_NOT_INIT
        assert lib.nwc_verify_batch(p, p, p, 1, None) == _lib.NWC_ERR_NOT_INIT
        assert b"nwc_init" in lib.nwc_last_error()


def test_build_id_matches_sources():
    """libnwc.so embeds the hash of the sources it was compiled from (narwhal_amd/build.py), and
    build() recompiles whenever they differ: the in-tree library is this tree's."""
    from narwhal_amd import _lib, build
    lib = _lib.load(init=False)
    assert lib.nwc_build_id().decode() == build.source_id() == build.embedded_id()
    assert build.up_to_date()


def test_diag_set_rejects_bad_knobs_without_a_device():
    from narwhal_amd import _lib
    lib = _lib.load(init=False)
    assert lib.nwc_diag_set(b"no_such_knob", 1) == _lib.NWC_ERR_ARG
    assert lib.nwc_diag_set(b"straus_nq", 0) == _lib.NWC_ERR_ARG
    assert lib.nwc_diag_set(b"straus_nq", 17) == _lib.NWC_ERR_ARG
    assert lib.nwc_diag_set(b"force_windows", 32) == _lib.NWC_ERR_ARG
    assert lib.nwc_diag_set(b"straus_nq", 12) == 0 and lib.nwc_diag_set(b"force_windows", 0) == 0


def test_gfx950_code_object_present():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", LIB], capture_output=True, text=True).stdout
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob
