"""The Rust shim (rust/crypto_nwc) declares exactly the C ABI of include/nwc.h.

There is no cargo in this image, so the crate is not compiled here; this test checks mechanically
that its `extern "C"` block has every header entry point, with the same parameter count and
types in the same order and the same return type, so the binding cannot drift from the ABI.
"""
import os
import re

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "nwc.h")
FFI = os.path.join(ROOT, "rust", "crypto_nwc", "src", "ffi.rs")

# C parameter type -> Rust FFI type
C2RUST = {
    "const uint8_t*": "*const u8", "uint8_t*": "*mut u8", "const uint32_t*": "*const u32",
    "const uint64_t*": "*const u64", "uint64_t*": "*mut u64", "uint32_t*": "*mut u32", "int32_t*": "*mut i32", "double*": "*mut f64",
    "const void*": "*const c_void", "void*": "*mut c_void", "const char*": "*const c_char",
    "nwc_digester*": "*mut nwc_digester", "nwc_memory*": "*mut nwc_memory", "int64_t": "i64", "size_t*": "*mut usize", "size_t": "usize", "uint32_t": "u32", "uint64_t": "u64", "int": "c_int", "void": None,
}


def _c_param_type(p: str) -> str:
    p = " ".join(p.split())
    m = re.match(r"(const )?(\w+)\s*(\*?)\s*(\w+)(\[\d+\])?$", p)
    assert m, p
    const, base, star, _, arr = m.groups()
    if arr:   # `const uint8_t msg32[32]` decays to a pointer
        star = "*"
    return ("const " if const else "") + base + star


def c_decls():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w ]*?[\s\*]+)(nwc_\w+)\s*\(([^)]*)\)\s*;", text):
        ret = " ".join(m.group(1).split()).replace(" *", "*")
        args = [a for a in m.group(3).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(2)] = (C2RUST[ret], [C2RUST[_c_param_type(a)] for a in args])
    return out


def rust_decls():
    text = open(FFI).read()
    block = text[text.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (nwc_\w+)\s*\(([^)]*)\)\s*(->\s*([^;]+))?;", block):
        args = [a.split(":", 1)[1].strip() for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = (m.group(4).strip() if m.group(4) else None, args)
    return out


def test_every_header_function_is_declared_identically():
    c, r = c_decls(), rust_decls()
    assert len(c) >= 24
    assert set(c) == set(r), set(c) ^ set(r)
    for name, sig in c.items():
        assert r[name] == sig, (name, sig, r[name])


def test_build_rs_compiles_with_the_shared_recipe_and_id():
    """build.rs takes hipcc's whole argument list from narwhal_amd/build.py --hipcc-args (one
    recipe), whose list carries -DNWC_BUILD_ID=<source_id>: a cargo-built library reports the same
    build id as the in-tree one (crypto_nwc::build_id), so the provenance check reaches Rust."""
    import subprocess
    import sys
    from narwhal_amd import build as nb
    rs = open(os.path.join(ROOT, "rust", "crypto_nwc", "build.rs")).read()
    assert 'arg(src.join("narwhal_amd/build.py"))' in rs and '.arg("--hipcc-args")' in rs
    assert "Command::new(&hipcc).args(&args)" in rs and "-DNWC_BUILD_ID=" in rs
    lib = open(os.path.join(ROOT, "rust", "crypto_nwc", "src", "lib.rs")).read()
    assert "pub fn build_id() -> String" in lib and "nwc_build_id()" in lib
    out = subprocess.run([sys.executable, os.path.join(ROOT, "narwhal_amd", "build.py"), "--hipcc-args", "/x/libnwc.so"],
                         capture_output=True, text=True, check=True).stdout.splitlines()
    assert out == nb.hipcc_args("/x/libnwc.so")
    assert '-DNWC_BUILD_ID="%s"' % nb.source_id() in out
    # the in-tree build compiles with exactly this list (build.py: [HIPCC] + hipcc_args(...))
    assert "[HIPCC] + hipcc_args(" in open(os.path.join(ROOT, "narwhal_amd", "build.py")).read()


def test_crate_files_present():
    for f in ("Cargo.toml", "build.rs", "src/lib.rs", "src/ffi.rs"):
        assert os.path.exists(os.path.join(ROOT, "rust", "crypto_nwc", f)), f
    lib = open(os.path.join(ROOT, "rust", "crypto_nwc", "src", "lib.rs")).read()
    for fn in ("pub fn verify_strict", "pub fn verify_batch", "pub fn digest32", "pub fn set_committee"):
        assert fn in lib
