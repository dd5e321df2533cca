"""Builds libnwc.so for gfx950 in-tree (hipcc cross-compiles; no GPU needed).

    python -m narwhal_amd.build            # incremental
    python -m narwhal_amd.build --force
    python narwhal_amd/build.py --hipcc-args OUT   # the argument list (rust/crypto_nwc/build.rs)
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libnwc.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-shared",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                  [os.path.join(ROOT, "include", "nwc.h")])


def source_id() -> str:
    """Hash of the library's sources (contents and tree-relative names) and compile flags: the build
    id libnwc.so embeds (nwc_build_id) and smoke() / tests check against the tree they run from."""
    h = hashlib.sha256(" ".join(f for f in FLAGS if not f.startswith("-I")).encode())
    for s in sources():
        h.update(os.path.relpath(s, ROOT).encode() + b"\0")
        with open(s, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:20]


def embedded_id(path: str = OUT):
    """The build id a built library carries ("NWC_BUILD_ID:<id>" in its bytes), or None."""
    try:
        blob = open(path, "rb").read()
    except OSError:
        return None
    i = blob.find(b"NWC_BUILD_ID:")
    if i < 0:
        return None
    j = blob.find(b"\0", i)
    return blob[i + 13:j].decode(errors="replace")


def up_to_date() -> bool:
    """The in-tree library is current iff it embeds the hash of the present sources (not by
    mtime: a copied tree keeps the .so but not the timestamps' meaning)."""
    return os.path.exists(OUT) and embedded_id(OUT) == source_id()


def hipcc_args(out: str) -> list:
    """The whole hipcc argument list of libnwc.so (flags, the build id, output, source): the one
    recipe both this script and the Rust shim's build.rs (`build.py --hipcc-args OUT`) compile
    with, so a cargo-built library carries the same nwc_build_id as an in-tree one."""
    return FLAGS + ['-DNWC_BUILD_ID="%s"' % source_id(), "-o", out, os.path.join(CSRC, "nwc_api.hip")]


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC] + hipcc_args(OUT + ".tmp")
    if verbose:
        print("[narwhal_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    if "--hipcc-args" in sys.argv:
        # rust/crypto_nwc/build.rs: one argument per line
        print("\n".join(hipcc_args(sys.argv[sys.argv.index("--hipcc-args") + 1])))
    elif "--source-id" in sys.argv:
        print(source_id())
    else:
        build(force="--force" in sys.argv)
