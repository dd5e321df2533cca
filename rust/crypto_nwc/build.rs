// Builds libnwc.so for gfx950 with hipcc and links it into the crate.
// NWC_SRC points at this repository (default: two levels up from this crate).
//
// The hipcc argument list -- flags, -DNWC_BUILD_ID="<hash of the sources and flags>", output and
// source -- comes from the repository's own recipe (`python3 narwhal_amd/build.py --hipcc-args
// OUT`), so the library cargo builds reports the same nwc_build_id() (crypto_nwc::build_id()) as
// the in-tree build of the same sources, and the provenance check reaches the Rust path.
use std::{env, path::PathBuf, process::Command};

fn main() {
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src = env::var("NWC_SRC").map(PathBuf::from).unwrap_or_else(|_| manifest.join("../.."));
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let python = env::var("PYTHON").unwrap_or_else(|_| "python3".into());
    let lib = out.join("libnwc.so");
    let recipe = Command::new(&python)
        .arg(src.join("narwhal_amd/build.py"))
        .arg("--hipcc-args")
        .arg(&lib)
        .output()
        .expect("running narwhal_amd/build.py --hipcc-args (the shared build recipe)");
    assert!(recipe.status.success(), "narwhal_amd/build.py --hipcc-args failed");
    let args: Vec<String> = String::from_utf8(recipe.stdout)
        .expect("utf-8 argument list")
        .lines()
        .map(str::to_owned)
        .collect();
    assert!(args.iter().any(|a| a.starts_with("-DNWC_BUILD_ID=")), "the recipe carries the build id");
    let status = Command::new(&hipcc).args(&args).status().expect("running hipcc");
    assert!(status.success(), "hipcc failed building libnwc.so");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=nwc");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
    println!("cargo:rerun-if-changed={}", src.join("narwhal_amd/csrc").display());
    println!("cargo:rerun-if-changed={}", src.join("narwhal_amd/build.py").display());
    println!("cargo:rerun-if-changed={}", src.join("include/nwc.h").display());
}
