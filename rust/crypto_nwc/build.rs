// Builds libnwc.so for gfx950 with hipcc and links it into the crate.
// NWC_SRC points at this repository (default: two levels up from this crate).
use std::{env, path::PathBuf, process::Command};

fn main() {
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src = env::var("NWC_SRC").map(PathBuf::from).unwrap_or_else(|_| manifest.join("../.."));
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let status = Command::new(&hipcc)
        .args(&["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-shared"])
        .arg(format!("-I{}", src.join("include").display()))
        .arg(format!("-I{}", src.join("narwhal_amd/csrc").display()))
        .arg("-o")
        .arg(out.join("libnwc.so"))
        .arg(src.join("narwhal_amd/csrc/nwc_api.hip"))
        .status()
        .expect("running hipcc");
    assert!(status.success(), "hipcc failed building libnwc.so");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=nwc");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
    println!("cargo:rerun-if-changed={}", src.join("narwhal_amd/csrc").display());
    println!("cargo:rerun-if-changed={}", src.join("include/nwc.h").display());
}
