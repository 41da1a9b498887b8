// build.rs — compile the HIP engine for gfx950 and link it.
use std::{env, path::PathBuf, process::Command};
fn main() {
    let engine = PathBuf::from(env::var("COCONUT_HIP_DIR").expect("path to coconut-rust_amd"));
    let ok = Command::new("make").arg("-C").arg(&engine).arg("-j4").status().unwrap().success();
    assert!(ok, "building libcoconut_hip.so failed");
    println!("cargo:rustc-link-search=native={}", engine.display());
    println!("cargo:rustc-link-lib=dylib=coconut_hip");
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rerun-if-changed={}", engine.join("csrc").display());
}
