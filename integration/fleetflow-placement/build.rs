//! Builds libfleetplace.so for gfx950 by running fleetflow_amd/csrc/Makefile itself -- objects and
//! library under OUT_DIR -- so the crate links the library the bench measures: the same sources,
//! translation units (fp_pipe.hip with -DFPP_SPLIT_BIG, fp_pipe_big.hip under its own LLVM machine
//! scheduler) and flags, with no second copy of the recipe to drift.  Or links a prebuilt one.
//!
//!   FLEETPLACE_LIB_DIR=/path/with/libfleetplace.so   use a prebuilt library
//!   FLEETPLACE_SRC=/path/to/fleetflow_amd/csrc       HIP sources + Makefile (default: ../../fleetflow_amd/csrc)
//!   HIPCC=/opt/rocm/bin/hipcc                         compiler (default: the Makefile's)
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    println!("cargo:rerun-if-env-changed=FLEETPLACE_LIB_DIR");
    println!("cargo:rerun-if-env-changed=FLEETPLACE_SRC");
    println!("cargo:rerun-if-env-changed=HIPCC");
    if let Ok(dir) = env::var("FLEETPLACE_LIB_DIR") {
        println!("cargo:rustc-link-search=native={dir}");
        println!("cargo:rustc-link-lib=dylib=fleetplace");
        println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
        return;
    }
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src = env::var("FLEETPLACE_SRC")
        .map(PathBuf::from)
        .unwrap_or_else(|_| manifest.join("../../fleetflow_amd/csrc"));
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    // a directory: cargo re-runs the script when any file under it changes (every source, header
    // and the Makefile), and the header the sources include
    println!("cargo:rerun-if-changed={}", src.display());
    println!("cargo:rerun-if-changed={}", src.join("../../include/fleetplace.h").display());
    let mut cmd = Command::new("make");
    cmd.arg("-C").arg(&src)
        .arg(format!("BUILD={}", out.join("obj").display()))
        .arg(format!("OUT={}", out.join("libfleetplace.so").display()))
        .arg("-j8");
    if let Ok(hipcc) = env::var("HIPCC") {
        cmd.arg(format!("HIPCC={hipcc}"));
    }
    let status = cmd.status().unwrap_or_else(|e| panic!("cannot run make: {e} (set FLEETPLACE_LIB_DIR to a prebuilt libfleetplace.so)"));
    assert!(status.success(), "make failed building libfleetplace.so");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=fleetplace");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
}
