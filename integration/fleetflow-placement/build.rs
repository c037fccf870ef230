//! Builds libfleetplace.so with hipcc for gfx950 (the same recipe as
//! fleetflow_amd/csrc/Makefile), or links a prebuilt one.
//!
//!   FLEETPLACE_LIB_DIR=/path/with/libfleetplace.so   use a prebuilt library
//!   FLEETPLACE_SRC=/path/to/fleetflow_amd/csrc       HIP sources (default: ../../fleetflow_amd/csrc)
//!   HIPCC=/opt/rocm/bin/hipcc                         compiler (default)
use std::env;
use std::path::PathBuf;
use std::process::Command;

const SOURCES: [&str; 7] = [
    "fp_ctx.hip", "fp_place.hip", "fp_pipe.hip", "fp_order.hip", "fp_feas.hip", "fp_gen.hip", "fp_small.hip",
];

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
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".to_string());
    let mut cmd = Command::new(&hipcc);
    cmd.args(["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics", "-o"])
        .arg(out.join("libfleetplace.so"));
    for s in SOURCES {
        let p = src.join(s);
        println!("cargo:rerun-if-changed={}", p.display());
        cmd.arg(p);
    }
    for h in ["fp_internal.h", "fp_pipe_asm.h", "fp_pipe_sys.h", "fp_pipe_sysv.h", "fp_small.h", "../../include/fleetplace.h"] {
        println!("cargo:rerun-if-changed={}", src.join(h).display());
    }
    let status = cmd.status().unwrap_or_else(|e| panic!("cannot run {hipcc}: {e} (set FLEETPLACE_LIB_DIR to a prebuilt libfleetplace.so)"));
    assert!(status.success(), "hipcc failed building libfleetplace.so");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=fleetplace");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
}
