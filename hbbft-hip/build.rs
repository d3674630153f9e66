//! Builds libhbrbc.so with hipcc for gfx950 (hbbft_amd/csrc/Makefile: kernels,
//! C ABI, hiprtc specialiser, pairing and state-machine kernels) and links it.
//! HBRBC_LIB_DIR=<dir holding libhbrbc.so> links a prebuilt library instead
//! (e.g. the one __graft_entry__.build() produced, with its jit/ code objects).
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    println!("cargo:rerun-if-env-changed=HBRBC_LIB_DIR");
    println!("cargo:rerun-if-env-changed=HIPCC");
    let lib_dir = match env::var("HBRBC_LIB_DIR") {
        Ok(dir) => PathBuf::from(dir),
        Err(_) => {
            let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
            let root = manifest.parent().expect("hbbft-hip sits beside hbbft_amd/").to_path_buf();
            let csrc = root.join("hbbft_amd").join("csrc");
            for f in &["kernels.hip", "api.hip", "jit.hip", "wire.hip", "pairing.hip", "sim.hip",
                       "version.cpp", "device_common.hpp", "launchers.hpp", "jit.hpp",
                       "bls_consts.hpp", "Makefile"] {
                println!("cargo:rerun-if-changed={}", csrc.join(f).display());
            }
            println!("cargo:rerun-if-changed={}", root.join("include").join("hbrbc.h").display());
            // hipcc --offload-arch=gfx950 (no CUDA shims, no dual code paths)
            let mut make = Command::new("make");
            make.arg("-s").arg("-C").arg(&csrc);
            if let Ok(hipcc) = env::var("HIPCC") {
                make.arg(format!("HIPCC={}", hipcc));
            }
            let status = make.status().expect("running make (hipcc) for libhbrbc.so");
            assert!(status.success(), "building libhbrbc.so with hipcc failed");
            root.join("hbbft_amd")
        }
    };
    println!("cargo:rustc-link-search=native={}", lib_dir.display());
    println!("cargo:rustc-link-lib=dylib=hbrbc");
    // the specialised encoders / decoders are found beside the library (jit/)
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib_dir.display());
}
