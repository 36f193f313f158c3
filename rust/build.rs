// build.rs -- for `cargo build --features hip`: builds libssbls.so (the MI355X threshold-BLS engine)
// with hipcc for gfx950 and links it into the dvf crate (src/crypto/impls/hip.rs).  Without the
// feature it does nothing, so the blst build is unchanged.
//
//   SSBLS_DIR      checkout of the engine repository: its csrc/*.hip are compiled here, exactly the
//                  line of safestakeoperator_amd/build.py (hipcc --offload-arch=gfx950 -O3 -fPIC)
//   SSBLS_LIB_DIR  or: a directory holding a prebuilt libssbls.so (no hipcc needed)
//   ROCM_PATH      default /opt/rocm
use std::env;
use std::path::PathBuf;
use std::process::Command;

// the translation units of libssbls.so (safestakeoperator_amd/build.py SOURCES)
const SOURCES: &[&str] = &[
    "ssbls.hip", "ssb_k_lane.hip", "ssb_k_verify.hip", "ssb_k_pair.hip", "ssb_k_hash.hip", "ssb_k_combine.hip",
    "ssb_k_msm.hip", "ssb_k_bisect.hip", "ssb_k_wire.hip", "ssb_k_dkg.hip", "ssb_k_fused.hip", "ssb_collector.hip",
];

fn main() {
    println!("cargo:rerun-if-changed=build.rs");
    println!("cargo:rerun-if-env-changed=SSBLS_DIR");
    println!("cargo:rerun-if-env-changed=SSBLS_LIB_DIR");
    println!("cargo:rerun-if-env-changed=ROCM_PATH");
    if env::var_os("CARGO_FEATURE_HIP").is_none() {
        return;
    }
    let rocm = PathBuf::from(env::var("ROCM_PATH").unwrap_or_else(|_| String::from("/opt/rocm")));
    let lib_dir = match env::var_os("SSBLS_LIB_DIR") {
        Some(d) => PathBuf::from(d),
        None => {
            let src = PathBuf::from(env::var_os("SSBLS_DIR").expect(
                "--features hip: set SSBLS_DIR (engine checkout, compiled with hipcc) or SSBLS_LIB_DIR (prebuilt libssbls.so)",
            ));
            let csrc = src.join("safestakeoperator_amd").join("csrc");
            let out = PathBuf::from(env::var_os("OUT_DIR").unwrap());
            let hipcc = rocm.join("bin").join("hipcc");
            let mut objs = Vec::new();
            for s in SOURCES {
                let file = csrc.join(s);
                println!("cargo:rerun-if-changed={}", file.display());
                let obj = out.join(s.replace(".hip", ".o"));
                let st = Command::new(&hipcc)
                    .args(["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-unused-value", "-c", "-o"])
                    .arg(&obj)
                    .arg(&file)
                    .status()
                    .expect("hipcc not found (ROCM_PATH)");
                assert!(st.success(), "hipcc failed on {}", file.display());
                objs.push(obj);
            }
            let lib = out.join("libssbls.so");
            let st = Command::new(&hipcc)
                .args(["--offload-arch=gfx950", "-shared", "-fPIC", "-o"])
                .arg(&lib)
                .args(&objs)
                .status()
                .expect("hipcc not found (ROCM_PATH)");
            assert!(st.success(), "linking libssbls.so failed");
            out
        }
    };
    println!("cargo:rustc-link-search=native={}", lib_dir.display());
    println!("cargo:rustc-link-lib=dylib=ssbls");
    println!("cargo:rustc-link-search=native={}", rocm.join("lib").display());
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    // test and binary targets find the library at run time without LD_LIBRARY_PATH
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib_dir.display());
}
