//! Links libquack_hip.so (built by `make -C sidekick_amd/csrc`, gfx950).
//! QUACK_HIP_LIB_DIR overrides the directory; the default is the library's
//! in-tree location relative to this crate (rust/quack -> sidekick_amd/).
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = match env::var("QUACK_HIP_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../sidekick_amd"),
    };
    let dir = dir.canonicalize().unwrap_or(dir);
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=quack_hip");
    // the library runs from its build directory unless installed elsewhere
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rerun-if-env-changed=QUACK_HIP_LIB_DIR");
    println!("cargo:rerun-if-changed=../../include/quack_hip.h");
}
