// Links libzkm_hip.so the way crates/core/machine/build.rs links its native row library: a search
// path from the environment, a `links` key in Cargo.toml, rerun when the header changes.
fn main() {
    let dir = std::env::var("ZKM_HIP_LIB_DIR").expect("set ZKM_HIP_LIB_DIR to the directory of libzkm_hip.so");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=zkm_hip");
    println!("cargo:rerun-if-env-changed=ZKM_HIP_LIB_DIR");
    println!("cargo:rerun-if-changed={dir}/../include/zkm_hip.h");
}
