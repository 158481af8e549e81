// Link libtapeec.so: TAPEEC_LIB_DIR names the directory holding it (the repo's tape_amd/ after
// `make -C tape_amd`, or an install prefix).  The library needs the ROCm runtime at run time.
fn main() {
    let dir = std::env::var("TAPEEC_LIB_DIR").unwrap_or_else(|_| "/opt/tapeec/lib".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=tapeec");
    println!("cargo:rerun-if-env-changed=TAPEEC_LIB_DIR");
}
