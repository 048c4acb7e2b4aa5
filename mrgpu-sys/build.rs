// Links libmrgpu.so.  MRGPU_LIB_DIR overrides the location (default: the in-tree build output of
// `make -C mapreduce_rust_amd/csrc`); the rpath lets the worker binary find it without LD_LIBRARY_PATH.
fn main() {
    let dir = std::env::var("MRGPU_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{here}/../mapreduce_rust_amd/lib")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=mrgpu");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=MRGPU_LIB_DIR");
    println!("cargo:rerun-if-changed=../include/mrgpu.h");
}
