// Link libmassrt.so (built by `make -C mass-raytrace_amd`). MASSRT_LIB_DIR
// overrides the default in-tree location.
fn main() {
    let dir = std::env::var("MASSRT_LIB_DIR").unwrap_or_else(|_| {
        format!("{}/../../mass-raytrace_amd/massrt", env!("CARGO_MANIFEST_DIR"))
    });
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=massrt");
    println!("cargo:rerun-if-env-changed=MASSRT_LIB_DIR");
}
