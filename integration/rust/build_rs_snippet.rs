// Two lines for the reference's build.rs (it already has one): link the engine built
// in-tree by `make -C two-pass-lanczos_amd/csrc` (or __graft_entry__.build()).
// TPL_AMD_DIR = the root of this repository.
println!("cargo:rustc-link-search=native={}/two-pass-lanczos_amd/tpl_amd", env!("TPL_AMD_DIR"));
println!("cargo:rustc-link-lib=dylib=tpl_amd");
