"""The Rust side of the drop-in boundary ("the Rust shim exists only as
prose"): rust/tapeec-sys/src/lib.rs is generated from include/tape_ec.h by
scripts/gen_rust_sys.py and must be current; it declares every exported entry point, and its
structs carry the same fields as the header (and as the ctypes mirror the tests run through).
No Rust toolchain exists in this image, so the crates are not compiled here."""
import os
import re
import subprocess
import sys

from tape_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RS = os.path.join(ROOT, "rust", "tapeec-sys", "src", "lib.rs")


def test_generated_binding_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gen_rust_sys.py"), "--check"])
    assert r.returncode == 0, "rust/tapeec-sys/src/lib.rs is stale: run scripts/gen_rust_sys.py"


def test_binding_declares_every_export():
    rs = open(RS).read()
    assert set(re.findall(r"pub fn (te_\w+)", rs)) == set(_lib.declared_symbols())


def test_struct_fields_match_ctypes_mirror():
    rs = open(RS).read()
    for name in ("te_clay_info", "te_slice_metadata", "te_slicer_cfg", "te_geometry", "te_repair_plan_info",
                 "te_object", "te_decode_object", "te_recover_object", "te_repair_object"):
        body = re.search(r"pub struct %s \{(.*?)\n\}" % name, rs, flags=re.S).group(1)
        fields = re.findall(r"pub (\w+):", body)
        mirror = [f[0] for f in getattr(_lib, name)._fields_]
        assert fields == mirror, (name, fields, mirror)


def test_pointer_constness():
    rs = open(RS).read()
    assert "pub fn te_clay_decode(c: *mut te_clay, chunks: *const *const u8," in rs
    assert "coders: *const *mut te_clay" in rs
    assert "pub fn te_clay_new(n: u32, k: u32, d: u32, out: *mut *mut te_clay) -> c_int;" in rs
