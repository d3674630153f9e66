"""The hbbft-hip Rust crate ("a new hbbft-hip backend crate ...
built by build.rs with hipcc").  No Rust toolchain exists in this image, so
the crate is checked, not compiled: src/ffi.rs is what gen_ffi.py generates
from include/hbrbc.h, every `extern "C"` it declares exists in the header
with the same arity and in the built libhbrbc.so, the facade in src/lib.rs
calls only declared functions, and the Rust shown in INTEGRATION.md is the
crate's own text."""
import ctypes
import importlib.util
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = os.path.join(ROOT, "hbbft-hip")


def _gen():
    spec = importlib.util.spec_from_file_location("gen_ffi", os.path.join(CRATE, "gen_ffi.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _rust_fns(text):
    """{name: [parameter strings]} of every `pub fn hbrbc_*` in an extern block."""
    out = {}
    for m in re.finditer(r"pub fn (hbrbc_\w+)\((.*?)\)", text):
        params = [p.strip() for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = params
    return out


def test_ffi_rs_is_generated_from_the_header():
    committed = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    assert committed == _gen().generate(), "regenerate: python hbbft-hip/gen_ffi.py > hbbft-hip/src/ffi.rs"


def test_every_extern_matches_the_header_and_the_library():
    g = _gen()
    hdr = {name: params for _, name, params in g.c_functions(open(os.path.join(ROOT, "include", "hbrbc.h")).read())}
    rs = _rust_fns(open(os.path.join(CRATE, "src", "ffi.rs")).read())
    assert set(rs) == set(hdr)
    for name, params in rs.items():
        assert len(params) == len(hdr[name]), name
        # parameter names kept (a renamed one would hint at a reordering)
        for rp, cp in zip(params, hdr[name]):
            cname = re.match(r".*?(\w+)(\s*\[\d+\])?$", cp).group(1)
            assert rp.split(":")[0].rstrip("_") == cname, (name, rp, cp)
    lib_path = os.path.join(ROOT, "hbbft_amd", "libhbrbc.so")
    if not os.path.exists(lib_path):
        pytest.skip("libhbrbc.so not built")
    L = ctypes.CDLL(lib_path)
    for name in rs:
        assert hasattr(L, name), name


def test_sm_args_layouts_agree():
    """HbrbcSmArgs (Rust), hbrbc_sm_args (C) and rbc_sim.SmArgs (ctypes): same
    fields in the same order."""
    from hbbft_amd.rbc_sim import SmArgs
    g = _gen()
    hdr = open(os.path.join(ROOT, "include", "hbrbc.h")).read()
    c_fields = [n for n, _ in g.struct_fields(hdr, "hbrbc_sm_args")]
    rs = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    body = re.search(r"pub struct HbrbcSmArgs \{(.*?)\}", rs, flags=re.S).group(1)
    rs_fields = [m.group(1).rstrip("_") for m in re.finditer(r"pub (\w+):", body)]
    py_fields = [n.rstrip("_") for n, _ in SmArgs._fields_]
    assert c_fields == rs_fields == py_fields


def test_facade_calls_declared_functions_only():
    rs = _rust_fns(open(os.path.join(CRATE, "src", "ffi.rs")).read())
    lib_rs = open(os.path.join(CRATE, "src", "lib.rs")).read()
    used = set(re.findall(r"ffi::(hbrbc_\w+)", lib_rs))
    assert used and used <= set(rs), used - set(rs)
    build = open(os.path.join(CRATE, "build.rs")).read()
    assert "hipcc" in build and "rustc-link-lib=dylib=hbrbc" in build
    toml = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'name = "hbbft-hip"' in toml and 'build = "build.rs"' in toml


def test_integration_md_quotes_the_crate():
    """Every fenced block of INTEGRATION.md whose first line is
    `// hbbft-hip/<path>` is a verbatim excerpt of that file."""
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```rust\n// (hbbft-hip/[\w./]+)\n(.*?)```", md, flags=re.S)
    assert len(blocks) >= 3
    for path, body in blocks:
        text = open(os.path.join(ROOT, path)).read()
        assert body.strip() in text, path
