"""The Rust side of the drop-in boundary (integration/rust/: build.rs, src/hip.rs, src/batch.rs) checked
against the C ABI it binds (include/coconut_hip.h).  No Rust toolchain exists in this image, so the
Rust is not compiled here; what can be checked is checked: every function the header declares has
exactly one `extern "C"` declaration in src/hip.rs with the same parameter count and the Rust types
the C types map to, and nothing else is declared; every entry point src/batch.rs calls is declared."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "coconut_hip.h")
RS = os.path.join(ROOT, "integration", "rust", "src")

# C type (whitespace-normalised) -> Rust FFI type
C2R = {
    "int": "c_int", "cc_status": "c_int", "cc_group_mode": "c_int", "size_t": "usize", "uint64_t": "u64",
    "const char*": "*const c_char", "const uint8_t*": "*const u8", "uint8_t*": "*mut u8",
    "const uint32_t*": "*const u32", "uint32_t*": "*mut u32", "const uint64_t*": "*const u64",
    "const int32_t*": "*const i32", "int32_t*": "*mut i32", "int*": "*mut c_int", "float*": "*mut f32",
    "void*": "*mut c_void", "cc_ctx*": "*mut CcCtx", "const cc_ctx*": "*const CcCtx", "cc_ctx**": "*mut *mut CcCtx",
}


def _c_decls():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"^\s*((?:const\s+)?[a-z_0-9]+\s*\*?)\s*(cc_\w+)\(([^;{]*?)\);", src, flags=re.M | re.S):
        params = [] if args.strip() == "void" else [a.strip() for a in args.split(",")]
        types = []
        for p in params:
            p = re.sub(r"\s+", " ", p)
            m = re.match(r"(.*?[\s*])(\w+)$", p)
            types.append(re.sub(r"\s*\*", "*", m.group(1).strip()))
        out[name] = (re.sub(r"\s*\*", "*", ret.strip()), types)
    return out


def _rust_decls():
    src = open(os.path.join(RS, "hip.rs")).read()
    block = src[src.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    block = re.sub(r"//[^\n]*", "", block)
    out = {}
    for name, args, ret in re.findall(r"pub fn (cc_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        params = [a.strip() for a in args.split(",") if a.strip()]
        out.setdefault(name, []).append(([re.sub(r"\s+", " ", p.split(":", 1)[1].strip()) for p in params],
                                         (ret or "()").strip()))
    return out


def test_every_header_function_is_declared_once_with_matching_types():
    c, r = _c_decls(), _rust_decls()
    assert len(c) >= 38, sorted(c)
    assert set(c) == set(r), (sorted(set(c) - set(r)), sorted(set(r) - set(c)))
    for name, (cret, ctypes_) in c.items():
        assert len(r[name]) == 1, name
        rtypes, rret = r[name][0]
        assert len(rtypes) == len(ctypes_), (name, ctypes_, rtypes)
        for ct, rt in zip(ctypes_, rtypes):
            assert C2R[ct] == rt, (name, ct, rt)
        assert C2R[cret] == rret, (name, cret, rret)


def test_batch_shim_calls_only_declared_entry_points():
    declared = set(_rust_decls())
    called = set(re.findall(r"\b(cc_\w+)\(", open(os.path.join(RS, "batch.rs")).read()))
    assert called and called <= declared, sorted(called - declared)
    for f in ("cc_verify_batch", "cc_signature_aggregate_batch", "cc_verkey_aggregate_batch", "cc_pok_verify_batch"):
        assert f in called, f


def test_build_script_builds_and_links_the_engine():
    b = open(os.path.join(ROOT, "integration", "rust", "build.rs")).read()
    assert "COCONUT_HIP_DIR" in b and "rustc-link-lib=dylib=coconut_hip" in b and "make" in b
    mk = open(os.path.join(ROOT, "coconut-rust_amd", "Makefile")).read()
    assert "--offload-arch=$(ARCH)" in mk and "ARCH ?= gfx950" in mk and "libcoconut_hip.so" in mk


def _fn_body(src, name):
    i = src.index(f"fn {name}(")
    j = src.find("\n    pub fn ", i + 1)
    k = src.find("\npub fn ", i + 1)
    ends = [e for e in (j, k) if e > 0]
    return src[i:min(ends) if ends else len(src)]


def test_safe_wrappers_guard_every_length_the_c_side_reads():
    """the safe wrappers must assert, before the unsafe call, every length the C ABI derives
    its reads from (else a shorter Vec is a heap over-read reachable from safe code)."""
    b = open(os.path.join(RS, "batch.rs")).read()
    h = open(os.path.join(RS, "hip.rs")).read()
    need = {
        "verify_batch": ["messages.len(), sigs.len()", "m.len() == q"],
        "aggregate_batch": ["b.len() == len", "len >= threshold"],
        "new_batch": ["r.ciphertexts.len() == k", "r.known_messages.len() == q - k", "cm.len(), n * sb"],
        "verify_shares_batch": ["set_of.len() == ids.len()", "shares.len() == ids.len()", "s.len() == t",
                                "(k as usize) < sets.len()"],
        "pok_verify_batch": ["chal.len(), n", "revealed_msgs.len() == n", "m.len() == r", "p.4.len() == nresp",
                             "p.0.len() == sb", "p.2.len() == ob", "p.3.len() == ob"],
    }
    for fn, guards in need.items():
        bodies = [_fn_body(b, fn)] if fn != "aggregate_batch" else \
            [b[m.start():] for m in re.finditer(r"fn aggregate_batch\(", b)]
        for body in bodies:
            body = body[:body.index("unsafe")]  # the guards come before the FFI call
            for g in guards:
                assert g in body, (fn, g)
    assert "x.len() == ob && y.len() == q * ob" in _fn_body(h, "set_verkey")
    assert "g_tilde.len(), self.oth_bytes()" in _fn_body(h, "set_params")


def test_single_credential_stays_on_the_reference_cpu_path():
    """one Signature::verify through the engine (~2.1 ms) is not faster than the
    reference's own CPU verify on one thread (~1.9 ms), so below GPU_MIN_BATCH the shim calls the
    reference's verify (signature.rs:473) and only batches reach cc_verify_batch."""
    b = open(os.path.join(RS, "batch.rs")).read()
    m = re.search(r"pub const GPU_MIN_BATCH: usize = (\d+);", b)
    assert m and int(m.group(1)) == 2
    body = _fn_body(b, "verify_batch")
    cut = body.index("if sigs.len() < GPU_MIN_BATCH")
    assert cut < body.index("cc_verify_batch(")
    assert ".verify(m, vk, params)" in body[cut:body.index("cc_verify_batch(")]
