// src/hip.rs — the extern "C" layer over libcoconut_hip.so (include/coconut_hip.h), one declaration
// per entry point of the header, in the header's order.  A maintainer adds `pub mod hip;` and
// `pub mod batch;` to src/lib.rs (reference src/lib.rs:26-31 lists the crate's modules) and
// `build = "build.rs"` to Cargo.toml (Cargo.toml.fragment).  Not compiled here (no Rust toolchain in
// this image); tests/test_rust_binding.py checks every declaration against the C header.
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)] pub struct CcCtx { _p: [u8; 0] }
pub const CC_SIG_G2: c_int = 0;   // reference default feature (lib.rs:3-4)
pub const CC_SIG_G1: c_int = 1;
// argument ceilings (coconut_hip.h CC_MAX_*): a larger count is CC_ERR_DECODE
pub const CC_MAX_BATCH: usize = 1 << 26;
pub const CC_MAX_IDS: usize = 1 << 16;
pub const CC_MAX_Q: usize = 4096;
pub const CC_MAX_PARTS: usize = 1 << 16;

extern "C" {
    pub fn cc_status_str(status: c_int) -> *const c_char;
    pub fn cc_version() -> *const c_char;
    // contexts: one per calling thread; a device set spans GPUs (RCCL communicators inside)
    pub fn cc_ctx_create(device: c_int, mode: c_int, out: *mut *mut CcCtx) -> c_int;
    pub fn cc_ctx_create_multi(device_mask: u64, mode: c_int, out: *mut *mut CcCtx) -> c_int;
    pub fn cc_ctx_num_devices(ctx: *const CcCtx, ndev: *mut c_int) -> c_int;
    pub fn cc_ctx_destroy(ctx: *mut CcCtx) -> c_int;
    pub fn cc_ctx_mode(ctx: *const CcCtx, mode_out: *mut c_int) -> c_int;
    pub fn cc_set_params(ctx: *mut CcCtx, g_tilde: *const u8) -> c_int;
    pub fn cc_set_verkey(ctx: *mut CcCtx, x: *const u8, y: *const u8, q: usize) -> c_int;
    // Signature::verify (signature.rs:473-478); rlc = 1: RLC batch mode with exact fallback
    pub fn cc_verify_batch(ctx: *mut CcCtx, n: usize, q: usize, sigma1: *const u8, sigma2: *const u8,
                           msgs: *const u8, vk_x: *const u8, vk_y: *const u8, verdicts: *mut u8,
                           gt: *mut u8, rlc: c_int) -> c_int;
    pub fn cc_verify_batch_device(ctx: *mut CcCtx, n: usize, q: usize, d_sigma1: *const u8, d_sigma2: *const u8,
                                  d_msgs: *const u8, d_verdicts: *mut u8, d_gt: *mut u8, stream: *mut c_void) -> c_int;
    // one verkey per credential (the reference's per-call vk), buffers in HBM
    pub fn cc_verify_batch_pervk_device(ctx: *mut CcCtx, n: usize, q: usize, d_sigma1: *const u8,
                                        d_sigma2: *const u8, d_msgs: *const u8, d_vk_x: *const u8, d_vk_y: *const u8,
                                        d_verdicts: *mut u8, d_gt: *mut u8, stream: *mut c_void) -> c_int;
    pub fn cc_set_table_bits(ctx: *mut CcCtx, verkey_bits: c_int, issuer_bits: c_int) -> c_int;
    pub fn cc_table_bits(ctx: *const CcCtx, verkey_bits: *mut c_int, issuer_bits: *mut c_int) -> c_int;
    pub fn cc_device_error(ctx: *mut CcCtx, stream: *mut c_void, out: *mut u32) -> c_int;
    // concurrent verify batches on one context (K workspace slots, round-robin; K caller streams)
    pub fn cc_set_concurrency(ctx: *mut CcCtx, slots: c_int) -> c_int;
    pub fn cc_concurrency(ctx: *const CcCtx, slots: *mut c_int) -> c_int;
    // RLC partial: CC_RLC_PARTIAL_WORDS (929) u32 = Fp12 product, flag, 16 window sums
    pub fn cc_rlc_partial_words() -> c_int;
    pub fn cc_rlc_partial_device(ctx: *mut CcCtx, n: usize, q: usize, base_index: u64, seed32: *const u8,
                                 d_sigma1: *const u8, d_sigma2: *const u8, d_msgs: *const u8,
                                 d_partial: *mut u32, stream: *mut c_void) -> c_int;
    pub fn cc_rlc_finish_device(ctx: *mut CcCtx, nparts: usize, d_partials: *const u32, d_accept: *mut u8,
                                d_gt: *mut u8, stream: *mut c_void) -> c_int;
    // Signature::aggregate (signature.rs:448-470), Verkey::aggregate (signature.rs:483-526)
    pub fn cc_signature_aggregate_batch(ctx: *mut CcCtx, n: usize, len: usize, t: usize, ids: *const u64,
                                        sigma1: *const u8, sigma2: *const u8, out1: *mut u8, out2: *mut u8) -> c_int;
    pub fn cc_signature_aggregate_batch_device(ctx: *mut CcCtx, n: usize, len: usize, t: usize, d_ids: *const u64,
                                               d_sigma1: *const u8, d_sigma2: *const u8, d_out1: *mut u8,
                                               d_out2: *mut u8, stream: *mut c_void) -> c_int;
    pub fn cc_verkey_aggregate_batch(ctx: *mut CcCtx, n: usize, len: usize, t: usize, q: usize, ids: *const u64,
                                     x: *const u8, y: *const u8, out_x: *mut u8, out_y: *mut u8) -> c_int;
    pub fn cc_set_issuers(ctx: *mut CcCtx, n_issuers: usize, q: usize, ids: *const u64, x: *const u8,
                          y: *const u8) -> c_int;
    pub fn cc_verkey_aggregate_ids(ctx: *mut CcCtx, n: usize, len: usize, t: usize, ids: *const u64,
                                   out_x: *mut u8, out_y: *mut u8) -> c_int;
    pub fn cc_verkey_aggregate_ids_device(ctx: *mut CcCtx, n: usize, len: usize, t: usize, d_ids: *const u64,
                                          d_out_x: *mut u8, d_out_y: *mut u8, stream: *mut c_void) -> c_int;
    pub fn cc_aggregate_credential_batch_device(ctx: *mut CcCtx, n: usize, len: usize, t: usize, d_ids: *const u64,
                                                d_sigma1: *const u8, d_sigma2: *const u8, d_out1: *mut u8,
                                                d_out2: *mut u8, d_out_x: *mut u8, d_out_y: *mut u8,
                                                stream: *mut c_void) -> c_int;
    // PoKOfSignatureProof::verify (pok_sig.rs:103-105)
    pub fn cc_pok_verify_batch(ctx: *mut CcCtx, n: usize, q: usize, r: usize, nresp: usize,
                               sigma1: *const u8, sigma2: *const u8, j: *const u8, t: *const u8,
                               responses: *const u8, chal: *const u8, revealed_idx: *const u64,
                               revealed_msgs: *const u8, verdicts: *mut u8, gt: *mut u8) -> c_int;
    pub fn cc_pok_verify_batch_device(ctx: *mut CcCtx, n: usize, q: usize, r: usize, nresp: usize,
                                      d_sigma1: *const u8, d_sigma2: *const u8, d_j: *const u8, d_t: *const u8,
                                      d_responses: *const u8, d_chal: *const u8, revealed_idx: *const u64,
                                      d_revealed_msgs: *const u8, d_verdicts: *mut u8, d_gt: *mut u8,
                                      stream: *mut c_void) -> c_int;
    // §8(f): codec, hash-to-curve, issuer side, keygen
    pub fn cc_subgroup_check(ctx: *mut CcCtx, group: c_int, n: usize, points: *const u8, status: *mut u8) -> c_int;
    pub fn cc_hash_to_curve(ctx: *mut CcCtx, group: c_int, n: usize, data: *const u8, offsets: *const u64,
                            out: *mut u8) -> c_int;
    pub fn cc_hash_msg(ctx: *mut CcCtx, n: usize, data: *const u8, offsets: *const u64, out48: *mut u8) -> c_int;
    pub fn cc_blind_sign_batch(ctx: *mut CcCtx, n: usize, q: usize, k: usize, commitment: *const u8,
                               known: *const u8, ciphertexts: *const u8, x: *const u8, y: *const u8,
                               out_h: *mut u8, out_c1: *mut u8, out_c2: *mut u8) -> c_int;
    pub fn cc_sigreq_proof_bytes(ctx: *const CcCtx, k: usize) -> usize;
    pub fn cc_sigreq_verify_batch(ctx: *mut CcCtx, n: usize, q: usize, k: usize, g: *const u8, h: *const u8,
                                  commitment: *const u8, known: *const u8, ciphertexts: *const u8,
                                  elgamal_pk: *const u8, proofs: *const u8, chal: *const u8,
                                  verdicts: *mut u8) -> c_int;
    pub fn cc_vss_verify_batch(ctx: *mut CcCtx, n: usize, t: usize, g: *const u8, h: *const u8,
                               commitments: *const u8, n_sets: usize, set_of: *const u32, ids: *const u64,
                               shares: *const u8, verdicts: *mut u8) -> c_int;
    pub fn cc_fixed_base_mul(ctx: *mut CcCtx, group: c_int, base: *const u8, n: usize, scalars: *const u8,
                             out: *mut u8) -> c_int;
    pub fn cc_last_timing(ctx: *const CcCtx, prep_ms: *mut f32, miller_ms: *mut f32, fexp_ms: *mut f32) -> c_int;
    pub fn cc_set_timing(ctx: *mut CcCtx, enabled: c_int) -> c_int;
    // device self-test of the lazy field core (test infrastructure; no context)
    pub fn cc_selftest_lazy(op: c_int, n: usize, a: *const i32, b: *const i32, c: *const i32, d: *const i32,
                            out: *mut i32) -> c_int;
}

/// Owner of one `cc_ctx` (one per calling thread: the C ABI's threading contract).
pub struct HipCtx {
    pub raw: *mut CcCtx,
}

impl HipCtx {
    /// `cc_ctx_create(device, mode)`; mode CC_SIG_G2 for the reference's default feature.
    pub fn new(device: c_int, mode: c_int) -> Result<HipCtx, c_int> {
        let mut raw = std::ptr::null_mut();
        let st = unsafe { cc_ctx_create(device, mode, &mut raw) };
        if st != 0 { Err(st) } else { Ok(HipCtx { raw }) }
    }
    /// A device set (bit d of `mask` = GPU d): batches shard by credential, RLC all-gathers inside.
    pub fn new_multi(mask: u64, mode: c_int) -> Result<HipCtx, c_int> {
        let mut raw = std::ptr::null_mut();
        let st = unsafe { cc_ctx_create_multi(mask, mode, &mut raw) };
        if st != 0 { Err(st) } else { Ok(HipCtx { raw }) }
    }
    pub fn mode(&self) -> c_int {
        let mut m = 0;
        self.check(unsafe { cc_ctx_mode(self.raw, &mut m) });
        m
    }
    pub fn status_str(&self, st: c_int) -> String {
        unsafe { std::ffi::CStr::from_ptr(cc_status_str(st)) }.to_string_lossy().into_owned()
    }
    /// Panics where the reference panics (assert!/unwrap); the codes mirror src/errors.rs:6-24.
    pub fn check(&self, st: c_int) {
        assert_eq!(st, 0, "{}", self.status_str(st));
    }
    /// Encoded sizes (amcl_wrapper to_bytes): SignatureGroup / OtherGroup element under this context's mode.
    pub fn sig_bytes(&self) -> usize { if self.mode() == CC_SIG_G2 { 192 } else { 97 } }
    pub fn oth_bytes(&self) -> usize { if self.mode() == CC_SIG_G2 { 97 } else { 192 } }
    /// Idempotent: the same g~ again is a byte compare.
    pub fn set_params(&self, g_tilde: &[u8]) {
        assert_eq!(g_tilde.len(), self.oth_bytes(), "g~ encoding");  // len-guard: the C side reads oth_bytes
        self.check(unsafe { cc_set_params(self.raw, g_tilde.as_ptr()) });
    }
    /// Idempotent: the same verkey again is a byte compare; a new one builds fixed-base tables.
    pub fn set_verkey(&self, x: &[u8], y: &[u8], q: usize) {
        let ob = self.oth_bytes();
        assert!(x.len() == ob && y.len() == q * ob, "verkey encoding");  // len-guard: X 1 x ob, Y q x ob
        self.check(unsafe { cc_set_verkey(self.raw, x.as_ptr(), y.as_ptr(), q) });
    }
}

impl Drop for HipCtx {
    fn drop(&mut self) {
        unsafe { cc_ctx_destroy(self.raw) };
    }
}
