/* coconut_hip.h — C ABI of the MI355X batch-verification engine for Coconut credentials.
 *
 * Drop-in boundary for the reference's verifier hot path (3for/coconut-rust, read-only at
 * /root/reference).  The reference has no FFI of its own; these entry points are what its Rust
 * API would bind through `extern "C"` (binding shown in INTEGRATION.md):
 *
 *   cc_verify_batch / cc_verify_batch_device / cc_verify_batch_pervk_device
 *        replaces  Signature::verify              src/signature.rs:473-478
 *                  (-> ps_sig Signature::verify [EXT], via transforms signature.rs:83-104)
 *   cc_signature_aggregate_batch
 *        replaces  Signature::aggregate           src/signature.rs:448-470
 *   cc_verkey_aggregate_batch
 *        replaces  Verkey::aggregate              src/signature.rs:483-526
 *   cc_pok_verify_batch
 *        replaces  ps_sig PoKOfSignatureProof::verify [EXT], called at src/pok_sig.rs:103-105
 *   cc_set_params / cc_set_verkey
 *        the Params (src/signature.rs:13-17, only g_tilde is read by verify) and Verkey
 *        (src/signature.rs:46-49) a batch is checked against
 *
 * Encodings are amcl_wrapper's `to_bytes`:
 *   Fr 48 B big-endian | G1 97 B = 0x04||x||y | G2 192 B = x.a||x.b||y.a||y.b | GT 576 B (AMCL FP12)
 * Group assignment (reference src/lib.rs:3-4,12-13): CC_SIG_G2 = the reference default build
 * (sigma, g, h in G2; X~, Y~, g~ in G1), CC_SIG_G1 = the other feature.
 *
 * All host pointers are caller-owned, read during the call and never retained.  A context owns
 * one HIP device, one stream and the device tables; use one context per calling thread.
 * A context made by cc_ctx_create_multi spans a device set (one single-device context and one RCCL
 * communicator per GPU, one host thread per GPU during a call): cc_set_params / cc_set_verkey apply
 * to every device and cc_verify_batch shards the batch by credential over the set (RLC mode: one
 * ncclAllGather of 3,716-byte partials over xGMI); the other entry points run on the
 * set's first device.
 * Streams: the *_device entry points take a caller stream; the library orders it against the
 * context's own stream (which the host entry points use) with events at entry and exit, so calls on
 * any mix of streams see the context's workspaces in program order.
 * Errors mirror the reference's failure modes (src/errors.rs:6-24): where the reference panics
 * (assert!/unwrap) the C ABI returns a code instead.
 * Empty batches: every batch entry point checks its context state and lengths first (CC_ERR_STATE,
 * CC_ERR_LEN, CC_ERR_BASES_EXPS, CC_ERR_THRESHOLD), then returns CC_OK for n = 0 without reading,
 * writing or launching anything; its buffer pointers may then be NULL (tests/test_gpu_empty.py).
 * Ceilings: n <= CC_MAX_BATCH credentials / proofs / points per call, an aggregation's ids per
 * credential (len) <= CC_MAX_IDS, q <= CC_MAX_Q messages, an RLC finish's gathered partials <=
 * CC_MAX_PARTS; a larger count is CC_ERR_DECODE before anything is read, allocated or launched (the
 * byte counts the library derives from them then never overflow).
 */
#ifndef COCONUT_HIP_H
#define COCONUT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CC_MAX_BATCH ((size_t)1 << 26)
#define CC_MAX_IDS ((size_t)1 << 16)
#define CC_MAX_Q ((size_t)4096)
#define CC_MAX_PARTS ((size_t)1 << 16)

typedef enum {
    CC_OK = 0,
    CC_ERR_LEN = -1,          /* CoconutErrorKind::UnsupportedNoOfMessages (verkey q != msgs)   */
    CC_ERR_BASES_EXPS = -2,   /* CoconutErrorKind::UnequalNoOfBasesExponents (PoK responses)    */
    CC_ERR_THRESHOLD = -3,    /* len < threshold: reference assert! panics (signature.rs:449,484) */
    CC_ERR_DECODE = -4,       /* malformed buffer sizes / missing params                           */
    CC_ERR_HIP = -5,          /* HIP runtime failure                                               */
    CC_ERR_RCCL = -6,         /* collective failure (RLC gather)                                   */
    CC_ERR_STATE = -7         /* call order: params / verkey not set                               */
} cc_status;

typedef enum { CC_SIG_G2 = 0, CC_SIG_G1 = 1 } cc_group_mode;

typedef struct cc_ctx cc_ctx;

const char* cc_status_str(int status);
const char* cc_version(void);

cc_status cc_ctx_create(int device, cc_group_mode mode, cc_ctx** out);
/* Device set: bit d of device_mask selects GPU d (SURVEY.md §8b `cc_ctx_create(device_mask, ...)`);
 * CC_ERR_RCCL if the communicators cannot be created. */
cc_status cc_ctx_create_multi(uint64_t device_mask, cc_group_mode mode, cc_ctx** out);
cc_status cc_ctx_num_devices(const cc_ctx* ctx, int* ndev);
cc_status cc_ctx_destroy(cc_ctx* ctx);
cc_status cc_ctx_mode(const cc_ctx* ctx, int* mode_out);

/* Params: only g_tilde (OtherGroup encoding) is used on the verify path. */
cc_status cc_set_params(cc_ctx* ctx, const uint8_t* g_tilde);

/* Shared verkey (X~, Y~[q]) for cc_verify_batch with vk == NULL: builds fixed-base tables on the
 * device (one-time cost, reported separately from batch throughput): the widest of 22 / 20 / 18 / 16 /
 * 14 / 12 / 10-bit windows whose q + 2 bases' tables fit 4 GiB and 40 % of the free HBM, else 8-bit
 * windows (cc_set_table_bits forces a width).  The same verkey again (bytes and width unchanged) is a
 * no-op.  On any failure the context is left WITHOUT a verkey (verify / RLC / PoK calls then return
 * CC_ERR_STATE). */
cc_status cc_set_verkey(cc_ctx* ctx, const uint8_t* X, const uint8_t* Y, size_t q);

/* Window widths of the fixed-base tables built by later cc_set_verkey / cc_set_issuers calls:
 * verkey_bits 0 (chosen by memory) or 8..22; issuer_bits 0 (chosen by memory) or 8..16.  A forced
 * width that does not fit HBM makes the building call fail.  cc_table_bits reports the widths of the
 * current tables (0: none built). */
cc_status cc_set_table_bits(cc_ctx* ctx, int verkey_bits, int issuer_bits);
cc_status cc_table_bits(const cc_ctx* ctx, int* verkey_bits, int* issuer_bits);

/* Batch Signature::verify.
 *   sigma1, sigma2 : n x SignatureGroup encodings
 *   msgs           : n x q x 48 B
 *   vk_X, vk_Y     : NULL => the shared verkey from cc_set_verkey; else n x OtherGroup and
 *                    n x q x OtherGroup (one verkey per credential)
 *   verdicts       : n bytes, 1 = verify() returned true
 *   gt_or_null     : n x 576 B, e(.,.)*e(.,.) as amcl_wrapper GT::to_bytes, or NULL
 *   rlc            : 0 = per-credential; 1 = random-linear-combination batch (all-or-fallback)
 * Returns CC_ERR_LEN if q differs from the shared verkey's q (the reference panics there).
 * Batch size picks the kernels, not the results: a batch of up to 4,096 credentials runs latency-bound
 * (one wave per Miller pair; up to 2,048 also one per final exponentiation and per shared-verkey prep,
 * up to 1,024 one per per-credential-verkey or PoK prep), a larger one throughput-bound (one lane pair per credential); verdicts and GT bytes are the
 * same either way. */
cc_status cc_verify_batch(cc_ctx* ctx, size_t n, size_t q, const uint8_t* sigma1, const uint8_t* sigma2,
                          const uint8_t* msgs, const uint8_t* vk_X, const uint8_t* vk_Y, uint8_t* verdicts,
                          uint8_t* gt_or_null, int rlc);

/* Same, with every buffer already in device memory (HBM-resident batch; the timed bench path).
 * Shared verkey only.  `stream` is a hipStream_t or NULL for the context's stream.  The call is
 * asynchronous with respect to the host; synchronise the stream before reading verdicts. */
cc_status cc_verify_batch_device(cc_ctx* ctx, size_t n, size_t q, const uint8_t* d_sigma1, const uint8_t* d_sigma2,
                                 const uint8_t* d_msgs, uint8_t* d_verdicts, uint8_t* d_gt_or_null, void* stream);

/* Per-credential verkeys with every buffer in device memory: Signature::verify(msgs, vk_i, params) for
 * each credential i with ITS OWN verkey (src/signature.rs:473-478 takes the verkey per call;
 * ps_sig's var-time MSM over [X~, Y~_1..q]): d_vk_X n x OtherGroup, d_vk_Y n x q x OtherGroup, the
 * rest as cc_verify_batch_device.  Needs only cc_set_params (g~); q <= 4096.  Asynchronous on
 * `stream` (NULL: the context stream). */
cc_status cc_verify_batch_pervk_device(cc_ctx* ctx, size_t n, size_t q, const uint8_t* d_sigma1,
                                       const uint8_t* d_sigma2, const uint8_t* d_msgs, const uint8_t* d_vk_X,
                                       const uint8_t* d_vk_Y, uint8_t* d_verdicts, uint8_t* d_gt_or_null,
                                       void* stream);

/* Concurrent verify batches on one context: with `slots` = K > 1, cc_verify_batch_device,
 * cc_verify_batch_pervk_device, cc_pok_verify_batch_device and cc_rlc_partial_device calls take K
 * workspace slots round-robin (each slot its own prep SoA, flags, Miller values, PoK d J tables and RLC
 * delta/fold buffers; the verkey tables are shared)
 * and are ordered only after the context's earlier work (tables, params) and the same slot's previous
 * batch — so K batches issued on K caller streams overlap on the device (one batch's kernel tails with
 * the next batch's kernels).  Every other
 * entry point, and cc_set_params / cc_set_verkey, first waits for the slots' batches.  The per-phase
 * timing (cc_last_timing) is meaningful with one slot only.  slots: 1 (default, every call ordered
 * against every other) .. 8.  cc_concurrency reports the current value. */
cc_status cc_set_concurrency(cc_ctx* ctx, int slots);
cc_status cc_concurrency(const cc_ctx* ctx, int* slots);

/* RLC batch mode, multi-GPU form.  Each GPU reduces its shard to one partial of
 * CC_RLC_PARTIAL_WORDS u32 (= cc_rlc_partial_words(): the Fp12 Miller product in the library's
 * Montgomery words, a fall-back flag, and the shard's 16 fold window sums, affine with identity
 * flags); the caller gathers the partials of all GPUs (RCCL all-gather over xGMI, or any transport)
 * and every GPU finishes with 16 window pairs per partial and ONE final exponentiation:
 *   cc_rlc_partial_device: deltas = ChaCha20(seed32, base_index + i), i < n (shared verkey only);
 *                          d_partial: CC_RLC_PARTIAL_WORDS x u32 device buffer; n = 0 (an empty
 *                          shard) writes the neutral partial (Fp12 one, flag clear, identity window
 *                          sums) so the rank still joins the gather.
 *   cc_rlc_finish_device : nparts partials (nparts x CC_RLC_PARTIAL_WORDS u32, device): their window
 *                          pairs, the product, the final exponentiation; *d_accept = 1 iff the whole
 *                          batch verifies (then every per-credential verdict is 1); 0 means "fall back
 *                          to per-credential verification" (a bad or identity credential somewhere).
 *                          d_gt optional (576 B, GT of the combined product).  Needs the verkey of the
 *                          partials (its g~ multiples); a cc_set_verkey waits for running finishes.
 * Both are asynchronous on `stream` (NULL: the context stream).  The partial is ordered against the
 * context's other work; the finish owns its buffers and is NOT, so on a second stream it may overlap
 * the next batch's partial (the caller orders d_partials before it, and two finishes of one context
 * one after the other); with cc_set_concurrency(K) successive partials take K slots and overlap too.  cc_verify_batch(..., rlc = 1) runs the single-GPU form with a fresh seed
 * from /dev/urandom and falls back by itself. */
#define CC_RLC_PARTIAL_WORDS 929
int cc_rlc_partial_words(void);
cc_status cc_rlc_partial_device(cc_ctx* ctx, size_t n, size_t q, uint64_t base_index, const uint8_t* seed32,
                                const uint8_t* d_sigma1, const uint8_t* d_sigma2, const uint8_t* d_msgs,
                                uint32_t* d_partial, void* stream);
cc_status cc_rlc_finish_device(cc_ctx* ctx, size_t nparts, const uint32_t* d_partials, uint8_t* d_accept,
                               uint8_t* d_gt_or_null, void* stream);

/* Batch Signature::aggregate: n independent aggregations of `len` (id, Signature) entries each;
 * only the first t entries are used, sigma_1 comes from entry 0, Lagrange over the de-duplicated
 * id set (signature.rs:448-470).  ids: n x len; sigma1/sigma2: n x len encodings;
 * out_sigma1/out_sigma2: n encodings. */
cc_status cc_signature_aggregate_batch(cc_ctx* ctx, size_t n, size_t len, size_t t, const uint64_t* ids,
                                       const uint8_t* sigma1, const uint8_t* sigma2, uint8_t* out_sigma1,
                                       uint8_t* out_sigma2);

/* Batch Verkey::aggregate (signature.rs:483-526): X: n x len, Y: n x len x q; outX: n; outY: n x q. */
cc_status cc_verkey_aggregate_batch(cc_ctx* ctx, size_t n, size_t len, size_t t, size_t q, const uint64_t* ids,
                                    const uint8_t* X, const uint8_t* Y, uint8_t* outX, uint8_t* outY);

/* Device-buffer form of cc_signature_aggregate_batch (inputs resident in HBM; the timed path of
 * BASELINE config 4).  Asynchronous on `stream` (NULL: the context stream). */
cc_status cc_signature_aggregate_batch_device(cc_ctx* ctx, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                              const uint8_t* d_sigma1, const uint8_t* d_sigma2,
                                              uint8_t* d_out_sigma1, uint8_t* d_out_sigma2, void* stream);

/* Issuer table for Verkey::aggregate at scale (BASELINE config 4: t = 67 of n = 100 issuers).  The
 * n_issuers verkeys (X: n_issuers x OtherGroup, Y: n_issuers x q x OtherGroup) and their signer ids
 * (unique) are decoded once and given fixed-base window tables in HBM (one-time cost; the widest
 * window in {16, 13, 12, 10, 8} whose tables fit 16 GiB and half the free HBM — 13-bit, 11 GB, for
 * 100 issuers x 7 G1 keys — or the width forced by cc_set_table_bits); a batch then passes only id
 * lists.  A failed call leaves no issuer table (CC_ERR_STATE afterwards).
 * cc_verkey_aggregate_ids(_device) computes, per credential, exactly
 * Verkey::aggregate(t, [(id_k, &issuer[id_k])]) (signature.rs:483-526): first t entries, Lagrange
 * over the de-duplicated id set.  ids: n x len.  An id without an issuer verkey (the reference would
 * index a missing key): the host form returns CC_ERR_DECODE before launching; the device form writes
 * the identity encoding for the affected outputs and raises the context's device error word
 * (CC_DEVERR_UNKNOWN_ID), which cc_device_error reads. */
cc_status cc_set_issuers(cc_ctx* ctx, size_t n_issuers, size_t q, const uint64_t* ids, const uint8_t* X,
                         const uint8_t* Y);
cc_status cc_verkey_aggregate_ids(cc_ctx* ctx, size_t n, size_t len, size_t t, const uint64_t* ids, uint8_t* outX,
                                  uint8_t* outY);
cc_status cc_verkey_aggregate_ids_device(cc_ctx* ctx, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                         uint8_t* d_outX, uint8_t* d_outY, void* stream);

/* Both aggregations of the same credentials, as a verifier holding per-credential shares does them:
 * Signature::aggregate(t, [(id_k, sig_k)]) (signature.rs:448-470) and Verkey::aggregate(t, [(id_k,
 * issuer[id_k])]) (signature.rs:483-526) over ONE id list per credential, so the Lagrange coefficients
 * (signature.rs:454-463 = 496-509) are computed once.  Outputs and errors as the two calls above
 * (device error word as cc_verkey_aggregate_ids_device).  Asynchronous on `stream`. */
cc_status cc_aggregate_credential_batch_device(cc_ctx* ctx, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                               const uint8_t* d_sigma1, const uint8_t* d_sigma2,
                                               uint8_t* d_out_sigma1, uint8_t* d_out_sigma2, uint8_t* d_outX,
                                               uint8_t* d_outY, void* stream);

/* Argument errors that only the device can see (ids checked inside a kernel of a *_device call):
 * synchronises `stream` (NULL: the context stream), returns the OR of the CC_DEVERR_* bits raised since
 * the last read in *out, and clears them. */
#define CC_DEVERR_UNKNOWN_ID 1u
cc_status cc_device_error(cc_ctx* ctx, void* stream, uint32_t* out);

/* Batch PoKOfSignatureProof::verify against the shared verkey and params.
 *   sigma1, sigma2  : n x SignatureGroup (sigma'_1, sigma'_2)
 *   J, T            : n x OtherGroup (J and the Schnorr commitment)
 *   responses       : n x (q - r + 1) x 48 B, order [g~, Y~_i for hidden i ascending]
 *   chal            : n x 48 B
 *   revealed_idx    : r indices (shared by the batch, ascending, < q)
 *   revealed_msgs   : n x r x 48 B
 * CC_ERR_BASES_EXPS if nresp != q - r + 1 (ps_sig returns UnequalNoOfBasesExponents). */
cc_status cc_pok_verify_batch(cc_ctx* ctx, size_t n, size_t q, size_t r, size_t nresp, const uint8_t* sigma1,
                              const uint8_t* sigma2, const uint8_t* J, const uint8_t* T, const uint8_t* responses,
                              const uint8_t* chal, const uint64_t* revealed_idx, const uint8_t* revealed_msgs,
                              uint8_t* verdicts, uint8_t* gt_or_null);

/* Same, with the per-proof buffers already in device memory (the timed bench path, config 5);
 * revealed_idx stays a host array of r indices.  Asynchronous on `stream` (NULL: context stream). */
cc_status cc_pok_verify_batch_device(cc_ctx* ctx, size_t n, size_t q, size_t r, size_t nresp, const uint8_t* d_sigma1,
                                     const uint8_t* d_sigma2, const uint8_t* d_J, const uint8_t* d_T,
                                     const uint8_t* d_responses, const uint8_t* d_chal, const uint64_t* revealed_idx,
                                     const uint8_t* d_revealed_msgs, uint8_t* d_verdicts, uint8_t* d_gt_or_null,
                                     void* stream);

/* Codec check: decode n encodings of `group` (1 = G1 97 B, 2 = G2 192 B) and
 * report per point 0 = identity (AMCL maps a bad prefix / off-curve point to infinity), 1 = on the
 * curve but outside the order-r subgroup, 2 = in G1 / G2.  The reference never tests membership on
 * verify, so cc_verify_batch keeps its semantics; the RLC batch mode uses the same tests internally
 * (a sigma or verkey point outside the subgroup makes the batch fall back to per-credential).
 * Tests: G1 phi(P) == -[x^2] P, G2 psi(Q) == [x] Q (eprint 2021/1130, 2022/352). */
cc_status cc_subgroup_check(cc_ctx* ctx, int group, size_t n, const uint8_t* points, uint8_t* status);

/* Batched amcl_wrapper `from_msg_hash`: n messages, message i =
 * data[offsets[i] .. offsets[i+1]) (offsets: n + 1 entries, offsets[0] = 0), each hashed with
 * SHAKE256 to 48 bytes and mapped to `group` (1 = G1, 2 = G2) by AMCL's try-and-increment `mapit`
 * with cofactor clearing; out: n encodings.  Params::new (signature.rs:22-32) hashes label || " : g",
 * " : g_tilde", " : y" || i; SignatureRequest::compute_h (signature.rs:197-206) hashes
 * commitment.to_bytes() || m_i.to_bytes().  Parity unpinned (AMCL restated, see oracle/).
 * cc_hash_msg: the 48-byte SHAKE256 digests alone (amcl_wrapper hash_msg). */
cc_status cc_hash_to_curve(cc_ctx* ctx, int group, size_t n, const uint8_t* data, const uint64_t* offsets,
                           uint8_t* out);
cc_status cc_hash_msg(cc_ctx* ctx, size_t n, const uint8_t* data, const uint64_t* offsets, uint8_t* out48);

/* Issuer-side batch, n signature requests with k hidden of q messages,
 * SignatureGroup encodings:
 *   cc_blind_sign_batch  : BlindSignature::new (signature.rs:382-433) under one issuer key
 *       commitment n x SG | known n x (q-k) x 48 | ciphertexts n x k x (c1, c2) | x 48 | y q x 48
 *       -> out_h (= compute_h), out_c1, out_c2 (n x SG each)
 *   cc_sigreq_verify_batch : SignatureRequestProof::verify (signature.rs:324-377), verdicts n bytes;
 *       g and h[0..k) are the Params' SignatureGroup generators; elgamal_pk n x SG; chal n x 48;
 *       proofs n x cc_sigreq_proof_bytes(ctx, k) bytes, per request:
 *         T_sk | r_sk | T_comm | r_comm[k+1] | k x (T_1 | r_1 | T_2 | r_2a | r_2b)
 *       (T = Schnorr commitment encodings, r = 48-byte responses).
 * CC_ERR_LEN if k > q (the reference's assert_eq!). */
cc_status cc_blind_sign_batch(cc_ctx* ctx, size_t n, size_t q, size_t k, const uint8_t* commitment,
                              const uint8_t* known, const uint8_t* ciphertexts, const uint8_t* x, const uint8_t* y,
                              uint8_t* out_h, uint8_t* out_c1, uint8_t* out_c2);
size_t cc_sigreq_proof_bytes(const cc_ctx* ctx, size_t k);
cc_status cc_sigreq_verify_batch(cc_ctx* ctx, size_t n, size_t q, size_t k, const uint8_t* g, const uint8_t* h,
                                 const uint8_t* commitment, const uint8_t* known, const uint8_t* ciphertexts,
                                 const uint8_t* elgamal_pk, const uint8_t* proofs, const uint8_t* chal,
                                 uint8_t* verdicts);

/* Pedersen VSS share verification (secret_sharing PedersenVSS::verify_share,
 * used by trusted_party_PVSS_keygen, reference keygen.rs:74-122, 334-349), n shares in G1:
 *   g * s + h * s' == sum_{k<t} id^k * C_k, C = commitments[set_of[i]] (n_sets x t x 97 B),
 *   shares n x (s, s') 48 B each, ids n x u64; verdicts n bytes.
 * The keygen derivation alpha_i = g~ * x_i, beta_ij = g~ * y_ij (keygen.rs:17-45) is
 * cc_fixed_base_mul. */
cc_status cc_vss_verify_batch(cc_ctx* ctx, size_t n, size_t t, const uint8_t* g, const uint8_t* h,
                              const uint8_t* commitments, size_t n_sets, const uint32_t* set_of, const uint64_t* ids,
                              const uint8_t* shares, uint8_t* verdicts);

/* Batch fixed-base scalar multiplication out_i = k_i * base (group 1 = G1, 2 = G2); scalars n x 48 B
 * big-endian Fr, out n encodings.  The keygen derivation g~ * x_i (reference src/keygen.rs:27-32)
 * and the issuer's h^e (src/signature.rs:423-428) in batch form. */
cc_status cc_fixed_base_mul(cc_ctx* ctx, int group, const uint8_t* base, size_t n, const uint8_t* scalars,
                            uint8_t* out);

/* Kernel timing of the last cc_verify_batch_device call (HIP events on the context stream):
 * milliseconds per phase {prep, miller, fexp}.  Used by bench.py for the roofline figure. */
cc_status cc_last_timing(const cc_ctx* ctx, float* prep_ms, float* miller_ms, float* fexp_ms);
cc_status cc_set_timing(cc_ctx* ctx, int enabled);

/* Device self-test of the lazy radix-2^28 field core the pairing kernels use (csrc/lazy.h): op 0
 * (a b + c d) / 2^392, op 1 a b / 2^392 (signed product scanning with Montgomery reduction), op 2 the
 * value reduction, op 3 the limb squeeze, on n elements of 14 signed 28-bit-radix limbs (host
 * arrays, n x 14 int32; b, c, d may be NULL for ops 1-3).  Test infrastructure: the tests drive it
 * at the limits of the compile-time bounds and compare with big-integer arithmetic.  Returns 0, or
 * -1 on a HIP error or an unknown op.  No context needed (current device). */
int cc_selftest_lazy(int op, size_t n, const int32_t* a, const int32_t* b, const int32_t* c, const int32_t* d,
                     int32_t* out);

#ifdef __cplusplus
}
#endif

#endif /* COCONUT_HIP_H */
