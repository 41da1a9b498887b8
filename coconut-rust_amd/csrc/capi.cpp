// C ABI implementation (include/coconut_hip.h): contexts, device tables, batch launches.
// Host side of the MI355X engine; every compute step runs in the HIP kernels of kernels.hip /
// aggregate.hip — there is no CPU fallback in this library.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/coconut_hip.h"
#include "rlc_part.h"
#include "slots.h"

extern "C" {
int cck_decode_points(int group, size_t n, const uint8_t* d_bytes, uint32_t* d_out, uint32_t* d_inf, hipStream_t st);
int cck_build_table(int group, int nbases, int wbits, const uint32_t* d_bases, const uint32_t* d_inf, uint32_t* d_pw,
                    uint32_t* d_table, int lazy_g2, hipStream_t st);
int cck_gtilde_lines(const uint32_t* d_gtilde_aff, uint32_t* d_lines, hipStream_t st);
int cck_lazy_form(size_t n, const uint32_t* d_in, uint32_t* d_out, hipStream_t st);
int cck_subgroup(int group, size_t n, const uint8_t* d_bytes, uint8_t* d_status, hipStream_t st);
int cck_hash_to_curve(int group, size_t n, const uint8_t* d_data, const uint64_t* d_offsets, uint8_t* d_out,
                      uint32_t* d_fail, hipStream_t st);
int cck_shake256_48(size_t n, const uint8_t* d_data, const uint64_t* d_offsets, uint8_t* d_out, hipStream_t st);
size_t cck_sigreq_proof_bytes(int group, int k);
int cck_vss_verify(size_t n, int t, const uint8_t* d_g, const uint8_t* d_h, const uint8_t* d_comms,
                   const uint32_t* d_set_of, const uint64_t* d_ids, const uint8_t* d_shares, uint32_t* d_scratch,
                   uint8_t* d_ok, hipStream_t st);
int cck_blind_assemble(int group, size_t n, int q, int k, const uint8_t* d_cts, const uint8_t* d_h,
                       const uint8_t* d_known, const uint8_t* d_x, const uint8_t* d_y, uint8_t* d_pts, uint32_t* d_sc,
                       hipStream_t st);
size_t cck_sigreq_scratch_words(int group, size_t n, int k);
int cck_sigreq_verify(int group, size_t n, int k, const uint8_t* d_g, const uint8_t* d_hvec, const uint8_t* d_comm,
                      const uint8_t* d_cts, const uint8_t* d_pk, const uint8_t* d_proof, const uint8_t* d_chal,
                      const uint8_t* d_hpts, uint32_t* d_scratch, uint8_t* d_ok, uint8_t* d_verdicts, hipStream_t st);
int cck_prep(int mode, size_t n, int q, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs,
             const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits, const uint32_t* d_binf_fixed,
             uint32_t* d_prep, uint32_t* d_flags, hipStream_t st);
int cck_prep_wide(int mode, size_t n, int q, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs,
                  const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits, const uint32_t* d_binf_fixed,
                  uint32_t* d_prep, uint32_t* d_flags, hipStream_t st);
size_t cck_prep_var_words(int mode, size_t n, size_t q);
int cck_prep_var(int mode, size_t n, int q, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_vkX,
                 const uint8_t* d_vkY, const uint8_t* d_msgs, uint32_t* d_scratch, uint32_t* d_prep,
                 uint32_t* d_flags, int wide, hipStream_t st);
int cck_miller_lz_g2(int twin, size_t n, size_t pstride, const uint32_t* d_prep, const uint32_t* d_flags,
                     const uint32_t* d_const, uint32_t* d_f, size_t fstride, size_t foff, uint32_t* d_qcheck,
                     hipStream_t st);
int cck_miller_lz_g1(int twin, size_t n, size_t pstride, const uint32_t* d_prep, const uint32_t* d_flags,
                     const uint32_t* d_const, uint32_t* d_f, size_t fstride, size_t foff, uint32_t* d_qcheck,
                     hipStream_t st);
int cck_miller4_lz_g2(size_t n, size_t pstride, const uint32_t* d_prep, const uint32_t* d_flags, uint32_t* d_f,
                      size_t fstride, size_t foff, uint32_t* d_qcheck, hipStream_t st);
int cck_miller4_lz_g1(size_t n, size_t pstride, const uint32_t* d_prep, const uint32_t* d_flags, uint32_t* d_f,
                      size_t fstride, size_t foff, uint32_t* d_qcheck, hipStream_t st);
size_t cck_fold_words(int mode, size_t n);
int cck_fold_pseudo();
int cck_fold_window(int mode, size_t n, uint32_t* d_work, uint32_t* d_partial, hipStream_t st);
int cck_fold(int mode, size_t n, const int8_t* d_dig, const uint32_t* d_pts, uint32_t* d_work, hipStream_t st);
int cck_fold_fixed(int mode, int q, const uint32_t* d_table, int wbits, const uint32_t* d_binf, uint32_t* d_pw,
                   uint8_t* d_finf, hipStream_t st);
int cck_miller_wide(size_t n, const uint32_t* d_prep, const uint32_t* d_flags, uint32_t* d_f, size_t fstride,
                    size_t foff, hipStream_t st);
int cck_f12_reduce_wide(size_t n, const uint32_t* d_in, uint32_t* d_out, hipStream_t st);
int cck_wide_pairs(int mode, size_t n, size_t ps, const uint32_t* d_prep, const uint32_t* d_flags,
                   const uint32_t* d_gaff, uint32_t* d_wprep, uint32_t* d_wflags, hipStream_t st);
int cck_fexp(size_t n, uint32_t* d_f, uint32_t* d_scratch, const uint32_t* d_flags, uint8_t* d_verdicts,
             uint8_t* d_gt, size_t wide_max, hipStream_t st);
int cck_lagrange(size_t n, size_t len, size_t t, const uint64_t* d_ids, uint32_t* d_l, hipStream_t st);
int cck_h_input_canon(int group, size_t n, size_t len, int kn, uint8_t* d_data, hipStream_t st);

size_t cck_straus_words(int group, size_t t);
int cck_msm_straus(int group, size_t ntask, size_t t, const uint8_t* d_pts, size_t pt_stride, size_t pt_jstride,
                   size_t pt_step, const uint32_t* d_l, size_t l_div, uint32_t* d_scratch, uint8_t* d_out,
                   hipStream_t st);
int cck_vk_agg_fixed(int group, size_t n, size_t len, size_t t, int q, const uint64_t* d_ids, const uint32_t* d_l,
                     const uint64_t* d_iss_ids, int n_iss, const uint32_t* d_table, int wbits, const uint32_t* d_binf,
                     uint8_t* d_outX, uint8_t* d_outY, uint32_t* d_err, hipStream_t st);
int cck_copy_rows(size_t n, size_t sb, const uint8_t* d_src, size_t pitch, uint8_t* d_dst, hipStream_t st);
int cck_fixed_mul(int group, size_t n, const uint8_t* d_ks, const uint32_t* d_table, uint32_t base_inf,
                  uint8_t* d_out, hipStream_t st);
int cck_prep_rlc(int mode, int part, size_t n, size_t ps, int q, uint64_t base_index, const uint32_t* d_key,
                 const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs, const uint32_t* d_table, int wbits,
                 const uint32_t* d_binf, uint32_t* d_prep, uint32_t* d_flags, uint32_t* d_any, uint32_t* d_pts,
                 int8_t* d_dig, hipStream_t st);
int cck_rlc_reduce(size_t n, uint32_t* d_a, uint32_t* d_b, const uint32_t* d_any, uint32_t* d_partial,
                   hipStream_t st);
int cck_rlc_gather(int mode, size_t k, const uint32_t* d_parts, const uint32_t* d_pw, const uint8_t* d_finf,
                   uint32_t* d_fw, size_t fs, uint32_t* d_prep, uint32_t* d_flags2, uint32_t* d_flag, hipStream_t st);
int cck_prep_pok(int mode, size_t n, int q, int r, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_J,
                 const uint8_t* d_T, const uint8_t* d_resp, const uint8_t* d_chal, const uint8_t* d_rev_msgs,
                 const uint32_t* d_rev_idx, const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits,
                 const uint32_t* d_binf, uint32_t* d_prep, uint32_t* d_flags, uint32_t* d_jtab, hipStream_t st);
int cck_prep_pok_wide(int mode, size_t n, int q, int r, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_J,
                 const uint8_t* d_T, const uint8_t* d_resp, const uint8_t* d_chal, const uint8_t* d_rev_msgs,
                 const uint32_t* d_rev_idx, const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits,
                 const uint32_t* d_binf, uint32_t* d_prep, uint32_t* d_flags, uint32_t* d_jtab, hipStream_t st);
}

namespace {

// fixed-base window tables (fixed.h): per base ceil(256 / wbits) windows of 2^wbits - 1 affine entries
static inline size_t tab_words(int group, int wbits) {
    return (size_t)((256 + wbits - 1) / wbits) * (((size_t)1 << wbits) - 1) * (group == 1 ? 24 : 48);
}
static inline size_t tab_nwin(int wbits) { return (size_t)((256 + wbits - 1) / wbits); }
// free HBM of the current device (0 if the runtime cannot say)
static size_t free_hbm() {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return fr;
}
constexpr size_t PREP_SLOTS = cc::slots::kPrepSlots;  // soa.h
// default HBM budget of a context's shared-verkey tables (wider: cc_set_table_bits)
constexpr double kVkTableBudget = 4.0 * (double)(1ull << 30);

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want) {
        if (want <= bytes) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, want) != hipSuccess) return -1;
        bytes = want;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

// The device policy of the slot bookkeeping (slots.h): hipMalloc'd buffers, HIP events and streams.
struct HipDev {
    using Buf = DevBuf;
    using Event = hipEvent_t;
    using Stream = hipStream_t;
    int ensure(DevBuf& b, size_t n) { return b.ensure(n); }
    int sync(hipEvent_t e) { return hipEventSynchronize(e) == hipSuccess ? 0 : -1; }
    int record(hipEvent_t e, hipStream_t s) { return hipEventRecord(e, s) == hipSuccess ? 0 : -1; }
    int wait(hipStream_t s, hipEvent_t e) { return hipStreamWaitEvent(s, e, 0) == hipSuccess ? 0 : -1; }
};
using VerifyWork = cc::slots::Work<DevBuf>;
using VerifySlot = cc::slots::SlotBufs<DevBuf>;  // slots 1 .. K-1 (slot 0: the context's workspaces)
using SlotPool = cc::slots::Pool<HipDev>;
using SlotFence = cc::slots::Fence<HipDev>;

// Pinned host staging for the few bytes a slot's batch uploads per call (the RLC delta seed, the PoK
// revealed indices): a copy from pageable memory may hold the host until the stream reaches it, i.e.
// until the slot's previous batch has run, which would serialize the in-flight batches.  A ring of kR
// entries, each reused only after its own copy (kR calls earlier on this slot) has completed.
struct Staging {
    static constexpr int kR = 4;
    uint8_t* host = nullptr;
    size_t bytes = 0;  // per entry
    hipEvent_t ev[kR] = {};
    bool used[kR] = {};
    int next = 0;
    // copies len bytes of src to d_dst on st through the next entry
    int upload(void* d_dst, const void* src, size_t len, hipStream_t st) {
        if (!len) return 0;
        if (len > bytes) {
            for (int e = 0; e < kR; e++)
                if (used[e] && hipEventSynchronize(ev[e]) != hipSuccess) return -1;
            if (host) (void)hipHostFree(host);
            host = nullptr;
            bytes = 0;
            const size_t want = (len + 63) & ~(size_t)63;
            if (hipHostMalloc((void**)&host, want * kR, hipHostMallocDefault) != hipSuccess) return -1;
            bytes = want;
            for (int e = 0; e < kR; e++) used[e] = false;
        }
        const int e = next;
        next = (next + 1) % kR;
        if (!ev[e] && hipEventCreateWithFlags(&ev[e], hipEventDisableTiming) != hipSuccess) return -1;
        if (used[e] && hipEventSynchronize(ev[e]) != hipSuccess) return -1;  // its copy kR calls ago
        uint8_t* h = host + (size_t)e * bytes;
        memcpy(h, src, len);
        if (hipMemcpyAsync(d_dst, h, len, hipMemcpyHostToDevice, st) != hipSuccess) return -1;
        if (hipEventRecord(ev[e], st) != hipSuccess) return -1;
        used[e] = true;
        return 0;
    }
    void release() {
        for (int e = 0; e < kR; e++) {
            if (used[e]) (void)hipEventSynchronize(ev[e]);
            if (ev[e]) (void)hipEventDestroy(ev[e]);
            ev[e] = nullptr;
            used[e] = false;
        }
        if (host) (void)hipHostFree(host);
        host = nullptr;
        bytes = 0;
    }
};

}  // namespace

struct cc_ctx {
    int device = 0;
    int mode = 0;  // 0 SigG2, 1 SigG1
    hipStream_t stream = nullptr;
    // params
    bool have_params = false;
    std::vector<uint8_t> gtilde_bytes;  // encoding as given (subgroup status at cc_set_verkey; idempotence)
    DevBuf gtilde_aff;   // OtherGroup affine (Montgomery, AoS)
    uint32_t gtilde_inf = 0;
    DevBuf gtilde_lines; // SigG1: Miller lines of g~
    DevBuf gtilde_lz;    // SigG2: g~ affine in the lazy field's R' form (the Miller loop's constant P)
    // verkey
    bool have_vk = false;
    size_t q = 0;
    DevBuf vk_aff;       // (q + 3) points: X~, Y~[q], g~, X~ (AoS)
    DevBuf vk_inf;       // (q + 3) flags
    DevBuf table;        // fixed-base tables for Y~[0..q), g~ and X~ (q + 2 bases; X~ for RLC)
    DevBuf table_inf;    // q + 2 base flags
    int wbits = 16;      // window width of `table`
    int force_vk_bits = 0, force_iss_bits = 0;  // cc_set_table_bits (0: chosen by memory)
    bool vk_subgroup = false;  // X~, Y~ and g~ all in the order-r subgroup (RLC soundness needs it)
    std::vector<uint8_t> vk_bytes;  // X~ || Y~ encodings of the current verkey (cc_set_verkey idempotence)
    int vk_built_force = 0;         // force_vk_bits when the current tables were built
    uint32_t X_inf = 0;
    // workspaces
    DevBuf in_s1, in_s2, in_msgs, in_vkX, in_vkY, in_aux[6];
    DevBuf prep, flags, fbuf, scratch, verdicts, gt, vkb, lag;  // vkb: per-credential-verkey MSM scratch
    DevBuf wide_prep, wide_flags, wide_f;  // batches of <= kWideMax: the one-wave-per-pair Miller path
    // RLC batch mode: ChaCha20 key, identity flag word, partial / gathered partials, verdict
    DevBuf rlc_key, rlc_any, rlc_part, rlc_flag, rlc_accept;
    // cc_rlc_finish_device's own buffers: Fp12 values (partial products, window pairs' Miller values),
    // the product tree's other half / the one-element fexp's scratch, the window pairs' prep and skip
    // flags, the combined product
    DevBuf fin_f, fin_scratch, fin_prep, fin_flags2, fin_part;
    hipEvent_t ev_fin = nullptr;  // end of the last finish: finishes of one context run in call order
    bool fin_recorded = false;
    // RLC g~-side fold (fold.hip): fold points, delta digits, sort/partials/bucket workspace; the fixed
    // points P_w = (256^w) g~ of the window pairs (SoA, built with the verkey tables) and their
    // identity flags
    DevBuf rlc_pts, rlc_dig, rlc_work, rlc_pw, rlc_finf;
    DevBuf pok_idx;  // revealed indices of the last PoK batch
    // issuer table (cc_set_issuers): sorted ids, decoded verkeys, per-base 8-bit window tables
    size_t iss_n = 0, iss_q = 0;
    std::vector<uint64_t> iss_ids_host;
    DevBuf iss_ids, iss_aff, iss_inf, iss_table;
    int iss_wbits = 8;  // window width of the issuer tables
    DevBuf agg_scratch;
    DevBuf dev_err;  // device-side argument errors of *_device calls (cc_device_error)
    uint32_t rlc_key_host[8] = {0};
    // timing
    bool timing = false;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    float last_ms[3] = {0, 0, 0};
    // orders a caller-supplied stream against the context stream (StreamOrder below)
    hipEvent_t ev_order = nullptr;
    // side stream (high priority; ev_fork / ev_join): Verkey::aggregate beside Signature::aggregate,
    // the RLC fold's window pairs beside the delta MSM
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // device set (cc_ctx_create_multi): one single-device context per GPU and one RCCL communicator
    // per GPU (ncclCommInitAll, this process drives every device); empty for a single-device context
    std::vector<cc_ctx*> peers;
    std::vector<ncclComm_t> comms;
    DevBuf rlc_gath;  // per peer: gathered partials (ndev x RLC_PART_WORDS words)
    // concurrent verify batches (cc_set_concurrency): with K > 1 slots, cc_verify_batch_device /
    // cc_verify_batch_pervk_device / cc_pok_verify_batch_device / cc_rlc_partial_device calls take the
    // slots round-robin and are ordered only after the context's earlier work (tables, params) and the
    // same slot's previous batch, so K batches on K caller streams overlap (slots.h).  pool.recs[0] is
    // the context's own workspaces (prep / flags / fbuf / vkb / scratch / pok_idx / wide_*); vslots
    // holds the buffers of slots 1 .. K-1; stage[k] slot k's pinned upload ring.  Every other entry point
    // first waits for every slot's last batch.
    int concurrency = 1;
    HipDev dev;
    SlotPool pool;
    std::vector<VerifySlot*> vslots;
    std::vector<Staging> stage;
};

// Every *_device entry point may run on a caller stream while the context's workspaces (prep, flags,
// fbuf, scratch, RLC buffers, verkey tables) are shared with the host entry points, which run on
// c->stream.  StreamOrder makes the caller's stream wait for everything already queued on c->stream
// at entry, and c->stream wait for the call's work at exit, so calls on any mix of streams touch the
// workspaces in program order (two device calls on different streams are chained through c->stream).
// stream st waits (on the device) for every concurrent verify slot's last batch
static void wait_slots(cc_ctx* c, hipStream_t st) { c->pool.wait_all(c->dev, st); }
// the host waits for every concurrent verify slot's last batch (before buffers a slot may still read
// are freed or rebuilt: tables, params, workspaces)
static void drain_slots(cc_ctx* c) { c->pool.drain(c->dev); }

// Argument ceilings of the batch entry points (coconut_hip.h CC_MAX_BATCH etc.): every size product the
// host computes (n x q x 192 bytes, n x len x 8, grid dimensions) stays far inside size_t and the launch
// limits, so a garbage count is CC_ERR_DECODE before anything is allocated, copied or launched.
constexpr size_t kMaxBatch = CC_MAX_BATCH;  // credentials / proofs / points per call
constexpr size_t kMaxIds = CC_MAX_IDS;      // ids per credential (aggregation `len`)
constexpr size_t kMaxParts = CC_MAX_PARTS;  // gathered partials of one RLC finish
constexpr size_t kMaxQ = CC_MAX_Q;          // messages per credential (cc_set_verkey's bound)

struct StreamOrder {
    cc_ctx* c;
    hipStream_t st;
    StreamOrder(cc_ctx* c_, hipStream_t s) : c(c_), st(s) {
        wait_slots(c, st);
        if (st != c->stream) {
            (void)hipEventRecord(c->ev_order, c->stream);
            (void)hipStreamWaitEvent(st, c->ev_order, 0);
        }
    }
    ~StreamOrder() {
        if (st != c->stream) {
            (void)hipEventRecord(c->ev_order, st);
            (void)hipStreamWaitEvent(c->stream, c->ev_order, 0);
        }
    }
};

// mode 0 (SigG2): d_const = g~ affine G1 in the lazy R' form (24 words); mode 1 (SigG1): g~ Miller lines
// (68 x 72 words).
// Pairing kernels run one credential per lane pair (tower_pl.h).  Miller values go to SoA elements
// [0, n) of stride n.
static int cck_miller(int mode, size_t n, const uint32_t* d_prep, const uint32_t* d_flags, const uint32_t* d_const,
                      uint32_t* d_f, hipStream_t st) {
    return mode == 0 ? cck_miller_lz_g2(0, n, n, d_prep, d_flags, d_const, d_f, n, 0, nullptr, st)
                     : cck_miller_lz_g1(0, n, n, d_prep, d_flags, d_const, d_f, n, 0, nullptr, st);
}
// the RLC credentials (pair 0 only: their second pairs are folded, fold.hip) four per lane pair
// through the shared-squaring loop (k_miller4, 1 wave/SIMD): ceil(n / 4) Miller values, each the
// product of four pairs' (the RLC multiplies them all), over the twin layout (prep stride ps >= ceil(n / 2))
static int cck_miller_quad(int mode, size_t n, size_t ps, const uint32_t* d_prep, const uint32_t* d_flags, uint32_t* d_f,
                           size_t fstride, uint32_t* d_qcheck, hipStream_t st) {
    return mode == 0 ? cck_miller4_lz_g2(n, ps, d_prep, d_flags, d_f, fstride, 0, d_qcheck, st)
                     : cck_miller4_lz_g1(n, ps, d_prep, d_flags, d_f, fstride, 0, nullptr, st);
}

static inline int sig_bytes(int mode) { return mode == 0 ? 192 : 97; }
static inline int oth_bytes(int mode) { return mode == 0 ? 97 : 192; }
static inline int oth_group(int mode) { return mode == 0 ? 1 : 2; }
static inline int sig_group(int mode) { return mode == 0 ? 2 : 1; }
static inline size_t aff_words(int group) { return group == 1 ? 24 : 48; }

// the context's own workspaces: concurrency slot 0, and every single-slot entry point
static VerifyWork ctx_work(cc_ctx* c) {
    return VerifyWork(&c->prep, &c->flags, &c->fbuf, &c->vkb, &c->scratch, &c->pok_idx, &c->wide_prep, &c->wide_flags,
                      &c->wide_f);
}

static inline cc_ctx* primary(cc_ctx* c) { return c && !c->peers.empty() ? c->peers[0] : c; }
static inline const cc_ctx* primary(const cc_ctx* c) { return c && !c->peers.empty() ? c->peers[0] : c; }

#define HIPCK(x)                                  \
    do {                                          \
        if ((x) != hipSuccess) return CC_ERR_HIP; \
    } while (0)
#define KCK(x)                     \
    do {                           \
        if ((x) != 0) return CC_ERR_HIP; \
    } while (0)

extern "C" {

const char* cc_status_str(int s) {
    switch (s) {
        case CC_OK: return "ok";
        case CC_ERR_LEN: return "UnsupportedNoOfMessages";
        case CC_ERR_BASES_EXPS: return "UnequalNoOfBasesExponents";
        case CC_ERR_THRESHOLD: return "fewer entries than threshold";
        case CC_ERR_DECODE: return "bad buffer / size";
        case CC_ERR_HIP: return "HIP runtime error";
        case CC_ERR_RCCL: return "RCCL error";
        case CC_ERR_STATE: return "params/verkey not set";
        default: return "unknown";
    }
}

// CC_SRC_HASH: tools/src_hash.py over csrc/, the header, the Makefile and the flags (Makefile)
#ifndef CC_SRC_HASH
#define CC_SRC_HASH "unknown"
#endif
const char* cc_version(void) { return "coconut-mi355x 0.2.0 (gfx950) src " CC_SRC_HASH; }

static_assert(CC_RLC_PARTIAL_WORDS == RLC_PART_WORDS, "coconut_hip.h and rlc_part.h disagree");
int cc_rlc_partial_words(void) { return RLC_PART_WORDS; }

cc_status cc_ctx_create(int device, cc_group_mode mode, cc_ctx** out) {
    if (!out || (mode != CC_SIG_G2 && mode != CC_SIG_G1)) return CC_ERR_DECODE;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return CC_ERR_HIP;
    HIPCK(hipSetDevice(device));
    cc_ctx* c = new cc_ctx();
    c->device = device;
    c->mode = (int)mode;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return CC_ERR_HIP;
    }
    for (auto& e : c->ev) (void)hipEventCreate(&e);
    (void)hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->ev_fin, hipEventDisableTiming);
    {
        // high priority: a launch on the side stream gets its wave slots before a full launch on the
        // context stream fills the chip
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi) != hipSuccess) c->side = nullptr;
    }
    c->pool.recs.resize(1);
    c->pool.recs[0].w = ctx_work(c);  // slot 0: the context's own workspaces
    c->stage.resize(1);
    *out = c;
    return CC_OK;
}

cc_status cc_ctx_destroy(cc_ctx* c) {
    if (!c) return CC_OK;
    if (!c->peers.empty()) {
        for (size_t k = 0; k < c->comms.size(); k++) {
            (void)hipSetDevice(c->peers[k]->device);
            ncclCommDestroy(c->comms[k]);
        }
        for (cc_ctx* p : c->peers) cc_ctx_destroy(p);
        delete c;
        return CC_OK;
    }
    (void)hipSetDevice(c->device);
    drain_slots(c);
    (void)hipStreamSynchronize(c->stream);
    for (VerifySlot* v : c->vslots) {
        v->each([](DevBuf& b) { b.release(); });
        delete v;
    }
    c->vslots.clear();
    for (auto& r : c->pool.recs)
        if (r.done) (void)hipEventDestroy(r.done);
    c->pool.recs.clear();
    for (Staging& g : c->stage) g.release();
    DevBuf* bufs[] = {&c->gtilde_aff, &c->gtilde_lines, &c->gtilde_lz, &c->vk_aff, &c->vk_inf, &c->table, &c->table_inf,
                      &c->in_s1, &c->in_s2, &c->in_msgs, &c->in_vkX, &c->in_vkY, &c->prep, &c->flags,
                      &c->fbuf, &c->scratch, &c->verdicts, &c->gt, &c->vkb, &c->lag, &c->wide_prep, &c->wide_flags, &c->wide_f,
                      &c->rlc_key, &c->rlc_any, &c->rlc_part, &c->rlc_flag, &c->rlc_accept, &c->fin_f, &c->fin_scratch, &c->fin_prep, &c->fin_flags2, &c->fin_part, &c->pok_idx, &c->rlc_gath,
                      &c->rlc_pts, &c->rlc_dig, &c->rlc_work, &c->rlc_pw, &c->rlc_finf,
                      &c->iss_ids, &c->iss_aff, &c->iss_inf, &c->iss_table, &c->agg_scratch, &c->dev_err};
    for (auto* b : bufs) b->release();
    for (auto& b : c->in_aux) b.release();
    for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
    if (c->ev_order) (void)hipEventDestroy(c->ev_order);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_fin) (void)hipEventDestroy(c->ev_fin);
    if (c->side) (void)hipStreamDestroy(c->side);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return CC_OK;
}

cc_status cc_ctx_mode(const cc_ctx* c, int* m) {
    if (!c || !m) return CC_ERR_DECODE;
    *m = c->mode;
    return CC_OK;
}

cc_status cc_set_timing(cc_ctx* c, int enabled) {
    c = primary(c);  // a device set forwards to its first device
    if (!c) return CC_ERR_DECODE;
    c->timing = enabled != 0;
    return CC_OK;
}

cc_status cc_last_timing(const cc_ctx* c, float* a, float* b, float* d) {
    c = primary(c);  // a device set forwards to its first device
    if (!c) return CC_ERR_DECODE;
    if (a) *a = c->last_ms[0];
    if (b) *b = c->last_ms[1];
    if (d) *d = c->last_ms[2];
    return CC_OK;
}

static cc_status decode_points_host(cc_ctx* c, int group, size_t n, const uint8_t* bytes, uint32_t* d_out,
                                    uint32_t* d_inf) {
    size_t eb = group == 1 ? 97 : 192;
    DevBuf tmp;
    if (tmp.ensure(eb * n + 16)) return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(tmp.p, bytes, eb * n, hipMemcpyHostToDevice, c->stream));
    KCK(cck_decode_points(group, n, tmp.as<uint8_t>(), d_out, d_inf, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    tmp.release();
    return CC_OK;
}

static cc_status subgroup_host(cc_ctx* c, int group, size_t n, const uint8_t* bytes, uint8_t* status) {
    size_t eb = group == 1 ? 97 : 192;
    DevBuf tmp, st;
    if (tmp.ensure(eb * n + 16) || st.ensure(n + 16)) return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(tmp.p, bytes, eb * n, hipMemcpyHostToDevice, c->stream));
    KCK(cck_subgroup(group, n, tmp.as<uint8_t>(), st.as<uint8_t>(), c->stream));
    HIPCK(hipMemcpyAsync(status, st.p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return CC_OK;
}

// Shared-verkey tables: by default the widest of 22 / 20 / 18 / 16 / 14 / 12 / 10-bit windows whose q + 2
// bases' tables fit kVkTableBudget (4 GiB) and 40 % of the free HBM — a drop-in verifier must not claim a
// shared GPU's memory: config 2 (q = 6, 8 G1 bases) gets 18 bits (15 windows of 262,143 entries, 3.0 GB),
// config 3 (q = 16) 16 bits (1.8 GB); 16 / 15 / 12 mixed additions per scalar at 16 / 18 / 22 bits.  Wider
// tables (22 bits: 4.8 / 9.7 GB a G1 / G2 base, +1.2 % on config 2, profiles/r03/vkbits) are opt-in through
// cc_set_table_bits, which forces a width in [8, 22]; else 8-bit windows (32 x 255 entries, 0.8 / 1.6 MB a
// base); a failed wide allocation falls back to 8 bits.  On failure the caller leaves the context without
// a verkey.
static cc_status rebuild_tables(cc_ctx* c) {
    // bases for the fixed-base tables: Y~[0..q), g~ (PoK Schnorr base), X~ (RLC) -> q + 2 bases
    int og = oth_group(c->mode);
    size_t aw = aff_words(og);
    int nb = (int)c->q + 2;
    int wb = c->force_vk_bits;
    // the old table is released first so its memory counts as free
    c->table.release();
    const double fr = (double)free_hbm();
    if (!wb) {
        const double cap = std::min(0.4 * fr, kVkTableBudget);
        wb = 8;
        for (int w : {22, 20, 18, 16, 14, 12, 10})
            if ((double)nb * (double)tab_words(og, w) * 4.0 <= cap) {
                wb = w;
                break;
            }
    }
    // a forced width is refused up front when it exceeds the free HBM: hipMalloc does not reliably fail
    // for sizes above it (the runtime may over-commit), and a build kernel writing such a table would not
    // end well
    if (fr > 0 && (double)nb * (double)tab_words(og, wb) * 4.0 > 0.9 * fr) {
        if (c->force_vk_bits || wb == 8) return CC_ERR_HIP;
        wb = 8;
    }
    if (c->table.ensure((size_t)nb * tab_words(og, wb) * 4)) {
        (void)hipGetLastError();  // clear the failed allocation's error
        if (wb == 8 || c->force_vk_bits) return CC_ERR_HIP;
        wb = 8;
        if (c->table.ensure((size_t)nb * tab_words(og, wb) * 4)) return CC_ERR_HIP;
    }
    c->wbits = wb;
    c->vk_built_force = c->force_vk_bits;
    if (c->table_inf.ensure((size_t)nb * 4)) return CC_ERR_HIP;
    // [Y~..., g~, X~] are contiguous in vk_aff (X~ at 0, Y~ at 1..q, g~ at q+1, X~ again at q+2)
    HIPCK(hipMemcpyAsync(c->table_inf.p, c->vk_inf.as<uint32_t>() + 1, (size_t)nb * 4, hipMemcpyDeviceToDevice,
                         c->stream));
    DevBuf pw;
    if (pw.ensure((size_t)nb * tab_nwin(c->wbits) * (og == 1 ? 36 : 72) * 4)) return CC_ERR_HIP;
    KCK(cck_build_table(og, nb, c->wbits, c->vk_aff.as<uint32_t>() + aw, c->table_inf.as<uint32_t>(), pw.as<uint32_t>(),
                        c->table.as<uint32_t>(), 1, c->stream));
    // the RLC window pairs' fixed points P_w = (256^w) g~ (g~ = base q); an RLC finish still running on
    // another stream reads them, so the rewrite waits for it
    if (c->rlc_pw.ensure((size_t)PREP_SLOTS * 12 * RLC_WINDOWS * 4) || c->rlc_finf.ensure(RLC_WINDOWS))
        return CC_ERR_HIP;
    if (c->fin_recorded) HIPCK(hipStreamWaitEvent(c->stream, c->ev_fin, 0));
    KCK(cck_fold_fixed(c->mode, (int)c->q, c->table.as<uint32_t>(), c->wbits, c->table_inf.as<uint32_t>(),
                       c->rlc_pw.as<uint32_t>(), c->rlc_finf.as<uint8_t>(), c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    pw.release();
    return CC_OK;
}

// subgroup status of the verkey points (X~ || Y~, q + 1 encodings) and the context's g~: the RLC accepts
// only when all are in the order-r subgroup.  Depends on g~ as well, so cc_set_params recomputes it
// whenever it rebinds g~ under an existing verkey.
static cc_status refresh_vk_subgroup(cc_ctx* c, const uint8_t* vk_all, size_t q) {
    c->vk_subgroup = false;
    const int og = oth_group(c->mode);
    std::vector<uint8_t> st(q + 1);
    cc_status s = subgroup_host(c, og, q + 1, vk_all, st.data());
    if (s) return s;
    uint8_t gst = 0;
    s = subgroup_host(c, og, 1, c->gtilde_bytes.data(), &gst);
    if (s) return s;
    bool ok = gst == 2;
    for (size_t k = 0; k <= q; k++) ok = ok && st[k] == 2;
    c->vk_subgroup = ok;
    return CC_OK;
}

cc_status cc_set_params(cc_ctx* c, const uint8_t* g_tilde) {
    if (!c || !g_tilde) return CC_ERR_DECODE;
    if (!c->peers.empty()) {
        for (cc_ctx* p : c->peers) {
            cc_status s = cc_set_params(p, g_tilde);
            if (s) return s;
        }
        c->have_params = true;
        return CC_OK;
    }
    // the same g~ again (a caller re-binding its Params every batch): nothing to do
    if (c->have_params && c->gtilde_bytes.size() == (size_t)oth_bytes(c->mode) &&
        !memcmp(c->gtilde_bytes.data(), g_tilde, c->gtilde_bytes.size()))
        return CC_OK;
    HIPCK(hipSetDevice(c->device));
    drain_slots(c);  // concurrent verify batches read g~ and the tables rebuilt below
    c->have_params = false;  // until the decode below has succeeded
    c->gtilde_bytes.clear();
    int og = oth_group(c->mode);
    size_t aw = aff_words(og);
    if (c->gtilde_aff.ensure(aw * 4)) return CC_ERR_HIP;
    DevBuf inf;
    if (inf.ensure(4)) return CC_ERR_HIP;
    cc_status s = decode_points_host(c, og, 1, g_tilde, c->gtilde_aff.as<uint32_t>(), inf.as<uint32_t>());
    if (s) return s;
    HIPCK(hipMemcpy(&c->gtilde_inf, inf.p, 4, hipMemcpyDeviceToHost));
    c->gtilde_bytes.assign(g_tilde, g_tilde + oth_bytes(c->mode));
    inf.release();
    if (c->mode == 1) {
        if (c->gtilde_lines.ensure(68 * 72 * 4)) return CC_ERR_HIP;
        KCK(cck_gtilde_lines(c->gtilde_aff.as<uint32_t>(), c->gtilde_lines.as<uint32_t>(), c->stream));
        HIPCK(hipStreamSynchronize(c->stream));
    } else {
        if (c->gtilde_lz.ensure(aw * 4)) return CC_ERR_HIP;
        KCK(cck_lazy_form(2, c->gtilde_aff.as<uint32_t>(), c->gtilde_lz.as<uint32_t>(), c->stream));
        HIPCK(hipStreamSynchronize(c->stream));
    }
    c->have_params = true;
    if (c->have_vk) {
        // refresh g~ slot of the verkey block and its table
        HIPCK(hipMemcpy(c->vk_aff.as<uint32_t>() + (c->q + 1) * aw, c->gtilde_aff.p, aw * 4, hipMemcpyDeviceToDevice));
        HIPCK(hipMemcpy(c->vk_inf.as<uint32_t>() + (c->q + 1), &c->gtilde_inf, 4, hipMemcpyHostToDevice));
        cc_status st = refresh_vk_subgroup(c, c->vk_bytes.data(), c->q);
        if (!st) st = rebuild_tables(c);
        if (st) {
            c->have_vk = false;
            c->q = 0;
            c->vk_bytes.clear();
        }
        return st;
    }
    return CC_OK;
}

cc_status cc_set_verkey(cc_ctx* c, const uint8_t* X, const uint8_t* Y, size_t q) {
    if (!c || !X || (q && !Y) || q > 4096) return CC_ERR_DECODE;
    if (!c->have_params) return CC_ERR_STATE;
    if (!c->peers.empty()) {
        c->have_vk = false;
        c->q = 0;
        for (cc_ctx* p : c->peers) {
            cc_status s = cc_set_verkey(p, X, Y, q);
            if (s) return s;
        }
        c->q = q;
        c->have_vk = true;
        return CC_OK;
    }
    int og = oth_group(c->mode);
    size_t eb = (size_t)oth_bytes(c->mode), aw = aff_words(og);
    std::vector<uint8_t> all((q + 1) * eb);
    memcpy(all.data(), X, eb);
    if (q) memcpy(all.data() + eb, Y, q * eb);
    // the same verkey again, tables built at the width now asked for: nothing to rebuild (a caller
    // binding its verkey every batch, INTEGRATION.md §3, pays a byte compare, not a table build)
    if (c->have_vk && c->q == q && c->vk_built_force == c->force_vk_bits && c->vk_bytes == all) return CC_OK;
    // no verkey until every step below has succeeded: a failed call leaves the context refusing
    // verify / RLC / PoK calls with CC_ERR_STATE instead of running on a half-built table
    HIPCK(hipSetDevice(c->device));
    drain_slots(c);  // concurrent verify batches read the verkey and its tables
    c->have_vk = false;
    c->q = 0;
    c->vk_bytes.clear();
    if (c->vk_aff.ensure((q + 3) * aw * 4) || c->vk_inf.ensure((q + 3) * 4)) return CC_ERR_HIP;
    cc_status s = decode_points_host(c, og, q + 1, all.data(), c->vk_aff.as<uint32_t>(), c->vk_inf.as<uint32_t>());
    if (s) return s;
    HIPCK(hipMemcpy(c->vk_aff.as<uint32_t>() + (q + 1) * aw, c->gtilde_aff.p, aw * 4, hipMemcpyDeviceToDevice));
    HIPCK(hipMemcpy(c->vk_inf.as<uint32_t>() + (q + 1), &c->gtilde_inf, 4, hipMemcpyHostToDevice));
    HIPCK(hipMemcpy(c->vk_aff.as<uint32_t>() + (q + 2) * aw, c->vk_aff.p, aw * 4, hipMemcpyDeviceToDevice));
    HIPCK(hipMemcpy(c->vk_inf.as<uint32_t>() + (q + 2), c->vk_inf.p, 4, hipMemcpyDeviceToDevice));
    HIPCK(hipMemcpy(&c->X_inf, c->vk_inf.p, 4, hipMemcpyDeviceToHost));
    {
        cc_status s2 = refresh_vk_subgroup(c, all.data(), q);
        if (s2) return s2;
    }
    c->q = q;
    cc_status st = rebuild_tables(c);
    if (st) {
        c->q = 0;
        return st;
    }
    c->vk_bytes.swap(all);
    c->have_vk = true;
    return CC_OK;
}

cc_status cc_set_table_bits(cc_ctx* c, int verkey_bits, int issuer_bits) {
    if (!c || (verkey_bits != 0 && (verkey_bits < 8 || verkey_bits > 22)) ||
        (issuer_bits != 0 && (issuer_bits < 8 || issuer_bits > 16)))
        return CC_ERR_DECODE;
    for (cc_ctx* p : c->peers) {
        p->force_vk_bits = verkey_bits;
        p->force_iss_bits = issuer_bits;
    }
    c->force_vk_bits = verkey_bits;
    c->force_iss_bits = issuer_bits;
    return CC_OK;
}

cc_status cc_table_bits(const cc_ctx* c, int* verkey_bits, int* issuer_bits) {
    c = primary(c);
    if (!c) return CC_ERR_DECODE;
    if (verkey_bits) *verkey_bits = c->have_vk ? c->wbits : 0;
    if (issuer_bits) *issuer_bits = c->iss_n ? c->iss_wbits : 0;
    return CC_OK;
}

// Small batches run latency-bound: their Miller loops one wave per pair (n <= kWideMax: fexp_pl.hip
// k_wide_pairs -> k_miller_wide -> k_f12_reduce_wide) instead of one lane pair per credential (k_miller:
// one 2-pair loop's latency on a lone wave, ~7.5 ms for any batch up to a few thousand), and their
// final exponentiation one wave per credential (n <= kFexpWideMax: k_fexp1, 1.33 ms) instead of a lane
// quad (k_fexp_q: ~3 ms floor).  Both wide kernels hold one wave a SIMD: 1,024 waves a round of the
// chip, i.e. 512 credentials a round of the Miller path (0.8 ms a round: eight rounds at 4,096, 6.4 ms,
// under the pair-lane loop's ~7.5-9 ms latency there), 1,024 of the fexp (two rounds, ~2.7 ms, still
// under the quad kernel's floor at 2,048).  The shared-verkey prep takes its one-wave form up to
// kFexpWideMax, the PoK and per-credential-verkey preps up to kPrepWideMax.  Measured:
// profiles/r05/wide_spread, thresholds, miller_wide_pipe, fexp_thr.
// (the thresholds live in slots.h with the workspace sizes they decide; k_miller_wide2, two waves a
// pair, takes launches of <= kWide2Max = 256 pairs, i.e. <= 128 credentials: fexp_pl.hip)
using cc::slots::kFexpWideMax;
using cc::slots::kPrepWideMax;
using cc::slots::kWideMax;
// the context's own workspaces (slot 0) grown to n credentials; scratch: the PoK prep's per-proof table
// of d J (15 Jacobian points, <= 15 x 84 words: SigG1's lazy G2 points), and the one-wave fexp's
// (fexp_pl.hip k_fexp1: 72 slots of 12 words an element); the batched fexp (fexp_q.hip) keeps its chain
// in registers
static cc_status ensure_work(cc_ctx* c, size_t n) {
    const cc::slots::Sizes sz = cc::slots::verify_sizes(n, 0, (n * 15 * 84 + 72 * 12) * 4, 0);
    const VerifyWork w = ctx_work(c);
    if (w.short_of(sz) || c->verdicts.bytes < n)
        drain_slots(c);  // a concurrent batch may still read the buffers about to be reallocated
    for (int j = 0; j < VerifyWork::kN; j++)
        if (w.at(j)->ensure(sz.at(j))) return CC_ERR_HIP;
    if (c->verdicts.ensure(n)) return CC_ERR_HIP;
    return CC_OK;
}

// the three verify launches on device buffers (VerifyWork, slots.h); timing per phase when enabled.
// d_vkX == NULL: the shared verkey's tables; else one verkey per credential (d_vkX n x OtherGroup, d_vkY
// n x q x OtherGroup; the Straus MSM of pervk.hip, its scratch in w.vkb, sized by the caller)
// the batch's Miller values into w.fbuf (SoA stride n): n <= kWideMax one wave per pair, else the
// pair-lane loop (one lane pair per credential, both pairs with a shared squaring)
static cc_status launch_miller(cc_ctx* c, const VerifyWork& w, size_t n, hipStream_t st) {
    if (n <= kWideMax) {
        const size_t m = 2 * n;
        KCK(cck_wide_pairs(c->mode, n, n, w.prep->as<uint32_t>(), w.flags->as<uint32_t>(), c->gtilde_aff.as<uint32_t>(),
                           w.wprep->as<uint32_t>(), w.wflags->as<uint32_t>(), st));
        KCK(cck_miller_wide(m, w.wprep->as<uint32_t>(), w.wflags->as<uint32_t>(), w.wf->as<uint32_t>(), m, 0, st));
        KCK(cck_f12_reduce_wide(m, w.wf->as<uint32_t>(), w.fbuf->as<uint32_t>(), st));
        return CC_OK;
    }
    const uint32_t* cst = c->mode == 0 ? c->gtilde_lz.as<uint32_t>() : c->gtilde_lines.as<uint32_t>();
    KCK(cck_miller(c->mode, n, w.prep->as<uint32_t>(), w.flags->as<uint32_t>(), cst, w.fbuf->as<uint32_t>(), st));
    return CC_OK;
}
static cc_status launch_verify(cc_ctx* c, const VerifyWork& w, size_t n, size_t q, const uint8_t* d_s1,
                               const uint8_t* d_s2, const uint8_t* d_msgs, const uint8_t* d_vkX, const uint8_t* d_vkY,
                               uint8_t* d_verdicts, uint8_t* d_gt, hipStream_t st) {
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
    if (d_vkX)
        KCK(cck_prep_var(c->mode, n, (int)q, d_s1, d_s2, d_vkX, d_vkY, d_msgs, w.vkb->as<uint32_t>(),
                         w.prep->as<uint32_t>(), w.flags->as<uint32_t>(), n <= kPrepWideMax, st));
    else  // small batches: one wave per credential, the MSM's window terms over its lanes
        KCK((n <= kFexpWideMax ? cck_prep_wide : cck_prep)(c->mode, n, (int)q, d_s1, d_s2, d_msgs,
                                                       c->vk_aff.as<uint32_t>(), c->X_inf, c->table.as<uint32_t>(),
                                                       c->wbits, c->table_inf.as<uint32_t>(), w.prep->as<uint32_t>(),
                                                       w.flags->as<uint32_t>(), st));
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    cc_status ms = launch_miller(c, w, n, st);
    if (ms) return ms;
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    // n <= kFexpWideMax: one wave per credential (k_fexp1, its chain in w.scratch: 72 x 12 x n words)
    KCK(cck_fexp(n, w.fbuf->as<uint32_t>(), w.scratch->as<uint32_t>(), w.flags->as<uint32_t>(), d_verdicts, d_gt,
                 kFexpWideMax, st));
    if (c->timing) (void)hipEventRecord(c->ev[3], st);
    return CC_OK;
}

static void collect_timing(cc_ctx* c) {
    if (!c->timing) return;
    (void)hipEventSynchronize(c->ev[3]);
    for (int k = 0; k < 3; k++) (void)hipEventElapsedTime(&c->last_ms[k], c->ev[k], c->ev[k + 1]);
}

// The next concurrent slot (round-robin, slots.h Pool): its workspaces grown to the batch's sizes once
// its last batch is done, and stream st ordered after the context stream's queued work (tables, params,
// other entry points) and after that last batch.  The caller holds a SlotFence that records the slot's
// completion on st on every exit.
static cc_status slot_begin(cc_ctx* c, hipStream_t st, const cc::slots::Sizes& sz, int& k, VerifyWork& w) {
    k = c->pool.take();
    w = c->pool.recs[(size_t)k].w;
    const int rc = c->pool.begin(c->dev, k, sz, st, c->stream, c->ev_order);
    return rc == -2 ? CC_ERR_STATE : rc ? CC_ERR_HIP : CC_OK;
}

// the *_device verify calls: with one slot, ordered against everything on the context (StreamOrder);
// with K > 1 (cc_set_concurrency), on the next slot round-robin, ordered only after the context
// stream's queued work (tables, params) and that slot's previous batch.
static cc_status verify_device(cc_ctx* c, size_t n, size_t q, const uint8_t* d_s1, const uint8_t* d_s2,
                               const uint8_t* d_msgs, const uint8_t* d_vkX, const uint8_t* d_vkY, uint8_t* d_verdicts,
                               uint8_t* d_gt, hipStream_t st) {
    const size_t vkw = d_vkX ? cck_prep_var_words(c->mode, n, q) * 4 : 0;
    if (c->concurrency <= 1) {
        cc_status s = ensure_work(c, n);
        if (s) return s;
        if (d_vkX && c->vkb.bytes < vkw) drain_slots(c);  // slot 0's batch may still read it
        StreamOrder order(c, st);
        if (d_vkX && c->vkb.ensure(vkw)) return CC_ERR_HIP;
        return launch_verify(c, ctx_work(c), n, q, d_s1, d_s2, d_msgs, d_vkX, d_vkY, d_verdicts, d_gt, st);
    }
    // the slot sizes its own workspaces (slot 0's too): no ensure_work, which would grow slot 0 for a
    // batch landing on another slot and drain every slot in flight
    int k = 0;
    VerifyWork w;
    cc_status s = slot_begin(c, st, cc::slots::verify_sizes(n, vkw, 0, 0), k, w);
    if (s) return s;
    SlotFence fence(c->pool, c->dev, k, st);
    s = launch_verify(c, w, n, q, d_s1, d_s2, d_msgs, d_vkX, d_vkY, d_verdicts, d_gt, st);
    if (s) return s;
    return fence.close() ? CC_ERR_HIP : CC_OK;
}

cc_status cc_set_concurrency(cc_ctx* c, int slots) {
    if (!c || slots < 1 || slots > 8) return CC_ERR_DECODE;
    for (cc_ctx* p : c->peers) {
        cc_status s = cc_set_concurrency(p, slots);
        if (s) return s;
    }
    if (!c->peers.empty()) {
        c->concurrency = slots;
        return CC_OK;
    }
    HIPCK(hipSetDevice(c->device));
    drain_slots(c);
    while ((int)c->vslots.size() > slots - 1) {
        VerifySlot* v = c->vslots.back();
        c->vslots.pop_back();
        v->each([](DevBuf& b) { b.release(); });
        delete v;
        if (c->pool.recs.back().done) (void)hipEventDestroy(c->pool.recs.back().done);
        c->pool.recs.pop_back();
        c->stage.back().release();
        c->stage.pop_back();
    }
    if (!c->pool.recs[0].done) HIPCK(hipEventCreateWithFlags(&c->pool.recs[0].done, hipEventDisableTiming));
    while ((int)c->vslots.size() < slots - 1) {
        SlotPool::Rec r;
        if (hipEventCreateWithFlags(&r.done, hipEventDisableTiming) != hipSuccess) return CC_ERR_HIP;
        VerifySlot* v = new VerifySlot;
        r.w = v->work();
        c->vslots.push_back(v);
        c->pool.recs.push_back(r);
        c->stage.emplace_back();
    }
    c->concurrency = slots;
    c->pool.next = 0;
    return CC_OK;
}

cc_status cc_concurrency(const cc_ctx* c, int* slots) {
    if (!c || !slots) return CC_ERR_DECODE;
    *slots = c->concurrency;
    return CC_OK;
}

cc_status cc_verify_batch_device(cc_ctx* c, size_t n, size_t q, const uint8_t* d_s1, const uint8_t* d_s2,
                                 const uint8_t* d_msgs, uint8_t* d_verdicts, uint8_t* d_gt, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!d_s1 || !d_s2 || !d_verdicts))) return CC_ERR_DECODE;
    if (!c->have_params || !c->have_vk) return CC_ERR_STATE;
    if (q != c->q) return CC_ERR_LEN;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    cc_status s = verify_device(c, n, q, d_s1, d_s2, d_msgs, nullptr, nullptr, d_verdicts, d_gt, st);
    if (s) return s;
    if (c->timing) collect_timing(c);
    return CC_OK;
}

cc_status cc_verify_batch_pervk_device(cc_ctx* c, size_t n, size_t q, const uint8_t* d_s1, const uint8_t* d_s2,
                                       const uint8_t* d_msgs, const uint8_t* d_vkX, const uint8_t* d_vkY,
                                       uint8_t* d_verdicts, uint8_t* d_gt, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || q > 4096 || (n && (!d_s1 || !d_s2 || !d_vkX || !d_verdicts || (q && (!d_msgs || !d_vkY)))))
        return CC_ERR_DECODE;
    if (!c->have_params) return CC_ERR_STATE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    cc_status s = verify_device(c, n, q, d_s1, d_s2, d_msgs, d_vkX, d_vkY, d_verdicts, d_gt, st);
    if (s) return s;
    if (c->timing) collect_timing(c);
    return CC_OK;
}


// ---------------------------------------------------------------- RLC batch mode (rlc.hip)
static int fresh_seed(uint8_t seed[32]) {
    FILE* f = fopen("/dev/urandom", "rb");
    if (!f) return -1;
    size_t got = fread(seed, 1, 32, f);
    fclose(f);
    return got == 32 ? 0 : -1;
}

// The RLC partial's workspaces: prep SoA (twin layout), flags, Miller values, the product tree's scratch,
// the delta key, the fall-back flag word, the fold points, delta digits and fold workspace.
struct RlcWork {
    DevBuf *prep, *flags, *fbuf, *scratch, *key, *any, *pts, *dig, *work;
};
static RlcWork ctx_rlc_work(cc_ctx* c) {
    return {&c->prep, &c->flags, &c->fbuf, &c->scratch, &c->rlc_key, &c->rlc_any, &c->rlc_pts, &c->rlc_dig, &c->rlc_work};
}
// sizes for n credentials; a concurrency slot whose buffers must grow waits for its last batch first
static int rlc_ensure(cc_ctx* c, const RlcWork& r, size_t n, SlotPool::Rec* sl) {
    const size_t PS = (n + 1) / 2, N = (n + 3) / 4;
    const size_t prep_b = (size_t)PREP_SLOTS * 12 * 4 * std::max(PS, n), flags_b = n * 4, fbuf_b = N * 144 * 4,
                 scr_b = ((N + 1) / 2) * 144 * 4 + n * 12 * 4 * 72, pts_b = n * 48 * 4, dig_b = 16 * n,
                 work_b = cck_fold_words(c->mode, n) * 4;
    const bool grow = r.prep->bytes < prep_b || r.flags->bytes < flags_b || r.fbuf->bytes < fbuf_b ||
                      r.scratch->bytes < scr_b || r.key->bytes < 32 || r.any->bytes < 4 || r.pts->bytes < pts_b ||
                      r.dig->bytes < dig_b || r.work->bytes < work_b;
    if (!grow) return 0;
    if (sl && sl->recorded && hipEventSynchronize(sl->done) != hipSuccess) return -1;
    return r.prep->ensure(prep_b) || r.flags->ensure(flags_b) || r.fbuf->ensure(fbuf_b) || r.scratch->ensure(scr_b) ||
           r.key->ensure(32) || r.any->ensure(4) || r.pts->ensure(pts_b) || r.dig->ensure(dig_b) ||
           r.work->ensure(work_b);
}

static cc_status launch_rlc_partial(cc_ctx* c, const RlcWork& w, size_t n, size_t q, uint64_t base_index,
                                    const uint8_t* seed32, const uint8_t* d_s1, const uint8_t* d_s2,
                                    const uint8_t* d_msgs, uint32_t* d_partial, hipStream_t st, Staging* stage) {
    const size_t PS = (n + 1) / 2;  // prep SoA stride (the twin layout: credentials 2 t, 2 t + 1 at element t)
    const size_t N = (n + 3) / 4;   // Miller values (four credentials' pairs each, k_miller4)
    if (stage) {  // a concurrency slot: through its pinned ring, so the host does not wait for the stream
        KCK(stage->upload(w.key->p, seed32, 32, st));
    } else {  // pageable source: the copy is staged before the call returns
        HIPCK(hipMemcpyAsync(w.key->p, seed32, 32, hipMemcpyHostToDevice, st));
    }
    HIPCK(hipMemsetAsync(w.any->p, 0, 4, st));
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
    auto prep_part = [&](int part) {
        return cck_prep_rlc(c->mode, part, n, PS, (int)q, base_index, w.key->as<uint32_t>(), d_s1, d_s2, d_msgs,
                            c->table.as<uint32_t>(), c->wbits, c->table_inf.as<uint32_t>(), w.prep->as<uint32_t>(),
                            w.flags->as<uint32_t>(), w.any->as<uint32_t>(), w.pts->as<uint32_t>(),
                            w.dig->as<int8_t>(), st);
    };
    KCK(prep_part(0));  // decode, subgroup checks, the fold's inputs
    if (!c->vk_subgroup) {
        // a verkey / g~ point outside the subgroup: the linear-combination argument does not hold,
        // so the batch is never accepted here and the caller verifies per credential (exact)
        static const uint32_t one = 1;
        HIPCK(hipMemcpyAsync(w.any->p, &one, 4, hipMemcpyHostToDevice, st));
    }
    // The second pairs fold into 16 window sums S_w (fold.hip).  The fold's short kernels run alone
    // (behind a full launch each would wait milliseconds for a free slot); the window sums (16 waves)
    // then run on the high-priority side stream beside the delta MSM and land in the partial's window
    // section; their pairs e(S_w, P_w) are evaluated in the finish, once per batch over every shard
    // (rlc_part.h), so the credentials' two-per-loop Miller launch stays at (n + 1) / 2 loops (2,048
    // waves at 131,072 credentials: the chip's wave slots).
    KCK(cck_fold(c->mode, n, w.dig->as<int8_t>(), w.pts->as<uint32_t>(), w.work->as<uint32_t>(), st));
    hipStream_t side = c->side ? c->side : st;
    if (side != st) {
        HIPCK(hipEventRecord(c->ev_fork, st));
        HIPCK(hipStreamWaitEvent(side, c->ev_fork, 0));
    }
    KCK(cck_fold_window(c->mode, n, w.work->as<uint32_t>(), d_partial, side));
    KCK(prep_part(1));  // delta X~ + sum (delta m_j) Y~_j
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    // SigG2: sigma_1's subgroup test comes from this loop's T (a failure raises rlc_any: fallback)
    KCK(cck_miller_quad(c->mode, n, PS, w.prep->as<uint32_t>(), w.flags->as<uint32_t>(), w.fbuf->as<uint32_t>(), N,
                        c->mode == 0 ? w.any->as<uint32_t>() : nullptr, st));
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    KCK(cck_rlc_reduce(N, w.fbuf->as<uint32_t>(), w.scratch->as<uint32_t>(), w.any->as<uint32_t>(), d_partial,
                       st));
    if (side != st) {  // the window section is part of the partial: the call ends when both are written
        HIPCK(hipEventRecord(c->ev_join, side));
        HIPCK(hipStreamWaitEvent(st, c->ev_join, 0));
    }
    if (c->timing) {
        (void)hipEventRecord(c->ev[3], st);
        collect_timing(c);
    }
    return CC_OK;
}

cc_status cc_rlc_partial_device(cc_ctx* c, size_t n, size_t q, uint64_t base_index, const uint8_t* seed32,
                                const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs, uint32_t* d_partial,
                                void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !seed32 || !d_partial || (n && (!d_s1 || !d_s2 || (q && !d_msgs)))) return CC_ERR_DECODE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!c->have_params || !c->have_vk) return CC_ERR_STATE;
    if (q != c->q) return CC_ERR_LEN;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (!n) {
        // empty shard (a batch smaller than the rank count): the neutral partial — Fp12 one (Montgomery
        // one in slot 0, zeros elsewhere), a clear fall-back flag and 16 identity window sums — so every
        // rank still joins the all-gather and the product over ranks is unchanged
        static const uint32_t kOne[12] = {0x03a9fb84u, 0xc57400d2u, 0x629c4a23u, 0x6147acdeu, 0x7e6d26cbu, 0x6b0f4b0bu,
                                          0xc2b7d6e1u, 0x91ecbde7u, 0x4fdd80b8u, 0xd56a23c3u, 0xf3a0d636u, 0x13317c30u};
        static const std::vector<uint32_t> kNeutral = [] {
            std::vector<uint32_t> v(RLC_PART_WORDS, 0u);
            memcpy(v.data(), kOne, sizeof(kOne));
            for (int w = 0; w < RLC_WINDOWS; w++) v[RLC_WIN_OFF + RLC_WIN_WORDS * w + 48] = 1u;
            return v;
        }();
        HIPCK(hipMemcpyAsync(d_partial, kNeutral.data(), RLC_PART_WORDS * 4, hipMemcpyHostToDevice, st));
        return CC_OK;
    }
    if (c->concurrency > 1) {  // the next concurrency slot (cc_set_concurrency): its own workspaces
        int k = 0;
        VerifyWork w;
        cc_status s = slot_begin(c, st, cc::slots::verify_sizes(n, 0, 0, 0), k, w);
        if (s) return s;
        SlotFence fence(c->pool, c->dev, k, st);
        VerifySlot* sl = k ? c->vslots[(size_t)k - 1] : nullptr;
        RlcWork r = sl ? RlcWork{&sl->prep, &sl->flags, &sl->fbuf, &sl->scratch, &sl->rkey, &sl->rany, &sl->rpts,
                                 &sl->rdig, &sl->rwork}
                       : ctx_rlc_work(c);
        if (rlc_ensure(c, r, n, &c->pool.recs[(size_t)k])) return CC_ERR_HIP;
        s = launch_rlc_partial(c, r, n, q, base_index, seed32, d_s1, d_s2, d_msgs, d_partial, st, &c->stage[(size_t)k]);
        if (s) return s;
        return fence.close() ? CC_ERR_HIP : CC_OK;
    }
    drain_slots(c);  // concurrent batches (cc_set_concurrency) may still use the buffers sized below
    cc_status s = ensure_work(c, n);
    if (s) return s;
    RlcWork r = ctx_rlc_work(c);
    if (rlc_ensure(c, r, n, nullptr)) return CC_ERR_HIP;
    StreamOrder order(c, st);
    return launch_rlc_partial(c, r, n, q, base_index, seed32, d_s1, d_s2, d_msgs, d_partial, st, nullptr);
}

cc_status cc_rlc_finish_device(cc_ctx* c, size_t nparts, const uint32_t* d_partials, uint8_t* d_accept,
                               uint8_t* d_gt, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !nparts || nparts > kMaxParts || !d_partials || !d_accept) return CC_ERR_DECODE;
    if (!c->have_params || !c->have_vk) return CC_ERR_STATE;  // the window pairs' P_w come with the verkey
    HIPCK(hipSetDevice(c->device));
    // the finish owns its buffers (Fp12 values, window-pair operands, fexp scratch, flag) and reads only
    // the verkey's P_w, so it is NOT ordered against the context's stream: on a caller stream it may
    // overlap the next batch's cc_rlc_partial_device (the caller orders d_partials itself).  Finishes of
    // one context are ordered among themselves (ev_fin): two finishes on different streams never share
    // the buffers at the same time, whichever engines or streams issue them; a verkey change waits for
    // the last finish before it rewrites P_w.
    const size_t k = nparts, NW = (size_t)RLC_WINDOWS * k, NF = k + NW;
    if (c->rlc_flag.ensure(4) || c->fin_f.ensure(NF * 144 * 4) ||
        c->fin_scratch.ensure(std::max(((NF + 1) / 2) * 144 * 4, (size_t)2 * 72 * 12 * 4)) ||
        c->fin_prep.ensure((size_t)PREP_SLOTS * 12 * NW * 4) || c->fin_flags2.ensure(NW * 4) ||
        c->fin_part.ensure(RLC_PART_WORDS * 4))
        return CC_ERR_HIP;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (c->fin_recorded) HIPCK(hipStreamWaitEvent(st, c->ev_fin, 0));
    // the partials' products (elements 0 .. k-1) and every shard's 16 window pairs e(S_w, P_w), one wave
    // each (latency-bound: one loop's length for any k up to 16 GPUs), to elements k .. 17 k - 1; the
    // product tree multiplies all 17 k; one final exponentiation, whose flag (a sigma was the identity or
    // outside the subgroup somewhere) forces a reject
    KCK(cck_rlc_gather(c->mode, k, d_partials, c->rlc_pw.as<uint32_t>(), c->rlc_finf.as<uint8_t>(),
                       c->fin_f.as<uint32_t>(), NF, c->fin_prep.as<uint32_t>(), c->fin_flags2.as<uint32_t>(),
                       c->rlc_flag.as<uint32_t>(), st));
    KCK(cck_miller_wide(NW, c->fin_prep.as<uint32_t>(), c->fin_flags2.as<uint32_t>(), c->fin_f.as<uint32_t>(), NF, k,
                        st));
    KCK(cck_rlc_reduce(NF, c->fin_f.as<uint32_t>(), c->fin_scratch.as<uint32_t>(), c->rlc_flag.as<uint32_t>(),
                       c->fin_part.as<uint32_t>(), st));
    KCK(cck_fexp(1, c->fin_part.as<uint32_t>(), c->fin_scratch.as<uint32_t>(), c->fin_part.as<uint32_t>() + RLC_FLAG,
                 d_accept, d_gt, 1, st));
    HIPCK(hipEventRecord(c->ev_fin, st));
    c->fin_recorded = true;
    return CC_OK;
}

// single-GPU RLC over host buffers: returns accept (1) / reject (0) in *accept
static cc_status rlc_host(cc_ctx* c, size_t n, size_t q, uint8_t* accept) {
    uint8_t seed[32];
    if (fresh_seed(seed)) return CC_ERR_HIP;
    if (c->rlc_part.ensure(RLC_PART_WORDS * 4) || c->rlc_accept.ensure(1)) return CC_ERR_HIP;
    cc_status s = cc_rlc_partial_device(c, n, q, 0, seed, c->in_s1.as<uint8_t>(), c->in_s2.as<uint8_t>(),
                                        c->in_msgs.as<uint8_t>(), c->rlc_part.as<uint32_t>(), c->stream);
    if (s) return s;
    s = cc_rlc_finish_device(c, 1, c->rlc_part.as<uint32_t>(), c->rlc_accept.as<uint8_t>(), nullptr, c->stream);
    if (s) return s;
    HIPCK(hipMemcpyAsync(accept, c->rlc_accept.p, 1, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return CC_OK;
}

static cc_status multi_verify(cc_ctx* c, size_t n, size_t q, const uint8_t* s1, const uint8_t* s2,
                              const uint8_t* msgs, const uint8_t* vkX, const uint8_t* vkY, uint8_t* verdicts,
                              uint8_t* gt, int rlc);

cc_status cc_verify_batch(cc_ctx* c, size_t n, size_t q, const uint8_t* s1, const uint8_t* s2, const uint8_t* msgs,
                          const uint8_t* vkX, const uint8_t* vkY, uint8_t* verdicts, uint8_t* gt, int rlc) {
    if (!c || (n && (!s1 || !s2 || !verdicts || (q && !msgs)))) return CC_ERR_DECODE;
    if (!c->have_params) return CC_ERR_STATE;
    const bool per_vk = vkX != nullptr;
    if (per_vk && ((q && !vkY) || q > 4096)) return CC_ERR_DECODE;
    if (!per_vk) {
        if (!c->have_vk) return CC_ERR_STATE;
        if (q != c->q) return CC_ERR_LEN;
    }
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    if (!c->peers.empty()) return multi_verify(c, n, q, s1, s2, msgs, vkX, vkY, verdicts, gt, rlc);
    HIPCK(hipSetDevice(c->device));
    drain_slots(c);  // concurrent device batches still using slot 0's workspaces (cc_set_concurrency)
    size_t sb = (size_t)sig_bytes(c->mode), ob = (size_t)oth_bytes(c->mode);
    if (c->in_s1.ensure(n * sb) || c->in_s2.ensure(n * sb) || c->in_msgs.ensure(n * q * 48 + 16) ||
        c->verdicts.ensure(n) || (gt && c->gt.ensure(n * 576)))
        return CC_ERR_HIP;
    cc_status s = ensure_work(c, n);
    if (s) return s;
    hipStream_t st = c->stream;
    HIPCK(hipMemcpyAsync(c->in_s1.p, s1, n * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->in_s2.p, s2, n * sb, hipMemcpyHostToDevice, st));
    if (q) HIPCK(hipMemcpyAsync(c->in_msgs.p, msgs, n * q * 48, hipMemcpyHostToDevice, st));
    const uint8_t* d_msgs = c->in_msgs.as<uint8_t>();
    if (rlc && !per_vk && !gt) {
        // whole-batch check; on reject (a bad or identity credential somewhere) fall through to the
        // per-credential path so every verdict equals the reference's
        uint8_t accept = 0;
        s = rlc_host(c, n, q, &accept);
        if (s) return s;
        if (accept) {
            memset(verdicts, 1, n);
            return CC_OK;
        }
    }
    if (per_vk) {
        if (c->in_vkX.ensure(n * ob) || c->in_vkY.ensure(n * q * ob + 16) ||
            c->vkb.ensure(cck_prep_var_words(c->mode, n, q) * 4))
            return CC_ERR_HIP;
        HIPCK(hipMemcpyAsync(c->in_vkX.p, vkX, n * ob, hipMemcpyHostToDevice, st));
        if (q) HIPCK(hipMemcpyAsync(c->in_vkY.p, vkY, n * q * ob, hipMemcpyHostToDevice, st));
    }
    s = launch_verify(c, ctx_work(c), n, q, c->in_s1.as<uint8_t>(),
                      c->in_s2.as<uint8_t>(), d_msgs, per_vk ? c->in_vkX.as<uint8_t>() : nullptr,
                      per_vk ? c->in_vkY.as<uint8_t>() : nullptr, c->verdicts.as<uint8_t>(),
                      gt ? c->gt.as<uint8_t>() : nullptr, st);
    if (s) return s;
    HIPCK(hipMemcpyAsync(verdicts, c->verdicts.p, n, hipMemcpyDeviceToHost, st));
    if (gt) HIPCK(hipMemcpyAsync(gt, c->gt.p, n * 576, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    collect_timing(c);
    return CC_OK;
}

cc_status cc_fixed_base_mul(cc_ctx* c, int group, const uint8_t* base, size_t n, const uint8_t* scalars,
                            uint8_t* out) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !base || (n && (!scalars || !out)) || (group != 1 && group != 2)) return CC_ERR_DECODE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    size_t eb = group == 1 ? 97 : 192, aw = aff_words(group);
    hipStream_t st = c->stream;
    DevBuf aff, inf, pw, table, ks, o;
    if (aff.ensure(aw * 4) || inf.ensure(4) || pw.ensure(tab_nwin(8) * (group == 1 ? 36 : 72) * 4) ||
        table.ensure(tab_words(group, 8) * 4) || ks.ensure(n * 48) || o.ensure(n * eb))
        return CC_ERR_HIP;
    cc_status s = decode_points_host(c, group, 1, base, aff.as<uint32_t>(), inf.as<uint32_t>());
    if (s) return s;
    uint32_t binf = 0;
    HIPCK(hipMemcpy(&binf, inf.p, 4, hipMemcpyDeviceToHost));
    KCK(cck_build_table(group, 1, 8, aff.as<uint32_t>(), inf.as<uint32_t>(), pw.as<uint32_t>(), table.as<uint32_t>(), 0,
                        st));
    HIPCK(hipMemcpyAsync(ks.p, scalars, n * 48, hipMemcpyHostToDevice, st));
    KCK(cck_fixed_mul(group, n, ks.as<uint8_t>(), table.as<uint32_t>(), binf, o.as<uint8_t>(), st));
    HIPCK(hipMemcpyAsync(out, o.p, n * eb, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    return CC_OK;
}

// Lagrange-weighted MSMs: windowed Straus over variable bases (aggregate.hip k_msm_straus)
static cc_status agg_scratch(cc_ctx* c, int group, size_t ntask, size_t t) {
    return c->agg_scratch.ensure(ntask * cck_straus_words(group, t) * 4 + 64) ? CC_ERR_HIP : CC_OK;
}

static cc_status launch_sig_aggregate(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                      const uint8_t* d_s1, const uint8_t* d_s2, uint8_t* d_o1, uint8_t* d_o2,
                                      hipStream_t st) {
    const size_t sb = (size_t)sig_bytes(c->mode);
    const int sg = sig_group(c->mode);
    if (c->lag.ensure(n * t * 32 + 32)) return CC_ERR_HIP;
    cc_status s = agg_scratch(c, sg, n, t);
    if (s) return s;
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
    KCK(cck_lagrange(n, len, t, d_ids, c->lag.as<uint32_t>(), st));
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    KCK(cck_msm_straus(sg, n, t, d_s2, len * sb, 0, sb, c->lag.as<uint32_t>(), 1, c->agg_scratch.as<uint32_t>(), d_o2, st));
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    // sigma_1 = sigs[0].sigma_1 (signature.rs:452): strided device copy of entry 0
    KCK(cck_copy_rows(n, sb, d_s1, len * sb, d_o1, st));
    if (c->timing) (void)hipEventRecord(c->ev[3], st);
    return CC_OK;
}

cc_status cc_signature_aggregate_batch_device(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                              const uint8_t* d_s1, const uint8_t* d_s2, uint8_t* d_out_s1,
                                              uint8_t* d_out_s2, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!d_ids || !d_s1 || !d_s2 || !d_out_s1 || !d_out_s2))) return CC_ERR_DECODE;
    if (len > kMaxIds) return CC_ERR_DECODE;
    if (len < t || len == 0) return CC_ERR_THRESHOLD;  // reference: assert!(sigs.len() >= threshold)
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    StreamOrder order(c, st);
    cc_status s = launch_sig_aggregate(c, n, len, t, d_ids, d_s1, d_s2, d_out_s1, d_out_s2, st);
    if (s) return s;
    if (c->timing) collect_timing(c);
    return CC_OK;
}

cc_status cc_signature_aggregate_batch(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* ids,
                                       const uint8_t* s1, const uint8_t* s2, uint8_t* out_s1, uint8_t* out_s2) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!ids || !s1 || !s2 || !out_s1 || !out_s2))) return CC_ERR_DECODE;
    if (len > kMaxIds) return CC_ERR_DECODE;
    if (len < t || len == 0) return CC_ERR_THRESHOLD;  // reference: assert!(sigs.len() >= threshold) + sigs[0]
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    size_t sb = (size_t)sig_bytes(c->mode);
    hipStream_t st = c->stream;
    DevBuf& d_ids = c->in_aux[0];
    DevBuf& d_pts = c->in_aux[1];
    DevBuf& d_out = c->in_aux[2];
    DevBuf& d_p1 = c->in_aux[3];
    DevBuf& d_o1 = c->in_aux[4];
    if (d_ids.ensure(n * len * 8) || d_pts.ensure(n * len * sb) || d_out.ensure(n * sb) || d_p1.ensure(n * len * sb) ||
        d_o1.ensure(n * sb))
        return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(d_ids.p, ids, n * len * 8, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_pts.p, s2, n * len * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_p1.p, s1, n * len * sb, hipMemcpyHostToDevice, st));
    cc_status s = launch_sig_aggregate(c, n, len, t, d_ids.as<uint64_t>(), d_p1.as<uint8_t>(), d_pts.as<uint8_t>(),
                                       d_o1.as<uint8_t>(), d_out.as<uint8_t>(), st);
    if (s) return s;
    HIPCK(hipMemcpyAsync(out_s2, d_out.p, n * sb, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(out_s1, d_o1.p, n * sb, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    return CC_OK;
}

cc_status cc_verkey_aggregate_batch(cc_ctx* c, size_t n, size_t len, size_t t, size_t q, const uint64_t* ids,
                                    const uint8_t* X, const uint8_t* Y, uint8_t* outX, uint8_t* outY) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!ids || !X || !outX || (q && (!Y || !outY))))) return CC_ERR_DECODE;
    if (len > kMaxIds) return CC_ERR_DECODE;
    if (len < t || len == 0) return CC_ERR_THRESHOLD;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    size_t ob = (size_t)oth_bytes(c->mode);
    int og = oth_group(c->mode);
    hipStream_t st = c->stream;
    DevBuf& d_ids = c->in_aux[0];
    DevBuf& d_X = c->in_aux[1];
    DevBuf& d_Y = c->in_aux[3];
    DevBuf& d_oX = c->in_aux[2];
    DevBuf& d_oY = c->in_aux[4];
    size_t ntask_y = n * q;
    size_t maxtask = ntask_y > n ? ntask_y : n;
    if (d_ids.ensure(n * len * 8) || d_X.ensure(n * len * ob) || d_Y.ensure(n * len * q * ob + 16) ||
        d_oX.ensure(n * ob) || d_oY.ensure(ntask_y * ob + 16) || c->lag.ensure(n * t * 32 + 32))
        return CC_ERR_HIP;
    cc_status s = agg_scratch(c, og, maxtask, t);
    if (s) return s;
    HIPCK(hipMemcpyAsync(d_ids.p, ids, n * len * 8, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_X.p, X, n * len * ob, hipMemcpyHostToDevice, st));
    if (q) HIPCK(hipMemcpyAsync(d_Y.p, Y, n * len * q * ob, hipMemcpyHostToDevice, st));
    KCK(cck_lagrange(n, len, t, d_ids.as<uint64_t>(), c->lag.as<uint32_t>(), st));
    KCK(cck_msm_straus(og, n, t, d_X.as<uint8_t>(), len * ob, 0, ob, c->lag.as<uint32_t>(), 1,
                       c->agg_scratch.as<uint32_t>(), d_oX.as<uint8_t>(), st));
    if (q)
        KCK(cck_msm_straus(og, ntask_y, t, d_Y.as<uint8_t>(), len * q * ob, ob, q * ob, c->lag.as<uint32_t>(), q,
                           c->agg_scratch.as<uint32_t>(), d_oY.as<uint8_t>(), st));
    HIPCK(hipMemcpyAsync(outX, d_oX.p, n * ob, hipMemcpyDeviceToHost, st));
    if (q) HIPCK(hipMemcpyAsync(outY, d_oY.p, ntask_y * ob, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    return CC_OK;
}

// ---------------------------------------------------------------- codec: subgroup membership (§8(f) row 1)
cc_status cc_subgroup_check(cc_ctx* c, int group, size_t n, const uint8_t* points, uint8_t* status) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (group != 1 && group != 2) || (n && (!points || !status))) return CC_ERR_DECODE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    return subgroup_host(c, group, n, points, status);
}

// ---------------------------------------------------------------- hash-to-curve (§8(f) row 2)
static cc_status stage_messages(cc_ctx* c, size_t n, const uint8_t* data, const uint64_t* offsets, DevBuf& d_data,
                                DevBuf& d_off) {
    if (offsets[0] != 0) return CC_ERR_DECODE;
    for (size_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i]) return CC_ERR_DECODE;
    const size_t total = offsets[n];
    if (total && !data) return CC_ERR_DECODE;
    if (d_data.ensure(total + 16) || d_off.ensure((n + 1) * 8)) return CC_ERR_HIP;
    if (total) HIPCK(hipMemcpyAsync(d_data.p, data, total, hipMemcpyHostToDevice, c->stream));
    HIPCK(hipMemcpyAsync(d_off.p, offsets, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    return CC_OK;
}

cc_status cc_hash_to_curve(cc_ctx* c, int group, size_t n, const uint8_t* data, const uint64_t* offsets, uint8_t* out) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (group != 1 && group != 2) || (n && (!offsets || !out))) return CC_ERR_DECODE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    const size_t eb = group == 1 ? 97 : 192;
    DevBuf d_data, d_off, d_out, d_fail;
    cc_status s = stage_messages(c, n, data, offsets, d_data, d_off);
    if (s) return s;
    if (d_out.ensure(n * eb) || d_fail.ensure(4)) return CC_ERR_HIP;
    HIPCK(hipMemsetAsync(d_fail.p, 0, 4, c->stream));
    KCK(cck_hash_to_curve(group, n, d_data.as<uint8_t>(), d_off.as<uint64_t>(), d_out.as<uint8_t>(),
                          d_fail.as<uint32_t>(), c->stream));
    uint32_t fail = 0;
    HIPCK(hipMemcpyAsync(out, d_out.p, n * eb, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipMemcpyAsync(&fail, d_fail.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return fail ? CC_ERR_DECODE : CC_OK;  // 4,096 failed tries (probability ~2^-4096)
}

cc_status cc_hash_msg(cc_ctx* c, size_t n, const uint8_t* data, const uint64_t* offsets, uint8_t* out48) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!offsets || !out48))) return CC_ERR_DECODE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    DevBuf d_data, d_off, d_out;
    cc_status s = stage_messages(c, n, data, offsets, d_data, d_off);
    if (s) return s;
    if (d_out.ensure(n * 48)) return CC_ERR_HIP;
    KCK(cck_shake256_48(n, d_data.as<uint8_t>(), d_off.as<uint64_t>(), d_out.as<uint8_t>(), c->stream));
    HIPCK(hipMemcpyAsync(out48, d_out.p, n * 48, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return CC_OK;
}

// ---------------------------------------------------------------- issuance (§8(f) row 3)
// h_r = compute_h(commitment_r, known_r) for every request, on the device (hash.hip)
static cc_status compute_h_batch(cc_ctx* c, size_t n, size_t q, size_t k, const uint8_t* comm, const uint8_t* known,
                                 DevBuf& d_h) {
    const size_t sb = (size_t)sig_bytes(c->mode), kn = q - k, len = sb + 48 * kn;
    std::vector<uint8_t> data(n * len);
    std::vector<uint64_t> off(n + 1);
    for (size_t r = 0; r < n; r++) {
        memcpy(&data[r * len], comm + r * sb, sb);
        if (kn) memcpy(&data[r * len + sb], known + r * kn * 48, kn * 48);
        off[r] = r * len;
    }
    off[n] = n * len;
    DevBuf d_data, d_off, d_fail;
    cc_status s = stage_messages(c, n, data.data(), off.data(), d_data, d_off);
    if (s) return s;
    if (d_h.ensure(n * sb) || d_fail.ensure(4)) return CC_ERR_HIP;
    HIPCK(hipMemsetAsync(d_fail.p, 0, 4, c->stream));
    // the reference hashes commitment.to_bytes() and the known messages' to_bytes() (canonical)
    KCK(cck_h_input_canon(sig_group(c->mode), n, len, (int)kn, d_data.as<uint8_t>(), c->stream));
    KCK(cck_hash_to_curve(sig_group(c->mode), n, d_data.as<uint8_t>(), d_off.as<uint64_t>(), d_h.as<uint8_t>(),
                          d_fail.as<uint32_t>(), c->stream));
    uint32_t fail = 0;
    HIPCK(hipMemcpyAsync(&fail, d_fail.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return fail ? CC_ERR_DECODE : CC_OK;  // as cc_hash_to_curve
}

cc_status cc_blind_sign_batch(cc_ctx* c, size_t n, size_t q, size_t k, const uint8_t* commitment, const uint8_t* known,
                              const uint8_t* ciphertexts, const uint8_t* x, const uint8_t* y, uint8_t* out_h,
                              uint8_t* out_c1, uint8_t* out_c2) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !x || (q && !y) || (n && (!commitment || !out_h || !out_c1 || !out_c2 || (k && !ciphertexts) ||
                                        (q > k && !known))))
        return CC_ERR_DECODE;
    if (q > kMaxQ) return CC_ERR_DECODE;
    if (k > q) return CC_ERR_LEN;  // reference: hidden + known == y.len() (assert_eq!)
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    const size_t sb = (size_t)sig_bytes(c->mode), t = k + 1;
    const int sg = sig_group(c->mode);
    hipStream_t st = c->stream;
    DevBuf d_h, d_cts, d_known, d_x, d_y, d_pts, d_sc, d_out;
    cc_status s = compute_h_batch(c, n, q, k, commitment, known, d_h);
    if (s) return s;
    if (d_cts.ensure(n * k * 2 * sb + 16) || d_known.ensure(n * (q - k) * 48 + 16) || d_x.ensure(48) ||
        d_y.ensure(q * 48 + 16) || d_pts.ensure(2 * n * t * sb) || d_sc.ensure(2 * n * t * 32) ||
        d_out.ensure(2 * n * sb))
        return CC_ERR_HIP;
    s = agg_scratch(c, sg, 2 * n, t);
    if (s) return s;
    if (k) HIPCK(hipMemcpyAsync(d_cts.p, ciphertexts, n * k * 2 * sb, hipMemcpyHostToDevice, st));
    if (q > k) HIPCK(hipMemcpyAsync(d_known.p, known, n * (q - k) * 48, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_x.p, x, 48, hipMemcpyHostToDevice, st));
    if (q) HIPCK(hipMemcpyAsync(d_y.p, y, q * 48, hipMemcpyHostToDevice, st));
    KCK(cck_blind_assemble(sg, n, (int)q, (int)k, d_cts.as<uint8_t>(), d_h.as<uint8_t>(), d_known.as<uint8_t>(),
                           d_x.as<uint8_t>(), d_y.as<uint8_t>(), d_pts.as<uint8_t>(), d_sc.as<uint32_t>(), st));
    KCK(cck_msm_straus(sg, 2 * n, t, d_pts.as<uint8_t>(), t * sb, 0, sb, d_sc.as<uint32_t>(), 1,
                       c->agg_scratch.as<uint32_t>(), d_out.as<uint8_t>(), st));
    std::vector<uint8_t> o(2 * n * sb);
    HIPCK(hipMemcpyAsync(o.data(), d_out.p, 2 * n * sb, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(out_h, d_h.p, n * sb, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    for (size_t r = 0; r < n; r++) {
        memcpy(out_c1 + r * sb, &o[(2 * r) * sb], sb);
        memcpy(out_c2 + r * sb, &o[(2 * r + 1) * sb], sb);
    }
    return CC_OK;
}

size_t cc_sigreq_proof_bytes(const cc_ctx* c, size_t k) {
    c = primary(c);
    return c ? cck_sigreq_proof_bytes(sig_group(c->mode), (int)k) : 0;
}

cc_status cc_sigreq_verify_batch(cc_ctx* c, size_t n, size_t q, size_t k, const uint8_t* g, const uint8_t* hvec,
                                 const uint8_t* commitment, const uint8_t* known, const uint8_t* ciphertexts,
                                 const uint8_t* elgamal_pk, const uint8_t* proofs, const uint8_t* chal,
                                 uint8_t* verdicts) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !g || (k && !hvec) ||
        (n && (!commitment || !elgamal_pk || !proofs || !chal || !verdicts || (k && !ciphertexts) || (q > k && !known))))
        return CC_ERR_DECODE;
    if (q > kMaxQ) return CC_ERR_DECODE;
    if (k > q) return CC_ERR_LEN;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    const size_t sb = (size_t)sig_bytes(c->mode);
    const int sg = sig_group(c->mode);
    const size_t pb = cck_sigreq_proof_bytes(sg, (int)k);
    hipStream_t st = c->stream;
    DevBuf d_h, d_g, d_hv, d_comm, d_cts, d_pk, d_pr, d_ch, d_scr, d_ok, d_v;
    cc_status s = compute_h_batch(c, n, q, k, commitment, known, d_h);
    if (s) return s;
    if (d_g.ensure(sb) || d_hv.ensure(k * sb + 16) || d_comm.ensure(n * sb) || d_cts.ensure(n * k * 2 * sb + 16) ||
        d_pk.ensure(n * sb) || d_pr.ensure(n * pb) || d_ch.ensure(n * 48) ||
        d_scr.ensure(cck_sigreq_scratch_words(sg, n, (int)k) * 4) || d_ok.ensure(n * (2 + 2 * k)) || d_v.ensure(n))
        return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(d_g.p, g, sb, hipMemcpyHostToDevice, st));
    if (k) HIPCK(hipMemcpyAsync(d_hv.p, hvec, k * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_comm.p, commitment, n * sb, hipMemcpyHostToDevice, st));
    if (k) HIPCK(hipMemcpyAsync(d_cts.p, ciphertexts, n * k * 2 * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_pk.p, elgamal_pk, n * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_pr.p, proofs, n * pb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_ch.p, chal, n * 48, hipMemcpyHostToDevice, st));
    KCK(cck_sigreq_verify(sg, n, (int)k, d_g.as<uint8_t>(), d_hv.as<uint8_t>(), d_comm.as<uint8_t>(),
                          d_cts.as<uint8_t>(), d_pk.as<uint8_t>(), d_pr.as<uint8_t>(), d_ch.as<uint8_t>(),
                          d_h.as<uint8_t>(), d_scr.as<uint32_t>(), d_ok.as<uint8_t>(), d_v.as<uint8_t>(), st));
    HIPCK(hipMemcpyAsync(verdicts, d_v.p, n, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    return CC_OK;
}

// ---------------------------------------------------------------- keygen: Pedersen VSS (§8(f) row 4)
cc_status cc_vss_verify_batch(cc_ctx* c, size_t n, size_t t, const uint8_t* g, const uint8_t* h,
                              const uint8_t* commitments, size_t n_sets, const uint32_t* set_of, const uint64_t* ids,
                              const uint8_t* shares, uint8_t* verdicts) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !g || !h || (n && (!commitments || !set_of || !ids || !shares || !verdicts)) || t == 0 || t > 4096 ||
        n > kMaxBatch || n_sets > kMaxBatch)
        return CC_ERR_DECODE;
    for (size_t i = 0; i < n; i++)
        if (set_of[i] >= n_sets) return CC_ERR_DECODE;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    DevBuf d_g, d_h, d_c, d_set, d_ids, d_sh, d_scr, d_ok;
    if (d_g.ensure(97) || d_h.ensure(97) || d_c.ensure(n_sets * t * 97) || d_set.ensure(n * 4) || d_ids.ensure(n * 8) ||
        d_sh.ensure(n * 96) || d_scr.ensure(n * (t + 2) * 33 * 4) || d_ok.ensure(n))
        return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(d_g.p, g, 97, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_h.p, h, 97, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_c.p, commitments, n_sets * t * 97, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_set.p, set_of, n * 4, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_ids.p, ids, n * 8, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(d_sh.p, shares, n * 96, hipMemcpyHostToDevice, st));
    KCK(cck_vss_verify(n, (int)t, d_g.as<uint8_t>(), d_h.as<uint8_t>(), d_c.as<uint8_t>(), d_set.as<uint32_t>(),
                       d_ids.as<uint64_t>(), d_sh.as<uint8_t>(), d_scr.as<uint32_t>(), d_ok.as<uint8_t>(), st));
    HIPCK(hipMemcpyAsync(verdicts, d_ok.p, n, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    return CC_OK;
}

// ---------------------------------------------------------------- issuer table (config 4)
cc_status cc_set_issuers(cc_ctx* c, size_t n_iss, size_t q, const uint64_t* ids, const uint8_t* X, const uint8_t* Y) {
    if (!c || !n_iss || !ids || !X || (q && !Y) || n_iss > (1u << 20) || q > 4096) return CC_ERR_DECODE;
    if (!c->peers.empty()) {
        for (cc_ctx* p : c->peers) {
            cc_status s = cc_set_issuers(p, n_iss, q, ids, X, Y);
            if (s) return s;
        }
        return CC_OK;
    }
    // no issuer table until every step below has succeeded (a failed call leaves CC_ERR_STATE behind,
    // never stale metadata over a rebuilt buffer)
    c->iss_n = 0;
    c->iss_q = 0;
    c->iss_ids_host.clear();
    HIPCK(hipSetDevice(c->device));
    drain_slots(c);  // concurrent verify batches (cc_set_concurrency) use buffers rebuilt here
    const int og = oth_group(c->mode);
    const size_t ob = (size_t)oth_bytes(c->mode), aw = aff_words(og);
    // rows sorted by id; ids must be unique (they are the signers' Shamir x-coordinates)
    std::vector<size_t> ord(n_iss);
    for (size_t k = 0; k < n_iss; k++) ord[k] = k;
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return ids[a] < ids[b]; });
    for (size_t k = 1; k < n_iss; k++)
        if (ids[ord[k]] == ids[ord[k - 1]]) return CC_ERR_DECODE;
    const size_t nb = n_iss * (q + 1);
    std::vector<uint8_t> enc(nb * ob);
    std::vector<uint64_t> sid(n_iss);
    for (size_t r = 0; r < n_iss; r++) {
        const size_t k = ord[r];
        sid[r] = ids[k];
        memcpy(&enc[(r * (q + 1)) * ob], X + k * ob, ob);
        for (size_t j = 0; j < q; j++) memcpy(&enc[(r * (q + 1) + 1 + j) * ob], Y + (k * q + j) * ob, ob);
    }
    // the widest window whose tables fit the budget (16 GiB of the 288 GB HBM, at most half of what is
    // free; cc_set_table_bits forces a width): t x nwin additions per aggregated key, nwin = ceil(256 / w).
    // The old table is released first so its memory counts as free (identical calls pick the same width).
    c->iss_table.release();
    const double budget = std::min(16.0 * (double)(1ull << 30), 0.5 * (double)free_hbm());
    int wb = 8;
    if (c->force_iss_bits >= 8 && c->force_iss_bits <= 16) {
        wb = c->force_iss_bits;
    } else {
        for (int cand : {16, 13, 12, 10})
            if ((double)(nb * tab_words(og, cand) * 4) <= budget) {
                wb = cand;
                break;
            }
    }
    if (c->iss_ids.ensure(n_iss * 8) || c->iss_aff.ensure(nb * aw * 4) || c->iss_inf.ensure(nb * 4))
        return CC_ERR_HIP;
    const double fr = (double)free_hbm();
    if (fr > 0 && (double)(nb * tab_words(og, wb) * 4) > 0.9 * fr) {  // see rebuild_tables
        if (c->force_iss_bits) return CC_ERR_HIP;
        wb = 8;
    }
    if (c->iss_table.ensure(nb * tab_words(og, wb) * 4)) {
        (void)hipGetLastError();  // clear the failed allocation's error
        if (c->force_iss_bits) return CC_ERR_HIP;
        wb = 8;                   // the wide table did not fit the free HBM
        if (c->iss_table.ensure(nb * tab_words(og, wb) * 4)) return CC_ERR_HIP;
    }
    cc_status s = decode_points_host(c, og, nb, enc.data(), c->iss_aff.as<uint32_t>(), c->iss_inf.as<uint32_t>());
    if (s) return s;
    HIPCK(hipMemcpy(c->iss_ids.p, sid.data(), n_iss * 8, hipMemcpyHostToDevice));
    DevBuf pw;
    if (pw.ensure(nb * tab_nwin(wb) * (og == 1 ? 36 : 72) * 4)) return CC_ERR_HIP;
    KCK(cck_build_table(og, (int)nb, wb, c->iss_aff.as<uint32_t>(), c->iss_inf.as<uint32_t>(), pw.as<uint32_t>(),
                        c->iss_table.as<uint32_t>(), 1, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    pw.release();
    c->iss_n = n_iss;
    c->iss_q = q;
    c->iss_wbits = wb;
    c->iss_ids_host = sid;
    return CC_OK;
}

static cc_status launch_vk_aggregate_ids(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                         uint8_t* d_oX, uint8_t* d_oY, hipStream_t st) {
    if (c->lag.ensure(n * t * 32 + 32)) return CC_ERR_HIP;
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
    KCK(cck_lagrange(n, len, t, d_ids, c->lag.as<uint32_t>(), st));
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    if (!c->dev_err.p) {  // sticky until cc_device_error reads it
        if (c->dev_err.ensure(4)) return CC_ERR_HIP;
        HIPCK(hipMemsetAsync(c->dev_err.p, 0, 4, st));
    }
    KCK(cck_vk_agg_fixed(oth_group(c->mode), n, len, t, (int)c->iss_q, d_ids, c->lag.as<uint32_t>(),
                         c->iss_ids.as<uint64_t>(), (int)c->iss_n, c->iss_table.as<uint32_t>(), c->iss_wbits,
                         c->iss_inf.as<uint32_t>(), d_oX, d_oY, c->dev_err.as<uint32_t>(), st));
    if (c->timing) {
        (void)hipEventRecord(c->ev[2], st);
        (void)hipEventRecord(c->ev[3], st);
    }
    return CC_OK;
}

cc_status cc_verkey_aggregate_ids_device(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                         uint8_t* d_outX, uint8_t* d_outY, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!d_ids || !d_outX || (c->iss_q && !d_outY)))) return CC_ERR_DECODE;
    if (!c->iss_n) return CC_ERR_STATE;
    if (len > kMaxIds) return CC_ERR_DECODE;
    if (len < t || len == 0) return CC_ERR_THRESHOLD;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    StreamOrder order(c, st);
    cc_status s = launch_vk_aggregate_ids(c, n, len, t, d_ids, d_outX, d_outY, st);
    if (s) return s;
    if (c->timing) collect_timing(c);
    return CC_OK;
}

// Signature::aggregate + Verkey::aggregate of the same credentials (same id lists): the Lagrange
// coefficients depend only on the ids (signature.rs:454-463 and 496-509 compute the same l_i), so one
// k_lagrange launch serves both MSMs.  Timing: (Lagrange, signature MSM, verkey MSM).
cc_status cc_aggregate_credential_batch_device(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* d_ids,
                                               const uint8_t* d_s1, const uint8_t* d_s2, uint8_t* d_out_s1,
                                               uint8_t* d_out_s2, uint8_t* d_outX, uint8_t* d_outY, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!d_ids || !d_s1 || !d_s2 || !d_out_s1 || !d_out_s2 || !d_outX || (c->iss_q && !d_outY))))
        return CC_ERR_DECODE;
    if (!c->iss_n) return CC_ERR_STATE;
    if (len > kMaxIds) return CC_ERR_DECODE;
    if (len < t || len == 0) return CC_ERR_THRESHOLD;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    StreamOrder order(c, st);
    const size_t sb = (size_t)sig_bytes(c->mode);
    const int sg = sig_group(c->mode);
    if (c->lag.ensure(n * t * 32 + 32)) return CC_ERR_HIP;
    cc_status s = agg_scratch(c, sg, n, t);
    if (s) return s;
    if (!c->dev_err.p) {
        if (c->dev_err.ensure(4)) return CC_ERR_HIP;
        HIPCK(hipMemsetAsync(c->dev_err.p, 0, 4, st));
    }
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
    // sigma_1 = sigs[0].sigma_1 (signature.rs:452): depends on neither MSM, so it goes first (behind the
    // Straus launch's one round of wave slots it waited milliseconds for a free slot)
    KCK(cck_copy_rows(n, sb, d_s1, len * sb, d_out_s1, st));
    KCK(cck_lagrange(n, len, t, d_ids, c->lag.as<uint32_t>(), st));
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    // the two MSMs share only the Lagrange coefficients: Signature::aggregate first on the caller's
    // stream (its launch is sized to one round of wave slots, cck_msm_straus), Verkey::aggregate on the
    // side stream behind it, filling the slots the Straus launch leaves and its tail
    hipStream_t side = c->side ? c->side : st;
    if (side != st) HIPCK(hipEventRecord(c->ev_fork, st));  // the coefficients are ready
    KCK(cck_msm_straus(sg, n, t, d_s2, len * sb, 0, sb, c->lag.as<uint32_t>(), 1, c->agg_scratch.as<uint32_t>(),
                       d_out_s2, st));
    if (side != st) HIPCK(hipStreamWaitEvent(side, c->ev_fork, 0));
    KCK(cck_vk_agg_fixed(oth_group(c->mode), n, len, t, (int)c->iss_q, d_ids, c->lag.as<uint32_t>(),
                         c->iss_ids.as<uint64_t>(), (int)c->iss_n, c->iss_table.as<uint32_t>(), c->iss_wbits,
                         c->iss_inf.as<uint32_t>(), d_outX, d_outY, c->dev_err.as<uint32_t>(), side));
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    if (side != st) {
        HIPCK(hipEventRecord(c->ev_join, side));
        HIPCK(hipStreamWaitEvent(st, c->ev_join, 0));
    }
    if (c->timing) {
        (void)hipEventRecord(c->ev[3], st);  // phases: Lagrange, Signature::aggregate (sharing the GPU), the
        collect_timing(c);                   // rest of Verkey::aggregate after it
    }
    return CC_OK;
}

cc_status cc_verkey_aggregate_ids(cc_ctx* c, size_t n, size_t len, size_t t, const uint64_t* ids, uint8_t* outX,
                                  uint8_t* outY) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!ids || !outX || (c->iss_q && !outY)))) return CC_ERR_DECODE;
    if (!c->iss_n) return CC_ERR_STATE;
    if (len > kMaxIds) return CC_ERR_DECODE;
    if (len < t || len == 0) return CC_ERR_THRESHOLD;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    for (size_t i = 0; i < n; i++)
        for (size_t k = 0; k < t; k++)
            if (!std::binary_search(c->iss_ids_host.begin(), c->iss_ids_host.end(), ids[i * len + k]))
                return CC_ERR_DECODE;  // id without an issuer verkey (the reference indexes a missing key)
    HIPCK(hipSetDevice(c->device));
    const size_t ob = (size_t)oth_bytes(c->mode), q = c->iss_q;
    hipStream_t st = c->stream;
    DevBuf& d_ids = c->in_aux[0];
    DevBuf& d_oX = c->in_aux[2];
    DevBuf& d_oY = c->in_aux[4];
    if (d_ids.ensure(n * len * 8) || d_oX.ensure(n * ob) || d_oY.ensure(n * q * ob + 16)) return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(d_ids.p, ids, n * len * 8, hipMemcpyHostToDevice, st));
    cc_status s = launch_vk_aggregate_ids(c, n, len, t, d_ids.as<uint64_t>(), d_oX.as<uint8_t>(), d_oY.as<uint8_t>(), st);
    if (s) return s;
    HIPCK(hipMemcpyAsync(outX, d_oX.p, n * ob, hipMemcpyDeviceToHost, st));
    if (q) HIPCK(hipMemcpyAsync(outY, d_oY.p, n * q * ob, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    return CC_OK;
}

cc_status cc_device_error(cc_ctx* c, void* stream, uint32_t* out) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || !out) return CC_ERR_DECODE;
    *out = 0;
    if (!c->dev_err.p) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    StreamOrder order(c, st);
    uint32_t v = 0;
    HIPCK(hipMemcpyAsync(&v, c->dev_err.p, 4, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemsetAsync(c->dev_err.p, 0, 4, st));
    HIPCK(hipStreamSynchronize(st));
    *out = v;
    return CC_OK;
}

// revealed indices (shared by the batch): < q and unique (ps_sig's HashMap keys); reference would panic
static cc_status check_revealed(size_t q, size_t r, const uint64_t* rev_idx, std::vector<uint32_t>& idx) {
    idx.assign(r ? r : 1, 0);
    for (size_t z = 0; z < r; z++) {
        if (rev_idx[z] >= q) return CC_ERR_LEN;  // reference would index out of bounds (panic)
        for (size_t y = 0; y < z; y++)
            if (rev_idx[y] == rev_idx[z]) return CC_ERR_DECODE;  // HashMap keys are unique
        idx[z] = (uint32_t)rev_idx[z];
    }
    return CC_OK;
}

static cc_status launch_pok(cc_ctx* c, const VerifyWork& w, size_t n, size_t q, size_t r, const uint8_t* d_s1,
                            const uint8_t* d_s2, const uint8_t* d_J, const uint8_t* d_T, const uint8_t* d_resp,
                            const uint8_t* d_chal, const uint32_t* d_idx, const uint8_t* d_rev_msgs, uint8_t* d_verdicts,
                            uint8_t* d_gt, hipStream_t st) {
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
    // small batches: one block of two waves per proof (the Schnorr terms over a wave's lanes)
    KCK((n <= kPrepWideMax ? cck_prep_pok_wide : cck_prep_pok)(
        c->mode, n, (int)q, (int)r, d_s1, d_s2, d_J, d_T, d_resp, d_chal, d_rev_msgs, d_idx, c->vk_aff.as<uint32_t>(),
        c->X_inf, c->table.as<uint32_t>(), c->wbits, c->table_inf.as<uint32_t>(), w.prep->as<uint32_t>(),
        w.flags->as<uint32_t>(), w.scratch->as<uint32_t>(), st));  // J*chal window table: the fexp scratch, free until fexp
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    cc_status ms = launch_miller(c, w, n, st);
    if (ms) return ms;
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    KCK(cck_fexp(n, w.fbuf->as<uint32_t>(), w.scratch->as<uint32_t>(), w.flags->as<uint32_t>(), d_verdicts, d_gt,
                 kFexpWideMax, st));
    if (c->timing) (void)hipEventRecord(c->ev[3], st);
    return CC_OK;
}

cc_status cc_pok_verify_batch_device(cc_ctx* c, size_t n, size_t q, size_t r, size_t nresp, const uint8_t* d_s1,
                                     const uint8_t* d_s2, const uint8_t* d_J, const uint8_t* d_T,
                                     const uint8_t* d_resp, const uint8_t* d_chal, const uint64_t* rev_idx,
                                     const uint8_t* d_rev_msgs, uint8_t* d_verdicts, uint8_t* d_gt, void* stream) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!d_s1 || !d_s2 || !d_J || !d_T || !d_chal || !d_verdicts || (nresp && !d_resp) ||
                     (r && (!rev_idx || !d_rev_msgs)))))
        return CC_ERR_DECODE;
    if (!c->have_params || !c->have_vk) return CC_ERR_STATE;
    if (q != c->q) return CC_ERR_LEN;
    std::vector<uint32_t> idx;
    cc_status s = check_revealed(q, r, rev_idx, idx);
    if (s) return s;
    if (nresp != q - r + 1) return CC_ERR_BASES_EXPS;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (c->concurrency > 1) {  // the next concurrency slot (cc_set_concurrency): its own tables of d J
        int k = 0;
        VerifyWork w;
        s = slot_begin(c, st, cc::slots::verify_sizes(n, 0, (n * 15 * 84 + 72 * 12) * 4, idx.size() * 4 + 4), k, w);
        if (s) return s;
        SlotFence fence(c->pool, c->dev, k, st);
        if (r) KCK(c->stage[(size_t)k].upload(w.idx->p, idx.data(), idx.size() * 4, st));  // pinned ring
        s = launch_pok(c, w, n, q, r, d_s1, d_s2, d_J, d_T, d_resp, d_chal, w.idx->as<uint32_t>(), d_rev_msgs,
                       d_verdicts, d_gt, st);
        if (s) return s;
        return fence.close() ? CC_ERR_HIP : CC_OK;
    }
    s = ensure_work(c, n);
    if (s) return s;
    StreamOrder order(c, st);
    if (c->pok_idx.ensure(idx.size() * 4)) return CC_ERR_HIP;
    HIPCK(hipMemcpyAsync(c->pok_idx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, st));
    s = launch_pok(c, ctx_work(c), n, q, r, d_s1, d_s2, d_J, d_T, d_resp, d_chal, c->pok_idx.as<uint32_t>(), d_rev_msgs,
                   d_verdicts, d_gt, st);
    if (s) return s;
    if (c->timing) collect_timing(c);
    return CC_OK;
}

cc_status cc_pok_verify_batch(cc_ctx* c, size_t n, size_t q, size_t r, size_t nresp, const uint8_t* s1,
                              const uint8_t* s2, const uint8_t* J, const uint8_t* T, const uint8_t* resp,
                              const uint8_t* chal, const uint64_t* rev_idx, const uint8_t* rev_msgs,
                              uint8_t* verdicts, uint8_t* gt) {
    c = primary(c);  // a device set forwards to its first device
    if (!c || (n && (!s1 || !s2 || !J || !T || !chal || !verdicts || (nresp && !resp) || (r && (!rev_idx || !rev_msgs)))))
        return CC_ERR_DECODE;
    if (!c->have_params || !c->have_vk) return CC_ERR_STATE;
    if (q != c->q) return CC_ERR_LEN;
    std::vector<uint32_t> idx;
    cc_status s = check_revealed(q, r, rev_idx, idx);
    if (s) return s;
    if (nresp != q - r + 1) return CC_ERR_BASES_EXPS;
    if (n > kMaxBatch) return CC_ERR_DECODE;
    if (!n) return CC_OK;
    HIPCK(hipSetDevice(c->device));
    drain_slots(c);  // concurrent device batches still using slot 0's workspaces (cc_set_concurrency)
    size_t sb = (size_t)sig_bytes(c->mode), ob = (size_t)oth_bytes(c->mode);
    hipStream_t st = c->stream;
    DevBuf& dJ = c->in_aux[0];
    DevBuf& dT = c->in_aux[1];
    DevBuf& dR = c->in_aux[2];
    DevBuf& dC = c->in_aux[3];
    DevBuf& dM = c->in_aux[4];
    DevBuf& dI = c->in_aux[5];
    if (c->in_s1.ensure(n * sb) || c->in_s2.ensure(n * sb) || dJ.ensure(n * ob) || dT.ensure(n * ob) ||
        dR.ensure(n * nresp * 48 + 16) || dC.ensure(n * 48) || dM.ensure(n * r * 48 + 16) || dI.ensure(r * 4 + 4) ||
        c->verdicts.ensure(n) || (gt && c->gt.ensure(n * 576)))
        return CC_ERR_HIP;
    s = ensure_work(c, n);
    if (s) return s;
    HIPCK(hipMemcpyAsync(c->in_s1.p, s1, n * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->in_s2.p, s2, n * sb, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(dJ.p, J, n * ob, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(dT.p, T, n * ob, hipMemcpyHostToDevice, st));
    if (nresp) HIPCK(hipMemcpyAsync(dR.p, resp, n * nresp * 48, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(dC.p, chal, n * 48, hipMemcpyHostToDevice, st));
    if (r) {
        HIPCK(hipMemcpyAsync(dM.p, rev_msgs, n * r * 48, hipMemcpyHostToDevice, st));
        HIPCK(hipMemcpyAsync(dI.p, idx.data(), r * 4, hipMemcpyHostToDevice, st));
    }
    s = launch_pok(c, ctx_work(c), n, q, r, c->in_s1.as<uint8_t>(), c->in_s2.as<uint8_t>(), dJ.as<uint8_t>(), dT.as<uint8_t>(),
                   dR.as<uint8_t>(), dC.as<uint8_t>(), dI.as<uint32_t>(), dM.as<uint8_t>(), c->verdicts.as<uint8_t>(),
                   gt ? c->gt.as<uint8_t>() : nullptr, st);
    if (s) return s;
    HIPCK(hipMemcpyAsync(verdicts, c->verdicts.p, n, hipMemcpyDeviceToHost, st));
    if (gt) HIPCK(hipMemcpyAsync(gt, c->gt.p, n * 576, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    collect_timing(c);
    return CC_OK;
}


// ---------------------------------------------------------------- device sets + RCCL
cc_status cc_ctx_create_multi(uint64_t device_mask, cc_group_mode mode, cc_ctx** out) {
    if (!out || !device_mask || (mode != CC_SIG_G2 && mode != CC_SIG_G1)) return CC_ERR_DECODE;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return CC_ERR_HIP;
    std::vector<int> devs;
    for (int d = 0; d < 64; d++)
        if ((device_mask >> d) & 1ull) {
            if (d >= ndev) return CC_ERR_HIP;
            devs.push_back(d);
        }
    cc_ctx* c = new cc_ctx();
    c->device = devs[0];
    c->mode = (int)mode;
    for (int d : devs) {
        cc_ctx* p = nullptr;
        cc_status s = cc_ctx_create(d, mode, &p);
        if (s) {
            for (cc_ctx* q : c->peers) cc_ctx_destroy(q);
            delete c;
            return s;
        }
        c->peers.push_back(p);
    }
    c->comms.resize(devs.size());
    if (ncclCommInitAll(c->comms.data(), (int)devs.size(), devs.data()) != ncclSuccess) {
        c->comms.clear();
        for (cc_ctx* q : c->peers) cc_ctx_destroy(q);
        delete c;
        return CC_ERR_RCCL;
    }
    *out = c;
    return CC_OK;
}

cc_status cc_ctx_num_devices(const cc_ctx* c, int* n) {
    if (!c || !n) return CC_ERR_DECODE;
    *n = c->peers.empty() ? 1 : (int)c->peers.size();
    return CC_OK;
}

}  // extern "C"

// run f(k, lo, hi) for every peer k on its own host thread over the contiguous shard [lo, hi)
template <class F>
static cc_status for_shards(cc_ctx* c, size_t n, F f) {
    const size_t k = c->peers.size();
    std::vector<cc_status> st(k, CC_OK);
    std::vector<std::thread> th;
    for (size_t d = 0; d < k; d++)
        th.emplace_back([&, d] { st[d] = f(d, n * d / k, n * (d + 1) / k); });
    for (auto& t : th) t.join();
    for (cc_status s : st)
        if (s) return s;
    return CC_OK;
}

extern "C" {

// Shard by credential over the device set.  Per-credential mode: every device verifies its slice, no
// collective.  RLC mode (shared verkey): every device reduces its slice to one RLC_PART_WORDS-word partial, ONE
// ncclAllGather over xGMI exchanges them, every device multiplies the gathered partials and runs the
// single final exponentiation; on reject every device falls back to per-credential verification.
static cc_status multi_verify(cc_ctx* c, size_t n, size_t q, const uint8_t* s1, const uint8_t* s2,
                              const uint8_t* msgs, const uint8_t* vkX, const uint8_t* vkY, uint8_t* verdicts,
                              uint8_t* gt, int rlc) {
    const size_t sb = (size_t)sig_bytes(c->mode), ob = (size_t)oth_bytes(c->mode);
    const size_t k = c->peers.size();
    if (rlc && !vkX && !gt) {
        uint8_t seed[32];
        if (fresh_seed(seed)) return CC_ERR_HIP;
        // stage each slice and compute its partial
        cc_status s = for_shards(c, n, [&](size_t d, size_t lo, size_t hi) -> cc_status {
            cc_ctx* p = c->peers[d];
            const size_t m = hi - lo;
            HIPCK(hipSetDevice(p->device));
            if (p->in_s1.ensure(m * sb + 16) || p->in_s2.ensure(m * sb + 16) || p->in_msgs.ensure(m * q * 48 + 16) ||
                p->rlc_part.ensure(RLC_PART_WORDS * 4) || p->rlc_gath.ensure(k * RLC_PART_WORDS * 4) || p->rlc_accept.ensure(1))
                return CC_ERR_HIP;
            if (m) {
                HIPCK(hipMemcpyAsync(p->in_s1.p, s1 + lo * sb, m * sb, hipMemcpyHostToDevice, p->stream));
                HIPCK(hipMemcpyAsync(p->in_s2.p, s2 + lo * sb, m * sb, hipMemcpyHostToDevice, p->stream));
                if (q) HIPCK(hipMemcpyAsync(p->in_msgs.p, msgs + lo * q * 48, m * q * 48, hipMemcpyHostToDevice, p->stream));
            }
            return cc_rlc_partial_device(p, m, q, lo, seed, p->in_s1.as<uint8_t>(), p->in_s2.as<uint8_t>(),
                                         p->in_msgs.as<uint8_t>(), p->rlc_part.as<uint32_t>(), p->stream);
        });
        if (s) return s;
        // the one exchange step: all-gather of the 3,716-byte (RLC_PART_WORDS = 929 words) partials
        if (ncclGroupStart() != ncclSuccess) return CC_ERR_RCCL;
        for (size_t d = 0; d < k; d++) {
            cc_ctx* p = c->peers[d];
            if (ncclAllGather(p->rlc_part.p, p->rlc_gath.p, RLC_PART_WORDS, ncclUint32, c->comms[d], p->stream) != ncclSuccess) {
                ncclGroupEnd();
                return CC_ERR_RCCL;
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return CC_ERR_RCCL;
        std::vector<uint8_t> acc(k, 0);
        s = for_shards(c, n, [&](size_t d, size_t, size_t) -> cc_status {
            cc_ctx* p = c->peers[d];
            HIPCK(hipSetDevice(p->device));
            cc_status r = cc_rlc_finish_device(p, k, p->rlc_gath.as<uint32_t>(), p->rlc_accept.as<uint8_t>(), nullptr,
                                               p->stream);
            if (r) return r;
            HIPCK(hipMemcpyAsync(&acc[d], p->rlc_accept.p, 1, hipMemcpyDeviceToHost, p->stream));
            HIPCK(hipStreamSynchronize(p->stream));
            return CC_OK;
        });
        if (s) return s;
        for (size_t d = 1; d < k; d++)
            if (acc[d] != acc[0]) return CC_ERR_RCCL;  // every device multiplies the same gathered partials
        if (acc[0]) {
            memset(verdicts, 1, n);
            return CC_OK;
        }
    }
    // per-credential verification of every slice (also the RLC fallback)
    return for_shards(c, n, [&](size_t d, size_t lo, size_t hi) -> cc_status {
        if (hi == lo) return CC_OK;
        return cc_verify_batch(c->peers[d], hi - lo, q, s1 + lo * sb, s2 + lo * sb, msgs + lo * q * 48,
                               vkX ? vkX + lo * ob : nullptr, vkX ? vkY + lo * q * ob : nullptr, verdicts + lo,
                               gt ? gt + lo * 576 : nullptr, 0);
    });
}

}  // extern "C"
