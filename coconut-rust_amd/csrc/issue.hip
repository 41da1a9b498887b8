// Issuer-side batch kernels for gfx950: the step before verify in issuance.
//
//   BlindSignature::new (reference src/signature.rs:382-433), per request:
//       h = compute_h(commitment, known)  (hash.hip, before this)
//       c~1 = sum_{i<k} y_i a_i,   c~2 = sum_{i<k} y_i b_i + h (x + sum_j y_{k+j} m_j)
//     k_blind_assemble lays every request's bases and scalars out for the windowed Straus MSM
//     (aggregate.hip k_msm_straus): task 2r = c~1 (k bases), task 2r+1 = c~2 (k+1 bases).
//   SignatureRequestProof::verify (src/signature.rs:324-377), one lane per Schnorr check:
//       check 0          : [g]                 vs elgamal_pk       (proof_elgamal_sk)
//       check 1          : [h_1..h_k, g]       vs commitment       (proof_commitment)
//       check 2+2i, 3+2i : [g] vs c1_i,  [pk, h] vs c2_i            (proof_ciphertexts[i])
//     each: MSM(bases || commitment, responses || challenge) - T == O (impl_PoK_VC! ProofX::verify
//     [EXT]) by interleaved double-and-add over decoded points; k_sigreq_combine ANDs a request's
//     checks with the response-equality rule proof_2.responses[1] == proof_commitment.responses[i].
#include "codec.h"
#include "fr.h"

using namespace cc;

namespace {

template <class F>
DEV bool dec_pt(Aff<F>& a, const uint8_t* p);
template <>
DEV bool dec_pt<Fp>(Aff<Fp>& a, const uint8_t* p) { return g1_decode(a, p); }
template <>
DEV bool dec_pt<Fp2>(Aff<Fp2>& a, const uint8_t* p) { return g2_decode(a, p); }

template <class F>
constexpr int eb() { return sizeof(F) == sizeof(Fp) ? 97 : 192; }

// byte offsets inside one request's proof record (layout of cc_sigreq_verify_batch)
struct ProofLayout {
    size_t sb, k;
    __host__ __device__ size_t t_sk() const { return 0; }
    __host__ __device__ size_t r_sk() const { return sb; }
    __host__ __device__ size_t t_comm() const { return sb + 48; }
    __host__ __device__ size_t r_comm(size_t i) const { return 2 * sb + 48 + 48 * i; }
    __host__ __device__ size_t ct(size_t i) const { return 2 * sb + 48 * (k + 2) + i * (2 * sb + 144); }
    __host__ __device__ size_t bytes() const { return ct(k); }
};

}  // namespace

// SignatureRequest::compute_h's input rows (signature.rs:197-206 hashes commitment.to_bytes() ||
// known_messages[i].to_bytes()): the caller's commitment bytes are decoded and re-encoded (an
// off-curve or non-canonical encoding becomes what amcl_wrapper's to_bytes of the decoded point
// gives) and every known message is reduced mod r into its canonical 48-byte encoding, in place.
// One row (len = SignatureGroup bytes + 48 kn) per lane.
template <class F>
__global__ __launch_bounds__(64) void k_h_input_canon(size_t n, size_t len, int kn, uint8_t* __restrict__ data) {
    const size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    uint8_t* row = data + r * len;
    Aff<F> a;
    const bool fin = dec_pt<F>(a, row);
    if (sizeof(F) == sizeof(Fp)) g1_encode(row, *reinterpret_cast<Aff<Fp>*>(&a), fin);
    else g2_encode(row, *reinterpret_cast<Aff<Fp2>*>(&a), fin);
#pragma unroll 1
    for (int j = 0; j < kn; j++) {
        uint8_t* p = row + eb<F>() + 48 * (size_t)j;
        Fp raw;
        be48_bytes(raw, p);
        uint32_t hi = raw.v[8] | raw.v[9] | raw.v[10] | raw.v[11], br = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) (void)__builtin_subc(raw.v[w], r_limb(w), br, &br);
        if (hi != 0 || br == 0) fr_reduce_slow(raw.v);
#pragma unroll 1
        for (int b = 0; b < 48; b++) {
            const int w = (47 - b) >> 2;  // big-endian: byte b holds bits 8 (47 - b)
            p[b] = w < 8 ? (uint8_t)(raw.v[w] >> (8 * ((47 - b) & 3))) : 0;
        }
    }
}

// scalars for the Straus tasks: canonical 8-limb Fr per (task, base); bases as encodings
template <class F>
__global__ __launch_bounds__(64) void k_blind_assemble(size_t n, int q, int k, const uint8_t* __restrict__ cts,
                                                       const uint8_t* __restrict__ hpts,
                                                       const uint8_t* __restrict__ known,
                                                       const uint8_t* __restrict__ x48,
                                                       const uint8_t* __restrict__ y48,
                                                       uint8_t* __restrict__ pts, uint32_t* __restrict__ sc) {
    const size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    constexpr int SB = eb<F>();
    const int t = k + 1;  // bases per task (c~1 uses the first k, its last scalar is 0)
    uint8_t* p1 = pts + (2 * r) * (size_t)t * SB;
    uint8_t* p2 = pts + (2 * r + 1) * (size_t)t * SB;
    uint32_t* s1 = sc + (2 * r) * (size_t)t * 8;
    uint32_t* s2 = sc + (2 * r + 1) * (size_t)t * 8;
    const uint8_t* c = cts + r * (size_t)k * 2 * SB;
    for (int i = 0; i < k; i++) {
        for (int b = 0; b < SB; b++) {
            p1[i * SB + b] = c[(2 * i) * SB + b];
            p2[i * SB + b] = c[(2 * i + 1) * SB + b];
        }
        Fr y;
        fr_from_be48(y, y48 + 48 * i);
        for (int w = 0; w < 8; w++) s1[i * 8 + w] = s2[i * 8 + w] = y.v[w];
    }
    // c~1's padding base: h with scalar 0 (contributes the identity)
    for (int b = 0; b < SB; b++) {
        p1[k * SB + b] = hpts[r * SB + b];
        p2[k * SB + b] = hpts[r * SB + b];
    }
    for (int w = 0; w < 8; w++) s1[k * 8 + w] = 0;
    // e = x + sum_j y_{k+j} m_j mod r
    Fr x;
    fr_from_be48(x, x48);
    uint32_t e[8];
    for (int w = 0; w < 8; w++) e[w] = x.v[w];
    for (int j = 0; j < q - k; j++) {
        Fr y, m;
        fr_from_be48(y, y48 + 48 * (k + j));
        fr_from_be48(m, known + (r * (size_t)(q - k) + j) * 48);
        uint32_t t2[8];
        fr_mul_canon(t2, y.v, m.v);
        Fm a, b, s;
        for (int w = 0; w < 8; w++) {
            a.v[w] = e[w];
            b.v[w] = t2[w];
        }
        // s = a + b mod r (both canonical)
        uint32_t cy = 0;
        for (int w = 0; w < 8; w++) s.v[w] = __builtin_addc(a.v[w], b.v[w], cy, &cy);
        fm_reduce_once(s, s.v);
        for (int w = 0; w < 8; w++) e[w] = s.v[w];
    }
    for (int w = 0; w < 8; w++) s2[k * 8 + w] = e[w];
}

// One Schnorr check per lane: sum_j resp_j B_j + chal * C - T == O
template <class F>
__global__ __launch_bounds__(64) void k_sigreq_checks(size_t n, int k, const uint8_t* __restrict__ g,
                                                      const uint8_t* __restrict__ hvec,
                                                      const uint8_t* __restrict__ commitment,
                                                      const uint8_t* __restrict__ cts,
                                                      const uint8_t* __restrict__ pk,
                                                      const uint8_t* __restrict__ proof,
                                                      const uint8_t* __restrict__ chal,
                                                      const uint8_t* __restrict__ hpts, uint32_t* __restrict__ scratch,
                                                      uint8_t* __restrict__ ok) {
    const int nchk = 2 + 2 * k;
    const size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (gi >= n * nchk) return;
    const size_t r = gi / nchk;
    const int c = (int)(gi % nchk);
    constexpr int SB = eb<F>();
    constexpr int AW = sizeof(Aff<F>) / 4;
    const ProofLayout L{(size_t)SB, (size_t)k};
    const uint8_t* pr = proof + r * L.bytes();
    // gather (base, scalar) pairs: the bases with their responses, then the commitment with chal
    const int maxp = k + 2;
    uint32_t* sp = scratch + gi * (size_t)maxp * (AW + 8 + 1);
    int m = 0;
    const uint8_t* T;
    auto put = [&](const uint8_t* base, const uint8_t* s48) {
        uint32_t* e = sp + (size_t)m * (AW + 8 + 1);
        Aff<F> a;
        const bool fin = dec_pt<F>(a, base);
        const uint32_t* aw = reinterpret_cast<const uint32_t*>(&a);
        for (int w = 0; w < AW; w++) e[w] = aw[w];
        Fr s;
        fr_from_be48(s, s48);
        for (int w = 0; w < 8; w++) e[AW + w] = s.v[w];
        e[AW + 8] = fin ? 1u : 0u;
        m++;
    };
    if (c == 0) {
        put(g, pr + L.r_sk());
        put(pk + r * SB, chal + r * 48);
        T = pr + L.t_sk();
    } else if (c == 1) {
        for (int i = 0; i < k; i++) put(hvec + (size_t)i * SB, pr + L.r_comm(i));
        put(g, pr + L.r_comm(k));
        put(commitment + r * SB, chal + r * 48);
        T = pr + L.t_comm();
    } else {
        const int i = (c - 2) >> 1;
        const uint8_t* ct = cts + (r * (size_t)k + i) * 2 * SB;
        const uint8_t* rec = pr + L.ct(i);
        if (((c - 2) & 1) == 0) {  // proof_1: [g] vs c1
            put(g, rec + SB);
            put(ct, chal + r * 48);
            T = rec;
        } else {  // proof_2: [pk, h] vs c2
            put(pk + r * SB, rec + 2 * SB + 48);
            put(hpts + r * SB, rec + 2 * SB + 96);
            put(ct + SB, chal + r * 48);
            T = rec + SB + 48;
        }
    }
    Jac<F> acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (int b = 254; b >= 0; b--) {
        jac_dbl(acc, acc);
#pragma unroll 1
        for (int j = 0; j < m; j++) {
            const uint32_t* e = sp + (size_t)j * (AW + 8 + 1);
            if (!e[AW + 8] || !((e[AW + (b >> 5)] >> (b & 31)) & 1u)) continue;
            Aff<F> a;
            uint32_t* aw = reinterpret_cast<uint32_t*>(&a);
            for (int w = 0; w < AW; w++) aw[w] = e[w];
            jac_add_aff(acc, acc, a);
        }
    }
    Aff<F> ta;
    if (dec_pt<F>(ta, T)) {
        FT<F>::neg(ta.y, ta.y);
        jac_add_aff(acc, acc, ta);
    }
    ok[gi] = jac_is_inf(acc) ? 1 : 0;
}

// verdict per request: every check passed and the hidden-message responses agree (as Fr values)
__global__ __launch_bounds__(64) void k_sigreq_combine(size_t n, int k, size_t sb, const uint8_t* __restrict__ proof,
                                                       const uint8_t* __restrict__ ok, uint8_t* __restrict__ verdicts) {
    const size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int nchk = 2 + 2 * k;
    const ProofLayout L{sb, (size_t)k};
    const uint8_t* pr = proof + r * L.bytes();
    bool good = true;
    for (int c = 0; c < nchk; c++) good = good && ok[r * nchk + c];
    for (int i = 0; i < k; i++) {
        Fr a, b;
        fr_from_be48(a, pr + L.ct(i) + 2 * sb + 96);
        fr_from_be48(b, pr + L.r_comm(i));
        for (int w = 0; w < 8; w++) good = good && a.v[w] == b.v[w];
    }
    verdicts[r] = good ? 1 : 0;
}

// Pedersen VSS verify_share (secret_sharing [EXT]; reference keygen.rs:334-349), one share per lane:
//     sum_{i<t} id^i C_i - s g - s' h == O      (G1; C = the dealer's coefficient commitments)
// by interleaved double-and-add over the t + 2 decoded points kept in the lane's scratch.
__global__ __launch_bounds__(64) void k_vss_verify(size_t n, int t, const uint8_t* __restrict__ g,
                                                   const uint8_t* __restrict__ h, const uint8_t* __restrict__ comms,
                                                   const uint32_t* __restrict__ set_of,
                                                   const uint64_t* __restrict__ ids,
                                                   const uint8_t* __restrict__ shares,
                                                   uint32_t* __restrict__ scratch, uint8_t* __restrict__ ok) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    constexpr int AW = sizeof(Aff<Fp>) / 4, EWS = AW + 8 + 1;
    uint32_t* sp = scratch + i * (size_t)(t + 2) * EWS;
    auto put = [&](int m, const uint8_t* base, const uint32_t sc[8]) {
        uint32_t* e = sp + (size_t)m * EWS;
        Aff<Fp> a;
        const bool fin = g1_decode(a, base);
        const uint32_t* aw = reinterpret_cast<const uint32_t*>(&a);
        for (int w = 0; w < AW; w++) e[w] = aw[w];
        for (int w = 0; w < 8; w++) e[AW + w] = sc[w];
        e[AW + 8] = fin ? 1u : 0u;
    };
    // -s, -s' (mod r)
    for (int z = 0; z < 2; z++) {
        Fr v;
        fr_from_be48(v, shares + (i * 2 + z) * 48);
        uint32_t o = 0, neg[8], br = 0;
        for (int w = 0; w < 8; w++) o |= v.v[w];
        for (int w = 0; w < 8; w++) neg[w] = __builtin_subc(rl(w), v.v[w], br, &br);
        if (!o)
            for (int w = 0; w < 8; w++) neg[w] = 0;
        put(z, z ? h : g, neg);
    }
    // id^k, k < t
    const uint64_t id = ids[i];
    uint32_t pw[8] = {1u, 0, 0, 0, 0, 0, 0, 0}, idv[8] = {(uint32_t)id, (uint32_t)(id >> 32), 0, 0, 0, 0, 0, 0};
    const uint8_t* C = comms + (size_t)set_of[i] * t * 97;
    for (int k = 0; k < t; k++) {
        put(2 + k, C + (size_t)k * 97, pw);
        uint32_t nx[8];
        fr_mul_canon(nx, pw, idv);
        for (int w = 0; w < 8; w++) pw[w] = nx[w];
    }
    Jac<Fp> acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (int b = 254; b >= 0; b--) {
        jac_dbl(acc, acc);
#pragma unroll 1
        for (int m = 0; m < t + 2; m++) {
            const uint32_t* e = sp + (size_t)m * EWS;
            if (!e[AW + 8] || !((e[AW + (b >> 5)] >> (b & 31)) & 1u)) continue;
            Aff<Fp> a;
            uint32_t* aw = reinterpret_cast<uint32_t*>(&a);
            for (int w = 0; w < AW; w++) aw[w] = e[w];
            jac_add_aff(acc, acc, a);
        }
    }
    ok[i] = jac_is_inf(acc) ? 1 : 0;
}

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

extern "C" {

int cck_h_input_canon(int group, size_t n, size_t len, int kn, uint8_t* d_data, hipStream_t st) {
    if (!n) return 0;
    if (group == 1)
        hipLaunchKernelGGL(k_h_input_canon<Fp>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, len, kn, d_data);
    else
        hipLaunchKernelGGL(k_h_input_canon<Fp2>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, len, kn, d_data);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t cck_sigreq_proof_bytes(int group, int k) {
    const size_t sb = group == 1 ? 97 : 192;
    return ProofLayout{sb, (size_t)k}.bytes();
}

int cck_blind_assemble(int group, size_t n, int q, int k, const uint8_t* d_cts, const uint8_t* d_h,
                       const uint8_t* d_known, const uint8_t* d_x, const uint8_t* d_y, uint8_t* d_pts, uint32_t* d_sc,
                       hipStream_t st) {
    if (!n) return 0;
    if (group == 1)
        hipLaunchKernelGGL(k_blind_assemble<Fp>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, q, k, d_cts, d_h, d_known,
                           d_x, d_y, d_pts, d_sc);
    else
        hipLaunchKernelGGL(k_blind_assemble<Fp2>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, q, k, d_cts, d_h, d_known,
                           d_x, d_y, d_pts, d_sc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t cck_sigreq_scratch_words(int group, size_t n, int k) {
    const size_t aw = group == 1 ? 24 : 48;
    return n * (size_t)(2 + 2 * k) * (size_t)(k + 2) * (aw + 9);
}

int cck_sigreq_verify(int group, size_t n, int k, const uint8_t* d_g, const uint8_t* d_hvec, const uint8_t* d_comm,
                      const uint8_t* d_cts, const uint8_t* d_pk, const uint8_t* d_proof, const uint8_t* d_chal,
                      const uint8_t* d_hpts, uint32_t* d_scratch, uint8_t* d_ok, uint8_t* d_verdicts, hipStream_t st) {
    if (!n) return 0;
    const size_t nchk = n * (size_t)(2 + 2 * k);
    if (group == 1)
        hipLaunchKernelGGL(k_sigreq_checks<Fp>, dim3(nblocks(nchk, 64)), dim3(64), 0, st, n, k, d_g, d_hvec, d_comm,
                           d_cts, d_pk, d_proof, d_chal, d_hpts, d_scratch, d_ok);
    else
        hipLaunchKernelGGL(k_sigreq_checks<Fp2>, dim3(nblocks(nchk, 64)), dim3(64), 0, st, n, k, d_g, d_hvec, d_comm,
                           d_cts, d_pk, d_proof, d_chal, d_hpts, d_scratch, d_ok);
    hipLaunchKernelGGL(k_sigreq_combine, dim3(nblocks(n, 64)), dim3(64), 0, st, n, k, (size_t)(group == 1 ? 97 : 192),
                       d_proof, d_ok, d_verdicts);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_vss_verify(size_t n, int t, const uint8_t* d_g, const uint8_t* d_h, const uint8_t* d_comms,
                   const uint32_t* d_set_of, const uint64_t* d_ids, const uint8_t* d_shares, uint32_t* d_scratch,
                   uint8_t* d_ok, hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(k_vss_verify, dim3(nblocks(n, 64)), dim3(64), 0, st, n, t, d_g, d_h, d_comms, d_set_of, d_ids,
                       d_shares, d_scratch, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
