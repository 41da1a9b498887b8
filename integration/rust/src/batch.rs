// src/batch.rs — batch entry points on the reference crate's own types (src/signature.rs), through
// src/hip.rs.  Encodings are exactly amcl_wrapper's to_bytes() (G1 97 B, G2 192 B, Fr 48 B), so the
// glue only concatenates.  Where the reference panics the shim panics too (HipCtx::check).
// Every wrapper asserts, before its unsafe call, each length the C side derives its reads from
// (`len-guard` lines; tests/test_rust_binding.py checks they are present): the C ABI reads n * q * 48
// bytes of messages, n * len entries of a batch, ..., so a shorter Vec would be a heap over-read.
use crate::hip::*;
use crate::signature::{BlindSignature, Params, Signature, SignatureRequest, Sigkey, Verkey};
use crate::{OtherGroup, SignatureGroup};
use amcl_wrapper::field_elem::FieldElement;
use amcl_wrapper::group_elem::GroupElement;
use amcl_wrapper::group_elem_g1::G1;
use std::os::raw::c_int;

/// Smallest batch routed to the GPU.  One `Signature::verify` costs ~2.1 ms through the engine (its
/// one-wave kernels' dependency chains) against ~1.9 ms for the reference's own CPU
/// path on one host thread; two credentials already take ~3.7 ms on the CPU and still ~2.1 ms on the
/// GPU.  So a single credential keeps the reference path and only batches go to the device.
pub const GPU_MIN_BATCH: usize = 2;

impl Signature {
    /// Batch form of `Signature::verify` (signature.rs:473-478): one verkey for the whole batch.
    /// Below GPU_MIN_BATCH credentials it is the reference's own verify, unchanged.
    pub fn verify_batch(sigs: &[Signature], messages: &[Vec<FieldElement>], vk: &Verkey,
                        params: &Params, ctx: &HipCtx) -> Vec<bool> {
        let q = vk.Y_tilde.len();
        assert_eq!(messages.len(), sigs.len(), "one message vector per signature");  // len-guard
        assert!(messages.iter().all(|m| m.len() == q), "Verkey valid for {} messages", q);  // len-guard
        if sigs.len() < GPU_MIN_BATCH {
            return sigs.iter().zip(messages).map(|(s, m)| s.verify(m, vk, params)).collect();
        }
        let s1: Vec<u8> = sigs.iter().flat_map(|s| s.sigma_1.to_bytes()).collect();
        let s2: Vec<u8> = sigs.iter().flat_map(|s| s.sigma_2.to_bytes()).collect();
        let m:  Vec<u8> = messages.iter().flatten().flat_map(|f| f.to_bytes()).collect();
        ctx.set_params(&params.g_tilde.to_bytes());
        ctx.set_verkey(&vk.X_tilde.to_bytes(),
                       &vk.Y_tilde.iter().flat_map(|y| y.to_bytes()).collect::<Vec<u8>>(), q);
        let mut verdicts = vec![0u8; sigs.len()];
        let st = unsafe { cc_verify_batch(ctx.raw, sigs.len(), q, s1.as_ptr(), s2.as_ptr(), m.as_ptr(),
                                          std::ptr::null(), std::ptr::null(), verdicts.as_mut_ptr(),
                                          std::ptr::null_mut(), 0) };
        assert_eq!(st, 0, "{}", ctx.status_str(st));
        verdicts.into_iter().map(|v| v == 1).collect()
    }

    /// Batch form of `Signature::aggregate` (signature.rs:448-470).
    pub fn aggregate_batch(threshold: usize, batches: &[Vec<(usize, Signature)>], ctx: &HipCtx) -> Vec<Signature> {
        if batches.is_empty() { return Vec::new(); }
        let len = batches[0].len();
        assert!(batches.iter().all(|b| b.len() == len), "every batch has the same length");  // len-guard
        assert!(len >= threshold);                                   // signature.rs:449
        let ids: Vec<u64> = batches.iter().flatten().map(|(i, _)| *i as u64).collect();
        let s1: Vec<u8> = batches.iter().flatten().flat_map(|(_, s)| s.sigma_1.to_bytes()).collect();
        let s2: Vec<u8> = batches.iter().flatten().flat_map(|(_, s)| s.sigma_2.to_bytes()).collect();
        let sb = ctx.sig_bytes();
        assert!(s1.len() == ids.len() * sb && s2.len() == ids.len() * sb, "signature encodings");  // len-guard
        let (mut o1, mut o2) = (vec![0u8; sb * batches.len()], vec![0u8; sb * batches.len()]);
        let st = unsafe { cc_signature_aggregate_batch(ctx.raw, batches.len(), len, threshold, ids.as_ptr(),
                                                       s1.as_ptr(), s2.as_ptr(), o1.as_mut_ptr(), o2.as_mut_ptr()) };
        assert_eq!(st, 0, "{}", ctx.status_str(st));
        o1.chunks(sb).zip(o2.chunks(sb)).map(|(a, b)| Signature {
            sigma_1: SignatureGroup::from_bytes(a).unwrap(), sigma_2: SignatureGroup::from_bytes(b).unwrap() }).collect()
    }
}

fn pack(msgs: &[Vec<u8>]) -> (Vec<u8>, Vec<u64>) {
    let mut offs = vec![0u64];
    let mut data = Vec::new();
    for m in msgs { data.extend_from_slice(m); offs.push(data.len() as u64); }
    (data, offs)
}

impl Params {
    /// Params::new (signature.rs:22-32) with every from_msg_hash on the GPU, one call per group.
    pub fn new_hip(msg_count: usize, label: &[u8], ctx: &HipCtx) -> Params {
        let (sg, og) = if ctx.mode() == CC_SIG_G2 { (2, 1) } else { (1, 2) };
        let eb = |g: c_int| if g == 1 { 97 } else { 192 };
        let mut sig_msgs = vec![[label, b" : g"].concat()];
        for i in 0..msg_count { sig_msgs.push([label, format!(" : y{}", i).as_bytes()].concat()); }
        let (data, offs) = pack(&sig_msgs);
        let mut sig = vec![0u8; sig_msgs.len() * eb(sg)];
        ctx.check(unsafe { cc_hash_to_curve(ctx.raw, sg, sig_msgs.len(), data.as_ptr(), offs.as_ptr(), sig.as_mut_ptr()) });
        let (data, offs) = pack(&[[label, b" : g_tilde"].concat()]);
        let mut gt = vec![0u8; eb(og)];
        ctx.check(unsafe { cc_hash_to_curve(ctx.raw, og, 1, data.as_ptr(), offs.as_ptr(), gt.as_mut_ptr()) });
        let chunks: Vec<&[u8]> = sig.chunks(eb(sg)).collect();
        Params { g: SignatureGroup::from_bytes(chunks[0]).unwrap(),
                 g_tilde: OtherGroup::from_bytes(&gt).unwrap(),
                 h: chunks[1..].iter().map(|c| SignatureGroup::from_bytes(c).unwrap()).collect() }
    }
}

impl BlindSignature {
    /// BlindSignature::new (signature.rs:382-433) for n requests under one Sigkey; every request
    /// has k hidden and q - k known messages.
    pub fn new_batch(reqs: &[SignatureRequest], sigkey: &Sigkey, ctx: &HipCtx) -> Vec<BlindSignature> {
        let (n, q) = (reqs.len(), sigkey.y.len());
        if n == 0 { return Vec::new(); }
        let k = reqs[0].ciphertexts.len();
        assert!(k <= q && reqs.iter().all(|r| r.ciphertexts.len() == k && r.known_messages.len() == q - k),
                "every request has k hidden and q - k known messages");  // len-guard
        let cm: Vec<u8> = reqs.iter().flat_map(|r| r.commitment.to_bytes()).collect();
        let kn: Vec<u8> = reqs.iter().flat_map(|r| r.known_messages.iter().flat_map(|m| m.to_bytes())).collect();
        let ct: Vec<u8> = reqs.iter().flat_map(|r| r.ciphertexts.iter()
                              .flat_map(|c| [c.0.to_bytes(), c.1.to_bytes()].concat())).collect();
        let y: Vec<u8> = sigkey.y.iter().flat_map(|v| v.to_bytes()).collect();
        let sb = ctx.sig_bytes();
        assert_eq!(cm.len(), n * sb, "commitment encodings");  // len-guard
        let (mut h, mut c1, mut c2) = (vec![0u8; n * sb], vec![0u8; n * sb], vec![0u8; n * sb]);
        ctx.check(unsafe { cc_blind_sign_batch(ctx.raw, n, q, k, cm.as_ptr(), kn.as_ptr(), ct.as_ptr(),
                                               sigkey.x.to_bytes().as_ptr(), y.as_ptr(),
                                               h.as_mut_ptr(), c1.as_mut_ptr(), c2.as_mut_ptr()) });
        (0..n).map(|i| BlindSignature {
            h: SignatureGroup::from_bytes(&h[i * sb..(i + 1) * sb]).unwrap(),
            blinded: (SignatureGroup::from_bytes(&c1[i * sb..(i + 1) * sb]).unwrap(),
                      SignatureGroup::from_bytes(&c2[i * sb..(i + 1) * sb]).unwrap()) }).collect()
    }
}

/// PedersenVSS::verify_share (keygen.rs:332-351) for n shares; share i is checked against
/// commitment set set_of[i] (each set t x G1 bytes).
pub fn verify_shares_batch(t: usize, g: &G1, h: &G1, sets: &[Vec<G1>], set_of: &[u32], ids: &[u64],
                           shares: &[(FieldElement, FieldElement)], ctx: &HipCtx) -> Vec<bool> {
    assert!(set_of.len() == ids.len() && shares.len() == ids.len(), "one set, id and share per check");  // len-guard
    assert!(sets.iter().all(|s| s.len() == t), "every commitment set has t points");  // len-guard
    assert!(set_of.iter().all(|&k| (k as usize) < sets.len()), "set index in range");  // len-guard
    let cm: Vec<u8> = sets.iter().flatten().flat_map(|c| c.to_bytes()).collect();
    let sh: Vec<u8> = shares.iter().flat_map(|(s, st)| [s.to_bytes(), st.to_bytes()].concat()).collect();
    let mut v = vec![0u8; ids.len()];
    ctx.check(unsafe { cc_vss_verify_batch(ctx.raw, ids.len(), t, g.to_bytes().as_ptr(), h.to_bytes().as_ptr(),
                                           cm.as_ptr(), sets.len(), set_of.as_ptr(), ids.as_ptr(), sh.as_ptr(),
                                           v.as_mut_ptr()) });
    v.into_iter().map(|b| b == 1).collect()
}

impl Verkey {
    /// Batch form of `Verkey::aggregate` (signature.rs:483-526): n aggregations of `len` (id, Verkey)
    /// entries each; only the first `threshold` are used (HashSet semantics of the ids as there).
    pub fn aggregate_batch(threshold: usize, batches: &[Vec<(usize, &Verkey)>], ctx: &HipCtx) -> Vec<Verkey> {
        if batches.is_empty() { return Vec::new(); }
        let (n, len) = (batches.len(), batches[0].len());
        assert!(batches.iter().all(|b| b.len() == len), "every batch has the same length");  // len-guard
        assert!(len >= threshold);                                   // signature.rs:484
        let q = batches[0][0].1.Y_tilde.len();
        assert!(batches.iter().flatten().all(|(_, vk)| vk.Y_tilde.len() == q));  // signature.rs:486-488
        let ids: Vec<u64> = batches.iter().flatten().map(|(i, _)| *i as u64).collect();
        let x: Vec<u8> = batches.iter().flatten().flat_map(|(_, vk)| vk.X_tilde.to_bytes()).collect();
        let y: Vec<u8> = batches.iter().flatten()
            .flat_map(|(_, vk)| vk.Y_tilde.iter().flat_map(|v| v.to_bytes())).collect();
        let ob = ctx.oth_bytes();
        assert!(x.len() == ids.len() * ob && y.len() == ids.len() * q * ob, "verkey encodings");  // len-guard
        let (mut ox, mut oy) = (vec![0u8; n * ob], vec![0u8; n * q * ob]);
        ctx.check(unsafe { cc_verkey_aggregate_batch(ctx.raw, n, len, threshold, q, ids.as_ptr(), x.as_ptr(),
                                                     y.as_ptr(), ox.as_mut_ptr(), oy.as_mut_ptr()) });
        (0..n).map(|i| Verkey {
            X_tilde: OtherGroup::from_bytes(&ox[i * ob..(i + 1) * ob]).unwrap(),
            Y_tilde: (0..q).map(|j| OtherGroup::from_bytes(&oy[(i * q + j) * ob..(i * q + j + 1) * ob]).unwrap())
                .collect::<Vec<OtherGroup>>().into() }).collect()
    }
}

/// PoKOfSignatureProof::verify (ps_sig, called at pok_sig.rs:103-105) for n proofs against one verkey:
/// each proof as its serialized parts (sigma'_1, sigma'_2, J, Schnorr commitment T, responses ordered
/// [g~, Y~_i for hidden i ascending] as ps_sig builds them), one challenge and the revealed messages
/// (indices shared by the batch, ascending).  CC_ERR_BASES_EXPS -> ps_sig's UnequalNoOfBasesExponents.
pub fn pok_verify_batch(proofs: &[(Vec<u8>, Vec<u8>, Vec<u8>, Vec<u8>, Vec<FieldElement>)], chal: &[FieldElement],
                        revealed_idx: &[u64], revealed_msgs: &[Vec<FieldElement>], vk: &Verkey, params: &Params,
                        ctx: &HipCtx) -> Vec<bool> {
    let (n, q, r) = (proofs.len(), vk.Y_tilde.len(), revealed_idx.len());
    if n == 0 { return Vec::new(); }
    let nresp = proofs[0].4.len();
    let (sb, ob) = (ctx.sig_bytes(), ctx.oth_bytes());
    assert_eq!(chal.len(), n, "one challenge per proof");  // len-guard
    assert!(revealed_msgs.len() == n && revealed_msgs.iter().all(|m| m.len() == r),
            "r revealed messages per proof");  // len-guard
    assert!(proofs.iter().all(|p| p.4.len() == nresp), "the same response count for every proof");  // len-guard
    assert!(proofs.iter().all(|p| p.0.len() == sb && p.1.len() == sb && p.2.len() == ob && p.3.len() == ob),
            "proof part encodings (sigma'_1, sigma'_2: SignatureGroup; J, T: OtherGroup)");  // len-guard
    ctx.set_params(&params.g_tilde.to_bytes());
    ctx.set_verkey(&vk.X_tilde.to_bytes(), &vk.Y_tilde.iter().flat_map(|y| y.to_bytes()).collect::<Vec<u8>>(), q);
    let cat = |f: &dyn Fn(&(Vec<u8>, Vec<u8>, Vec<u8>, Vec<u8>, Vec<FieldElement>)) -> Vec<u8>| -> Vec<u8> {
        proofs.iter().flat_map(|p| f(p)).collect()
    };
    let (s1, s2, j, t) = (cat(&|p| p.0.clone()), cat(&|p| p.1.clone()), cat(&|p| p.2.clone()), cat(&|p| p.3.clone()));
    let resp = cat(&|p| p.4.iter().flat_map(|v| v.to_bytes()).collect());
    let ch: Vec<u8> = chal.iter().flat_map(|c| c.to_bytes()).collect();
    let rm: Vec<u8> = revealed_msgs.iter().flatten().flat_map(|m| m.to_bytes()).collect();
    let mut v = vec![0u8; n];
    ctx.check(unsafe { cc_pok_verify_batch(ctx.raw, n, q, r, nresp, s1.as_ptr(), s2.as_ptr(), j.as_ptr(), t.as_ptr(),
                                           resp.as_ptr(), ch.as_ptr(), revealed_idx.as_ptr(), rm.as_ptr(),
                                           v.as_mut_ptr(), std::ptr::null_mut()) });
    v.into_iter().map(|b| b == 1).collect()
}

#[allow(dead_code)]
const _MODE_TYPE: c_int = CC_SIG_G2;
