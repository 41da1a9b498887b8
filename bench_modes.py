"""bench.py modes for BASELINE configs 4 and 5 (imported by bench.py; also the synthetic-data
generators of the GPU property tests).

config 4 (--mode aggregate): Threshold aggregation at scale — per credential one
  Signature::aggregate (signature.rs:448-470) over the partial signatures of a seeded random
  67-subset of n = 100 issuers, and one Verkey::aggregate (signature.rs:483-526) of the same
  subset's verkeys from the resident issuer table (cc_set_issuers).  10,000 credentials per GPU.
verify with per-credential verkeys (--mode verify-pervk / verify-pervk-g1): config 2's size (65,536
  credentials, q = 6) where every credential carries ITS OWN verkey, the reference's per-call
  Signature::verify(msgs, vk, params) (signature.rs:473-478): a variable-base Straus MSM per credential.
config 5 (--mode pok): PoKOfSignatureProof::verify (ps_sig [EXT], reference pok_sig.rs:103-105),
  q = 32, revealed {3,5,7,11,13,17,19,23}, 65,536 proofs per GPU; 1/16 with a corrupted response.

All group elements are k*G for known scalars k, produced by the product's GPU fixed-base
multiplication; expected outputs are known by construction and checked after the timed region.
"""
import ctypes
import json
import os
import time

import numpy as np

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
REVEALED = [3, 5, 7, 11, 13, 17, 19, 23]


def _fr(rng):
    return int.from_bytes(rng.bytes(32), "big") % R


def _be(v):
    return int(v % R).to_bytes(48, "big")


def _poly(c, x):
    acc = 0
    for a in reversed(c):
        acc = (acc * x + a) % R
    return acc


def make_aggregate_batch(ctx, mode, n, t=67, n_iss=100, q=6, seed=4):
    """Shamir-shared issuer keys (degree t-1) so any t-subset aggregates to the master key:
    X~ = x g~, Y~_j = y_j g~ exactly (the reference's check_key_aggregation, signature.rs:554-559)."""
    import coconut
    rng = np.random.default_rng(seed)
    og, sg = (1, 2) if mode == 0 else (2, 1)
    gen = {1: coconut.G1_GENERATOR, 2: coconut.G2_GENERATOR}
    ob, sb = (97, 192) if mode == 0 else (192, 97)
    fx = [_fr(rng) for _ in range(t)]
    fy = [[_fr(rng) for _ in range(t)] for _ in range(q)]
    gk = _fr(rng) or 1
    iss = np.arange(1, n_iss + 1, dtype=np.uint64)
    xk = [_poly(fx, int(i)) for i in iss]
    yk = [[_poly(fy[j], int(i)) for j in range(q)] for i in iss]
    sc = b"".join(_be(xk[k] * gk) + b"".join(_be(yk[k][j] * gk) for j in range(q)) for k in range(n_iss))
    keys = coconut.fixed_base_mul(ctx, og, gen[og], sc)
    X = b"".join(keys[(k * (q + 1)) * ob:(k * (q + 1) + 1) * ob] for k in range(n_iss))
    Y = b"".join(keys[(k * (q + 1) + 1) * ob:(k * (q + 1) + 1 + q) * ob] for k in range(n_iss))
    master = coconut.fixed_base_mul(ctx, og, gen[og], b"".join(_be(v * gk) for v in [fx[0]] + [fy[j][0] for j in range(q)]))
    ids = np.empty((n, t), dtype=np.uint64)
    hk, e2, exp2 = [], [], []
    for i in range(n):
        sub = rng.choice(n_iss, size=t, replace=False)
        ids[i] = iss[sub]
        m = [_fr(rng) for _ in range(q)]
        k = _fr(rng) or 1
        hk.append(k)
        for s_ in sub:
            e2.append(_be(k * (xk[s_] + sum(yk[s_][j] * m[j] for j in range(q)))))
        exp2.append(_be(k * (fx[0] + sum(fy[j][0] * m[j] for j in range(q)))))
    s1one = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(_be(k) for k in hk))
    s1 = b"".join(s1one[i * sb:(i + 1) * sb] * t for i in range(n))  # every entry carries sigma_1 = h
    s2 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(e2))
    want_s2 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(exp2))
    return dict(mode=mode, n=n, t=t, q=q, iss=iss, X=X, Y=Y, ids=ids, s1=s1, s2=s2, want_s1=s1one,
                want_s2=want_s2, want_X=master[:ob], want_Y=master[ob:], ob=ob, sb=sb)


def make_pok_batch(ctx, mode, n, q=32, revealed=REVEALED, seed=5, bad_every=16):
    """ps_sig PoK proofs with known discrete logs (oracle/coconut_ref.py pok_init / gen_proof):
    sigma' = (r1 h, r1 (sigma_2 + r2 h)), J = (r2 + sum_hidden y_i m_i) g~, T = (b_0 + sum y_i b_i) g~,
    responses b_i - chal * secret_i."""
    import coconut
    rng = np.random.default_rng(seed)
    og, sg = (1, 2) if mode == 0 else (2, 1)
    gen = {1: coconut.G1_GENERATOR, 2: coconut.G2_GENERATOR}
    x = _fr(rng)
    y = [_fr(rng) for _ in range(q)]
    gk = _fr(rng) or 1
    ob = 97 if og == 1 else 192
    vk = coconut.fixed_base_mul(ctx, og, gen[og], b"".join(_be(v * gk) for v in [x] + y + [1]))
    X, Y, g_tilde = vk[:ob], vk[ob:ob * (q + 1)], vk[ob * (q + 1):]
    hidden = [i for i in range(q) if i not in revealed]
    s1s, s2s, js, ts, resp, chal, rev = [], [], [], [], [], [], []
    expect = np.ones(n, dtype=np.uint8)
    for p in range(n):
        m = [_fr(rng) for _ in range(q)]
        k, r1, r2, c = _fr(rng) or 1, _fr(rng) or 1, _fr(rng), _fr(rng)
        s = (x + sum(y[i] * m[i] for i in range(q))) % R
        s1s.append(_be(k * r1))
        s2s.append(_be(r1 * k * (s + r2)))
        secrets = [r2] + [m[i] for i in hidden]
        ylog = [1] + [y[i] for i in hidden]
        bl = [_fr(rng) for _ in secrets]
        js.append(_be(gk * sum(a * b for a, b in zip(ylog, secrets))))
        ts.append(_be(gk * sum(a * b for a, b in zip(ylog, bl))))
        rs = [(b - c * sc) % R for b, sc in zip(bl, secrets)]
        if bad_every and p % bad_every == bad_every - 1:
            rs[-1] = (rs[-1] + 5) % R
            expect[p] = 0
        resp.append(b"".join(_be(v) for v in rs))
        chal.append(_be(c))
        rev.append(b"".join(_be(m[i]) for i in revealed))
    S1 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(s1s))
    S2 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(s2s))
    J = coconut.fixed_base_mul(ctx, og, gen[og], b"".join(js))
    T = coconut.fixed_base_mul(ctx, og, gen[og], b"".join(ts))
    return dict(mode=mode, n=n, q=q, revealed=list(revealed), X=X, Y=Y, g_tilde=g_tilde, s1=S1, s2=S2, J=J, T=T,
                resp=b"".join(resp), chal=b"".join(chal), rev=b"".join(rev), nresp=len(hidden) + 1, expect=expect)


def make_pervk_batch(ctx, mode, n, q, seed, bad_every=16):
    """n credentials, each under ITS OWN verkey (x_i, y_ij uniform in Fr; X~_i = x_i g~, Y~_ij = y_ij g~
    built by the product's cc_fixed_base_mul), uniform messages in Fr, sigma_1 = k G,
    sigma_2 = k (x_i + sum y_ij m_ij) G; every bad_every-th corrupted, cycling sigma_2 + G / m_0 + 1 /
    sigma_2 under another credential's key."""
    import coconut
    rng = np.random.default_rng(seed)
    og, sg = (1, 2) if mode == 0 else (2, 1)
    gen = {1: coconut.G1_GENERATOR, 2: coconut.G2_GENERATOR}
    gk = _fr(rng) or 1
    g_tilde = coconut.fixed_base_mul(ctx, og, gen[og], _be(gk))
    vk_sc, e1, e2, mb = [], [], [], []
    expect = np.ones(n, np.uint8)
    sks = [[_fr(rng) for _ in range(q + 1)] for _ in range(n)]
    for i in range(n):
        row = sks[i]
        m = [_fr(rng) for _ in range(q)]  # the messages the verifier is given
        k = _fr(rng) or 1
        vk_sc.extend(v * gk % R for v in row)
        x, signed = row[0], m
        kind = (i // bad_every) % 3 if bad_every and i % bad_every == bad_every - 1 else -1
        if kind >= 0:
            expect[i] = 0
        if kind == 1:
            signed = [(m[0] + 1) % R] + m[1:]  # signed over m_0 + 1
        elif kind == 2:
            x = sks[(i + 1) % n][0]  # signed under another credential's x
        e = k * (x + sum(y * mm for y, mm in zip(row[1:], signed))) % R
        if kind == 0:
            e = (e + 1) % R  # sigma_2 + G
        e1.append(_be(k))
        e2.append(_be(e))
        mb.append(b"".join(_be(v) for v in m))
    ob = 97 if og == 1 else 192
    vk = coconut.fixed_base_mul(ctx, og, gen[og], b"".join(_be(v) for v in vk_sc))
    X = b"".join(vk[(i * (q + 1)) * ob:(i * (q + 1) + 1) * ob] for i in range(n))
    Y = b"".join(vk[(i * (q + 1) + 1) * ob:(i + 1) * (q + 1) * ob] for i in range(n))
    s1 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(e1))
    s2 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(e2))
    return dict(X=X, Y=Y, g_tilde=g_tilde, s1=s1, s2=s2, msgs=b"".join(mb), expect=expect)


def _timed(args, step, dev, dist, ctx, phases=True):
    import torch
    from bench import _max_over_ranks
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.timing(phases)
    phase = np.zeros(3)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if phases:
            phase += np.array(ctx.last_timing())
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    ctx.timing(False)
    return _max_over_ranks(el, dist, dev), phase / max(args.steps, 1)


# Issuer-table window width the aggregate modes opt into (cc_set_table_bits): 16-bit windows, 16 windows a
# scalar — 70 GB of tables for 100 issuers x 7 G1 keys (SigG2), 141 GB for 7 G2 keys (SigG1), built in
# 0.35 / 1.3 s at setup.  The library's default (<= 16 GiB) picks 13 / 12 bits (20 / 22 windows);
# measured 16 against the default: config 4 +5.5 % (SigG2), +29 % (SigG1) (profiles/r04/issbits).
BENCH_ISS_BITS = 16


def iss_bits_for(args):
    """Issuer-table window width (cc_set_table_bits): --iss-bits (0: the library's choice by memory), else
    BENCH_ISS_BITS."""
    b = getattr(args, "iss_bits", None)
    return BENCH_ISS_BITS if b is None else b


def iss_table_gib(bits, nbases, g2):
    return round(nbases * -(-256 // bits) * ((1 << bits) - 1) * (192 if g2 else 96) / 2 ** 30, 1)


def bench_aggregate(args):
    import torch
    import coconut
    from bench import _dist_setup, to_dev, MADS_PER_M, peak_mad_per_s, opcounts
    world, rank, local, dist = _dist_setup()
    dev = torch.device("cuda", local)
    n = args.n or 10000
    sigm = 1 if args.mode.endswith("-g1") else 0  # aggregate-g1: SigG1 (sigma in G1, issuer keys in G2)
    ctx = coconut.Context(local, coconut.GroupMode.SIG_G1 if sigm else coconut.GroupMode.SIG_G2)
    t_set = time.perf_counter()
    b = make_aggregate_batch(ctx, sigm, n, seed=4000 + rank)
    gen_s = time.perf_counter() - t_set
    t_iss = time.perf_counter()
    ctx.set_table_bits(0, iss_bits_for(args))
    ctx.set_issuers(b["iss"], b["X"], b["Y"], b["q"])
    iss_ms = (time.perf_counter() - t_iss) * 1e3
    t, q, sb, ob = b["t"], b["q"], b["sb"], b["ob"]
    d_ids = torch.from_numpy(b["ids"].view(np.int64).copy()).to(dev)
    d_s1, d_s2 = to_dev(b["s1"], dev), to_dev(b["s2"], dev)
    o1 = torch.zeros(n * sb, dtype=torch.uint8, device=dev)
    o2 = torch.zeros(n * sb, dtype=torch.uint8, device=dev)
    oX = torch.zeros(n * ob, dtype=torch.uint8, device=dev)
    oY = torch.zeros(n * q * ob, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    sh = ctypes.c_void_p(stream.cuda_stream)
    lib = coconut._lib.lib
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    # both aggregations of each credential over its one id list: ONE Lagrange launch serves the signature
    # and the verkey MSM (cc_aggregate_credential_batch_device); timing = (Lagrange, sig MSM, vk MSM)

    def step():
        st = lib.cc_aggregate_credential_batch_device(ctx.h, n, t, t, P(d_ids), P(d_s1), P(d_s2), P(o1), P(o2),
                                                      P(oX), P(oY), sh)
        if st:
            raise RuntimeError(f"aggregate: {lib.cc_status_str(st).decode()}")

    el, phase = _timed(args, step, dev, dist, ctx)
    torch.cuda.synchronize(dev)
    if ctx.device_error(sh.value):
        raise SystemExit("aggregation raised a device error — refusing to report a number")
    ok = (bytes(o2.cpu().numpy()) == b["want_s2"] and bytes(o1.cpu().numpy()) == b["want_s1"]
          and bytes(oX.cpu().numpy()) == b["want_X"] * n and bytes(oY.cpu().numpy()) == b["want_Y"] * n)
    if not ok:
        raise SystemExit("aggregation outputs disagree with construction — refusing to report a number")
    value = n * world * args.steps / el
    opt_bits = ctx.table_bits()[1]
    from bench import default_tables_leg

    def agg_ok():
        return (bytes(o2.cpu().numpy()) == b["want_s2"] and bytes(oX.cpu().numpy()) == b["want_X"] * n
                and bytes(oY.cpu().numpy()) == b["want_Y"] * n and not ctx.device_error(sh.value))
    dflt = default_tables_leg(args, ctx, lambda: ctx.set_issuers(b["iss"], b["X"], b["Y"], b["q"]), step, agg_ok,
                              n, dev, dist, table_kind="issuer")
    dflt["issuer_table_gib"] = iss_table_gib(dflt["table_bits"], 100 * (q + 1), bool(sigm))
    if rank == 0:
        peak = peak_mad_per_s()
        # phases: Lagrange, Signature::aggregate (Verkey::aggregate runs concurrently on the side stream),
        # the rest of Verkey::aggregate after it; the roofline counts both MSMs' mads over their common span
        sig_ms, vk_ms = phase[1], phase[2]
        msm_ms = sig_ms + vk_ms
        # the op-count fixture covers SigG2; SigG1 lines report times only
        counts = opcounts("aggregate_sigg1_t67" if sigm else "aggregate_sigg2_t67")
        ach = (counts["straus_sigma2"] + counts["fixed_verkey"]) * MADS_PER_M * n / (msm_ms * 1e-3)
        dom = "signature_msm+verkey_msm (concurrent)"
        from bench import kernel_pmc_report
        rk = kernel_pmc_report("aggregate-g1" if sigm else "aggregate")
        out = {
            "metric": "aggregated credentials/sec (Signature::aggregate + Verkey::aggregate, t=67 of n=100)",
            "value": round(value, 1), "unit": "credentials/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (Fp 12x32-bit Montgomery limbs, integer-only)",
            "data": "synthetic (seeded Shamir-shared issuer keys; random 67-subsets; outputs checked = x g~, y_j g~, "
                    "(x + sum y m) h)",
            "config": {"workload": f"config4: {n:,} credentials per GPU, t=67 of n=100 issuers, msg_count={q}, "
                                   + ("SigG1" if sigm else "SigG2"),
                       "credentials_per_gpu": n, "threshold": t, "issuers": 100,
                       "parallelism": f"shard-by-credential x{world}", "issuer_table_bits": opt_bits,
                       "issuer_table_gib": iss_table_gib(opt_bits, 100 * (q + 1), bool(sigm))},
            **__import__("bench").lib_info(),
            "default_tables": dflt,
            "roofline": {"bound": "valu-int", "kernel": dom, "achieved": round(ach / 1e12, 3),
                         "peak": round(peak / 1e12, 3), "unit": "Tmad/s (v_mad_u64_u32, 32x32->64)",
                         "frac": round(ach / peak, 4),
                         "traffic": (rk or {}).get("kernels", {}).get(
                             "k_msm_straus<cc::Fp, 16>" if sigm else "k_msm_straus_g2lz_g", {}).get("hbm_bytes_per_launch"),
                         "traffic_unit": "HBM-side bytes per launch of the Straus kernel (PMC, 2 x FETCH_SIZE + "
                                         "WRITE_SIZE)"},
            "kernels": {"lagrange_ms": round(phase[0], 3), "msm_ms": round(msm_ms, 3),
                        "signature_msm_ms": round(sig_ms, 3), "verkey_msm_tail_ms": round(vk_ms, 3)},
            "rocprof_kernels": rk,
            "setup": {"issuer_tables_ms": round(iss_ms, 1), "synthetic_data_s": round(gen_s, 2)},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_aggregate(b, value)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


def cpu_aggregate(b, value):
    """oracle/c oc_signature_aggregate + oc_verkey_aggregate per credential, on the box's CPU share and on
    one thread, each sample >= 2 s (cpu_pool_rate)."""
    from bench import _oracle, cpu_pool_rate, cpu_report, host_threads
    oc = _oracle()
    t, q, sb, ob = b["t"], b["q"], b["sb"], b["ob"]

    def one(i):
        o1 = ctypes.create_string_buffer(sb)
        o2 = ctypes.create_string_buffer(sb)
        oX = ctypes.create_string_buffer(ob)
        oY = ctypes.create_string_buffer(ob * q)
        ids = np.ascontiguousarray(b["ids"][i])
        oc.oc_signature_aggregate(b["mode"], ctypes.c_size_t(t), ctypes.c_size_t(t), ids.ctypes.data_as(ctypes.c_void_p),
                                  b["s1"][i * t * sb:(i + 1) * t * sb], b["s2"][i * t * sb:(i + 1) * t * sb], o1, o2)
        rows = [int(v) - 1 for v in ids]
        Xs = b"".join(b["X"][r * ob:(r + 1) * ob] for r in rows)
        Ys = b"".join(b["Y"][r * q * ob:(r + 1) * q * ob] for r in rows)
        oc.oc_verkey_aggregate(b["mode"], ctypes.c_size_t(t), ctypes.c_size_t(t), ctypes.c_size_t(q),
                               ids.ctypes.data_as(ctypes.c_void_p), Xs, Ys, oX, oY)
        return o2.raw == b["want_s2"][i * sb:(i + 1) * sb] and oX.raw == b["want_X"]

    thr = host_threads()
    mt = cpu_pool_rate(one, b["n"], thr, 2.5)
    st = cpu_pool_rate(one, b["n"], 1, 2.5)
    return cpu_report(value, "credentials/s", "oc_signature_aggregate + oc_verkey_aggregate per credential", mt, st,
                      thr, all(mt[3]) and all(st[3]))


def bench_pok(args):
    import torch
    import coconut
    from bench import _dist_setup, to_dev, MADS_PER_M, peak_mad_per_s, opcounts
    world, rank, local, dist = _dist_setup()
    dev = torch.device("cuda", local)
    n = args.n or 65536
    sigm = 1 if args.mode.endswith("-g1") else 0  # pok-g1: SigG1 (sigma in G1, Schnorr MSM in G2)
    ctx = coconut.Context(local, coconut.GroupMode.SIG_G1 if sigm else coconut.GroupMode.SIG_G2)
    t0 = time.perf_counter()
    b = make_pok_batch(ctx, sigm, n, seed=5000 + rank)
    gen_s = time.perf_counter() - t0
    ctx.set_params(b["g_tilde"])
    from bench import vk_bits_for
    ctx.set_table_bits(vk_bits_for(args), 0)
    ctx.set_verkey(b["X"], b["Y"])
    q, r, nresp = b["q"], len(b["revealed"]), b["nresp"]
    D = {k: to_dev(b[k], dev) for k in ("s1", "s2", "J", "T", "resp", "chal", "rev")}
    # --inflight K batches on one context (cc_set_concurrency) and K streams, round-robin
    K = max(1, getattr(args, "inflight", 1))
    ctx.set_concurrency(K)
    d_vs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(K)]
    d_v = d_vs[0]
    ridx = (ctypes.c_uint64 * r)(*b["revealed"])
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    for s_ in streams:
        s_.wait_stream(torch.cuda.current_stream(dev))
    shs = [ctypes.c_void_p(s_.cuda_stream) for s_ in streams]
    lib = coconut._lib.lib
    P = lambda k: ctypes.c_void_p(D[k].data_ptr())  # noqa: E731
    rr = [0]

    def step():
        k = rr[0] % K
        rr[0] += 1
        st = lib.cc_pok_verify_batch_device(ctx.h, n, q, r, nresp, P("s1"), P("s2"), P("J"), P("T"), P("resp"),
                                            P("chal"), ridx, P("rev"), ctypes.c_void_p(d_vs[k].data_ptr()), None,
                                            shs[k])
        if st:
            raise RuntimeError(f"cc_pok_verify_batch_device: {lib.cc_status_str(st).decode()}")

    el, phase_ms = _timed(args, step, dev, dist, ctx, phases=K == 1)
    for k in range(K):
        if rr[0] > k and not np.array_equal(d_vs[k].cpu().numpy(), b["expect"]):
            raise SystemExit("PoK verdicts disagree with construction — refusing to report a number")
    K0 = K
    if K > 1:  # the per-kernel table from a separate single-batch pass
        ctx.set_concurrency(1)
        K = 1
        rr[0] = 0
        ctx.timing(True)
        ph = np.zeros(3)
        for _ in range(min(args.steps, 5)):
            step()
            ph += np.array(ctx.last_timing())
        ctx.timing(False)
        phase_ms = ph / max(min(args.steps, 5), 1)
    value = n * world * args.steps / el
    from bench import default_tables_leg, table_config
    opt_in = table_config(ctx, q)

    def rebind_dflt():  # the library-default tables at the headline's batches in flight
        nonlocal K
        ctx.set_verkey(b["X"], b["Y"])
        ctx.set_concurrency(K0)
        K = K0
        rr[0] = 0

    def check_dflt():
        ok = all(np.array_equal(d_vs[k].cpu().numpy(), b["expect"]) for k in range(min(K0, rr[0])))
        ctx.set_concurrency(1)
        return ok
    dflt = default_tables_leg(args, ctx, rebind_dflt, step, check_dflt, n, dev, dist, unit="proofs/s")
    dflt["batches_in_flight"] = K0
    dflt.update(table_config(ctx, q))
    from bench import latency_of

    def pok_launch(nn, d_vv, sh):  # the first nn proofs (proof-major inputs)
        st = lib.cc_pok_verify_batch_device(ctx.h, nn, q, r, nresp, P("s1"), P("s2"), P("J"), P("T"), P("resp"),
                                            P("chal"), ridx, P("rev"), ctypes.c_void_p(d_vv.data_ptr()), None, sh)
        if st:
            raise RuntimeError(f"cc_pok_verify_batch_device: {lib.cc_status_str(st).decode()}")
    latency = latency_of(ctx, pok_launch, b["expect"], dev, what="proofs")
    if rank == 0:
        from bench import kernel_table, cpu_info, kernel_pmc_report
        peak = peak_mad_per_s()
        counts = opcounts("pok_sigg1_q32_r8" if sigm else "pok_sigg2_q32_r8")
        kt = kernel_table(phase_ms, n, counts, 2 * 192 + 2 * 97 + (nresp + 1 + r) * 48, peak,
                          "k_prep_pok_g1pl" if sigm else "k_prep_pok_split", "pok-g1" if sigm else "pok")
        dom = max(kt, key=lambda k: kt[k]["ms"])
        out = {
            "metric": "verified PoK-of-signature proofs/sec (msg_count=32, 8 revealed)",
            "value": round(value, 1), "unit": "proofs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32/u32 (pairing kernels: 14 signed 28-bit-radix limbs, lazy; elsewhere 12x32-bit Montgomery; integer-only)",
            "data": "synthetic (seeded; proofs with known discrete logs built on the GPU; 1/16 bad response)",
            "config": {"workload": f"config5: {n:,} PoKOfSignatureProof::verify per GPU, q=32, revealed "
                                   f"{b['revealed']}, " + ("SigG1" if sigm else "SigG2"), "proofs_per_gpu": n,
                       "parallelism": f"shard-by-proof x{world}", **opt_in,
                       "batches_in_flight": max(1, getattr(args, "inflight", 1)),
                       "verkey_tables": "opt-in width (bench); library default <= 4 GiB"},
            **__import__("bench").lib_info(),
            "default_tables": dflt,
            "latency": latency,
            "roofline": {"bound": "valu-int", "kernel": dom, "achieved": kt[dom]["achieved_Tmad_s"],
                         "peak": round(peak / 1e12, 3), "unit": "Tmad/s (v_mad_u64_u32, 32x32->64)",
                         "frac": kt[dom]["frac"], "traffic": kt[dom].get("traffic_bytes"),
                         "traffic_unit": "HBM-side bytes per launch (PMC, 2 x FETCH_SIZE + WRITE_SIZE)"},
            "kernels": kt,
            "rocprof_kernels": kernel_pmc_report("pok-g1" if sigm else "pok"),
            "setup": {"synthetic_data_s": round(gen_s, 2), "verkey_table_bits": opt_in["verkey_table_bits"]},
        }
        if not args.no_cpu_baseline and world == 1:
            from bench import _oracle, cpu_pool_rate, cpu_report, host_threads
            oc = _oracle()
            ridx_c = (ctypes.c_uint64 * r)(*b["revealed"])
            sb, ob = (97, 192) if sigm else (192, 97)

            def one(p):
                gtb = ctypes.create_string_buffer(576)
                v = oc.oc_pok_verify(sigm, ctypes.c_size_t(q), ctypes.c_size_t(r), b["s1"][p * sb:(p + 1) * sb],
                                     b["s2"][p * sb:(p + 1) * sb], b["J"][p * ob:(p + 1) * ob],
                                     b["T"][p * ob:(p + 1) * ob], b["resp"][p * nresp * 48:(p + 1) * nresp * 48],
                                     ctypes.c_size_t(nresp), b["chal"][p * 48:(p + 1) * 48], ridx_c,
                                     b["rev"][p * r * 48:(p + 1) * r * 48], b["X"], b["Y"], b["g_tilde"], gtb)
                return int(v) == int(b["expect"][p])

            thr = host_threads()
            mt = cpu_pool_rate(one, n, thr, 2.5)
            st = cpu_pool_rate(one, n, 1, 2.5)
            out["cpu_baseline"] = cpu_report(value, "proofs/s", "oc_pok_verify per proof", mt, st, thr,
                                             all(mt[3]) and all(st[3]))
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


def bench_pervk(args):
    """Signature::verify with a distinct verkey per credential (cc_verify_batch_pervk_device): 65,536
    credentials, q = 6, inputs resident in HBM; verdicts checked against construction after timing."""
    import torch
    import coconut
    from bench import (_dist_setup, to_dev, MADS_PER_M, peak_mad_per_s, opcounts, kernel_table, lib_info,
                       cpu_baseline_verify)
    world, rank, local, dist = _dist_setup()
    dev = torch.device("cuda", local)
    n, q = args.n or 65536, 6
    mode = 1 if args.mode.endswith("-g1") else 0
    ctx = coconut.Context(local, coconut.GroupMode(mode))
    t0 = time.perf_counter()
    b = make_pervk_batch(ctx, mode, n, q, seed=6000 + rank + 100 * mode)
    gen_s = time.perf_counter() - t0
    ctx.set_params(b["g_tilde"])
    D = [to_dev(b[k], dev) for k in ("s1", "s2", "msgs", "X", "Y")]
    # --inflight K batches on one context (cc_set_concurrency) and K streams, round-robin
    K = max(1, getattr(args, "inflight", 1))
    ctx.set_concurrency(K)
    d_vs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(K)]
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    for s_ in streams:
        s_.wait_stream(torch.cuda.current_stream(dev))
    shs = [ctypes.c_void_p(s_.cuda_stream) for s_ in streams]
    lib = coconut._lib.lib
    P = [ctypes.c_void_p(x.data_ptr()) for x in D]
    rr = [0]

    def step():
        k = rr[0] % K
        rr[0] += 1
        st = lib.cc_verify_batch_pervk_device(ctx.h, n, q, *P, ctypes.c_void_p(d_vs[k].data_ptr()), None, shs[k])
        if st:
            raise RuntimeError(f"cc_verify_batch_pervk_device: {lib.cc_status_str(st).decode()}")

    el, phase_ms = _timed(args, step, dev, dist, ctx, phases=K == 1)
    for k in range(K):
        if rr[0] > k and not np.array_equal(d_vs[k].cpu().numpy(), b["expect"]):
            raise SystemExit("per-verkey verdicts disagree with construction — refusing to report a number")
    if K > 1:  # the per-kernel table from a separate single-batch pass
        ctx.set_concurrency(1)
        K = 1
        rr[0] = 0
        ctx.timing(True)
        ph = np.zeros(3)
        for _ in range(min(args.steps, 5)):
            step()
            ph += np.array(ctx.last_timing())
        ctx.timing(False)
        phase_ms = ph / max(min(args.steps, 5), 1)
    value = n * world * args.steps / el
    from bench import latency_of

    def pervk_launch(nn, d_vv, sh):  # the first nn credentials (credential-major inputs)
        st = lib.cc_verify_batch_pervk_device(ctx.h, nn, q, *P, ctypes.c_void_p(d_vv.data_ptr()), None, sh)
        if st:
            raise RuntimeError(f"cc_verify_batch_pervk_device: {lib.cc_status_str(st).decode()}")
    latency = latency_of(ctx, pervk_launch, b["expect"], dev)
    if rank == 0:
        key = "verify_sigg2_q6_pervk" if mode == 0 else "verify_sigg1_q6_pervk"
        counts = opcounts(key)
        peak = peak_mad_per_s()
        sb, ob = (192, 97) if mode == 0 else (97, 192)
        kt = kernel_table(phase_ms, n, counts, 2 * sb + q * 48 + (q + 1) * ob, peak,
                          "k_prep_sigg2_var" if mode == 0 else "k_prep_sigg1_var", args.mode)
        dom = max(kt, key=lambda k: kt[k]["ms"])
        total = sum(counts.values()) * MADS_PER_M * n
        out = {
            "metric": "verified credentials/sec (msg_count=6), one verkey per credential" + ("" if mode == 0 else " [SigG1]"),
            "value": round(value, 1), "unit": "credentials/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "int32/u32 (lazy 14 x 28-bit signed limbs in the MSM and pairing; integer-only)",
            "data": "synthetic (seeded; 65,536 distinct verkeys x_i g~, y_ij g~ and signatures built on the GPU by "
                    "cc_fixed_base_mul; 1/16 corrupted: sigma_2 + G, m_0 + 1, signed under another key)",
            "config": {"workload": f"Signature::verify with per-credential verkeys: {n:,} per GPU, msg_count=6, "
                                   + ("SigG2" if mode == 0 else "SigG1"),
                       "credentials_per_gpu": n, "msg_count": q, "parallelism": f"shard-by-credential x{world}",
                       "batches_in_flight": max(1, getattr(args, "inflight", 1))},
            **lib_info(),
            "roofline": {"bound": "valu-int", "kernel": dom, "achieved": kt[dom]["achieved_Tmad_s"],
                         "peak": round(peak / 1e12, 3), "unit": "Tmad/s (v_mad_u64_u32, 32x32->64)",
                         "frac": kt[dom]["frac"], "traffic": kt[dom].get("traffic_bytes"),
                         "traffic_unit": "HBM-side bytes per launch (PMC, 2 x FETCH_SIZE + WRITE_SIZE)",
                         "algorithmic_mads_per_credential": round(counts[dom] * MADS_PER_M),
                         "opcount_fixture": f"tests/fixtures/opcount.json {key}",
                         "whole_step_frac": round(total / (el / args.steps) / peak, 4)},
            "kernels": kt,
            "prep_over_miller": round(kt["prep"]["ms"] / kt["miller"]["ms"], 3) if kt["miller"]["ms"] else None,
            "latency": latency,
            "rocprof_kernels": __import__("bench").kernel_pmc_report(args.mode),
            "setup": {"synthetic_data_s": round(gen_s, 2)},
        }
        if not args.no_cpu_baseline and world == 1:
            cb = dict(mode=mode, q=q, n=n, s1=b["s1"], s2=b["s2"], msgs=b["msgs"], X=b["X"], Y=b["Y"],
                      g_tilde=b["g_tilde"], expect=b["expect"], per_vk=True)
            out["cpu_baseline"] = cpu_baseline_verify(cb, value, "per-credential verkeys")
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()
