#!/usr/bin/env python3
"""bench.py — batched Coconut Signature::verify throughput on MI355X (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): a batch of 65,536 independent
msg_count = 6 credential verifies per GPU against one shared aggregated verkey, reference default
group assignment (sigma in G2, verkey in G1).  1/16 of the credentials are corrupted (sigma_2 + G),
so the kernel sees the reject path too.  A "step" is one pass of the hot path over the whole batch:
decode + verkey MSM -> 2-pair Miller loop -> final exponentiation -> verdicts, with the serialized
inputs already resident in HBM (cc_verify_batch_device).

Synthetic data: sigma_1 = k G2, sigma_2 = k (x + sum y_j m_j) G2 with random k, m, x, y — computed
by the product's own GPU fixed-base multiplication (cc_fixed_base_mul), not by the oracle.

Multi-GPU (torch.distributed.run, one process per GPU): each rank verifies its own 65,536
credentials (weak scaling, no data-path collective); value = all credentials / max-over-ranks time.

cpu_baseline: the C restatement in oracle/ (test infrastructure, "port") timed on this host's
cores on a bounded sample of the same credentials (rank 0, N = 1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "coconut-rust_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_PER_GPU = 65536
Q = 6
MADS_PER_FPMUL = 288  # 12 x 12 limb products for a*b plus 12 x 12 for m*p (32x32->64 v_mad_u64_u32)
PEAK_MAD_PER_S = 2.74e13  # measured gfx950 v_mad_u64_u32 issue rate, tools/ubench_int.hip (profiles/)
HBM_PEAK_GBS = 8000.0
# PMC counters of the same build, collected by tools/pmc_round.sh (separate rocprofv3 --pmc passes)
# and summarised by tools/pmc_summary.py; bench.py cannot read counters in a plain run.
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_final", "pmc_summary.json")


def pmc_traffic(kernel_key):
    """HBM-side bytes per launch of the kernel whose name contains kernel_key: 2 x FETCH_SIZE (gfx950
    counts half of wide reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, both KiB; None if absent."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    for name, c in d.items():
        if kernel_key in name and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            return round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
    return None


def fp_mults_per_credential(q=Q):
    """Algorithmic Montgomery multiplications per credential of the implemented algorithm
    (SigG2, shared verkey, fixed-base 8-bit windows), per kernel.  Fp2 mul = 3, Fp2 sqr = 2,
    Fp4 mul = 9, Fp4 sqr = 6, Fp12 mul = 54, Fp12 sqr (CH-SQR2) = 36, cyclotomic sqr = 18,
    Fp inversion = 380 S + 190 M (Fermat, p - 2)."""
    g2_decode = 4 + 7                      # to-Montgomery + on-curve check
    madd = 11                              # Jacobian + affine (7M + 4S)
    prep = 2 * g2_decode + q * 32 * madd * 255 / 256 + 3
    line_dbl, line_add, line_mul = 21, 37, 39
    dbl_step = 36 + 2 * line_dbl + (6 + 4) + 2 * line_mul
    add_step = 2 * line_add + (6 + 4) + 2 * line_mul
    miller = 63 * dbl_step - 36 + 5 * add_step
    f12_inv = 3 * (6 + 9) + 27 + (4 + 570 + 4 + 6) + 27
    easy = f12_inv + 54 + 10 + 54
    pow_x = 63 * 18 + 5 * 54
    hard = (18 + 54) + 5 * pow_x + (54 + 54 + 10 + 54 + 15 + 54 + 10 + 54 + 54 + 15 + 54 + 54)
    return {"prep": prep, "miller": miller, "fexp": easy + hard}


def make_batch(ctx, n, q, seed, bad_every=16):  # bad_every = 0: all valid
    """Synthetic credentials built on the GPU with the product's fixed-base multiplication."""
    import coconut
    rng = np.random.default_rng(seed)
    x = int.from_bytes(rng.bytes(32), "big") % R_ORDER
    y = [int.from_bytes(rng.bytes(32), "big") % R_ORDER for _ in range(q)]
    gt_k = int.from_bytes(rng.bytes(32), "big") % R_ORDER
    gt_k = gt_k or 1
    # verkey relative to g~ = gt_k G1: X~ = x g~, Y~_j = y_j g~
    sc = b"".join(v.to_bytes(48, "big") for v in [x * gt_k % R_ORDER] + [yj * gt_k % R_ORDER for yj in y] + [gt_k])
    pts = coconut.fixed_base_mul(ctx, 1, coconut.G1_GENERATOR, sc)  # verkey + g~ in G1 (SigG2)
    X, Y, g_tilde = pts[:97], pts[97:97 * (q + 1)], pts[97 * (q + 1):]
    m = [[int.from_bytes(rng.bytes(32), "big") % R_ORDER for _ in range(q)] for _ in range(n)]
    ks = [int.from_bytes(rng.bytes(32), "big") % R_ORDER or 1 for _ in range(n)]
    e1, e2 = bytearray(), bytearray()
    expect = np.ones(n, dtype=np.uint8)
    for i in range(n):
        s = (x + sum(yj * mj for yj, mj in zip(y, m[i]))) % R_ORDER
        e = ks[i] * s % R_ORDER
        if bad_every and i % bad_every == bad_every - 1:
            e = (e + 1) % R_ORDER  # sigma_2 + G: must be rejected
            expect[i] = 0
        e1 += ks[i].to_bytes(48, "big")
        e2 += e.to_bytes(48, "big")
    s1 = coconut.fixed_base_mul(ctx, 2, coconut.G2_GENERATOR, bytes(e1))
    s2 = coconut.fixed_base_mul(ctx, 2, coconut.G2_GENERATOR, bytes(e2))
    msgs = b"".join(v.to_bytes(48, "big") for row in m for v in row)
    return dict(X=X, Y=Y, g_tilde=g_tilde, s1=s1, s2=s2, msgs=msgs, expect=expect)


def cpu_baseline(batch, q, threads, target_s=1.5):
    """Time the oracle's C restatement (oc_verify_batch, 64-bit Montgomery, AMCL-class
    algorithm) on `threads` host threads over a bounded sample of the same credentials."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    oc = ctypes.CDLL(so)
    sb = 192
    # calibrate on a small sample, then size the timed sample to ~target_s wall per thread group
    k0 = threads * 4
    ver = ctypes.create_string_buffer(k0)
    t = time.perf_counter()
    oc.oc_verify_batch(0, ctypes.c_size_t(k0), ctypes.c_size_t(q), batch["s1"][:k0 * sb], batch["s2"][:k0 * sb],
                       batch["msgs"][:k0 * q * 48], batch["X"], batch["Y"], 0, batch["g_tilde"], ver, None, threads)
    per = (time.perf_counter() - t) / k0
    k = int(min(len(batch["s1"]) // sb, max(threads * 8, target_s / max(per, 1e-6))))
    k = max(threads, (k // threads) * threads)
    ver = ctypes.create_string_buffer(k)
    t = time.perf_counter()
    oc.oc_verify_batch(0, ctypes.c_size_t(k), ctypes.c_size_t(q), batch["s1"][:k * sb], batch["s2"][:k * sb],
                       batch["msgs"][:k * q * 48], batch["X"], batch["Y"], 0, batch["g_tilde"], ver, None, threads)
    dt = time.perf_counter() - t
    agree = bool(np.array_equal(np.frombuffer(ver.raw, np.uint8), batch["expect"][:k]))
    return {"value": k / dt, "unit": "credentials/s", "cores": threads, "kind": "port",
            "sample": f"{k} credentials of the same batch (q={q}, shared vk, SigG2), {dt:.2f} s wall, "
                      f"oracle/c bls_oracle.c oc_verify_batch, {threads} threads; verdicts agree with "
                      f"construction: {agree}",
            "cpu_seconds": dt * threads}


def _dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    return world, rank, local, dist


def bench_rlc(args):
    """BASELINE config 3: batches of q = 16 credentials verified in RLC batch mode.  Each rank owns
    131,072 credentials (2^20 over 8 GPUs); a step = per-rank partial (delta-weighted Miller product
    of the slice) -> RCCL all-gather of the 580-byte partials -> one final exponentiation on every
    rank -> accept.  All credentials are valid, so the accept path is what is timed; the reject
    path (fallback) is checked once after the timed region."""
    import coconut
    from coconut.dist import DeviceEngine, gather_partials
    world, rank, local, dist = _dist_setup()
    n = args.n if args.n != N_PER_GPU else 131072
    q = 16
    ctx = coconut.Context(local, coconut.GroupMode.SIG_G2)
    batch = make_batch(ctx, n, q, seed=3000 + rank, bad_every=0)
    ctx.set_params(batch["g_tilde"])
    ctx.set_verkey(batch["X"], batch["Y"])
    dev = torch.device("cuda", local)
    up = lambda x: torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)  # noqa: E731
    d_s1, d_s2, d_m = up(batch["s1"]), up(batch["s2"]), up(batch["msgs"])
    eng = DeviceEngine(ctx, n, q, d_s1, d_s2, d_m, base_index=rank * n)

    def step():
        part = eng.partial()
        allp, k = gather_partials(part)
        return eng.finish(allp, k)

    for _ in range(args.warmup):
        assert step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ok = True
    for _ in range(args.steps):
        ok &= step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not ok:
        raise SystemExit("RLC rejected an all-valid batch — refusing to report a number")
    # reject path: one credential of rank 0's slice corrupted -> every rank must reject
    bad = d_s2.clone()
    if rank == 0:
        bad[:192] = d_s2[192:384]
    eng_bad = DeviceEngine(ctx, n, q, d_s1, bad, d_m, base_index=rank * n)
    pb, k = gather_partials(eng_bad.partial())
    if eng_bad.finish(pb, k):
        raise SystemExit("RLC accepted a corrupted batch — refusing to report a number")
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    value = n * world * args.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "verified credentials/sec, RLC batch mode (msg_count=16)",
            "value": round(value, 1), "unit": "credentials/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (Fp 12x32-bit storage, integer-only)",
            "data": "synthetic (seeded; all valid, reject path checked after timing)",
            "config": {"workload": "config3: RLC batch verify, msg_count=16, shared verkey, SigG2",
                       "credentials_per_gpu": n, "msg_count": q,
                       "parallelism": f"shard-by-credential x{world} + RCCL all-gather of Fp12 partials"}}))
    if dist:
        dist.destroy_process_group()
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=N_PER_GPU, help="credentials per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["verify", "rlc"], default="verify",
                    help="verify: config 2 (per-credential verdicts, the headline metric); "
                         "rlc: config 3 (RLC batch mode, q = 16, 131,072 per GPU, RCCL all-gather of partials)")
    args = ap.parse_args()
    if args.mode == "rlc":
        return bench_rlc(args)

    world, rank, local, dist = _dist_setup()
    device = local
    import coconut

    ctx = coconut.Context(device, coconut.GroupMode.SIG_G2)
    n, q = args.n, Q
    t_setup = time.perf_counter()
    batch = make_batch(ctx, n, q, seed=1000 + rank)
    ctx.set_params(batch["g_tilde"])
    t_vk = time.perf_counter()
    ctx.set_verkey(batch["X"], batch["Y"])
    vk_ms = (time.perf_counter() - t_vk) * 1e3
    setup_s = time.perf_counter() - t_setup

    dev = torch.device("cuda", device)
    d_s1 = torch.frombuffer(bytearray(batch["s1"]), dtype=torch.uint8).to(dev)
    d_s2 = torch.frombuffer(bytearray(batch["s2"]), dtype=torch.uint8).to(dev)
    d_m = torch.frombuffer(bytearray(batch["msgs"]), dtype=torch.uint8).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    # a dedicated (non-null) stream, ordered after the uploads; a NULL handle would select the
    # context's own non-blocking stream
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    sh = ctypes.c_void_p(stream.cuda_stream)
    lib = coconut._lib.lib

    def step():
        st = lib.cc_verify_batch_device(ctx.h, n, q, ctypes.c_void_p(d_s1.data_ptr()),
                                        ctypes.c_void_p(d_s2.data_ptr()), ctypes.c_void_p(d_m.data_ptr()),
                                        ctypes.c_void_p(d_v.data_ptr()), None, sh)
        if st != 0:
            raise RuntimeError(f"cc_verify_batch_device: {lib.cc_status_str(st).decode()}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    ctx.timing(True)
    phase = np.zeros(3)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        phase += np.array(ctx.last_timing())
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.timing(False)
    d_v_host = d_v.cpu().numpy()
    if args.steps + args.warmup == 0:
        step()
        torch.cuda.synchronize(dev)
        d_v_host = d_v.cpu().numpy()
    if not np.array_equal(d_v_host, batch["expect"]):
        raise SystemExit("verdicts disagree with construction — refusing to report a number")
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    total = n * world * args.steps
    value = total / elapsed

    if rank == 0:
        fm = fp_mults_per_credential(q)
        phase_ms = phase / args.steps
        names = ["prep", "miller", "fexp"]
        dom = int(np.argmax(phase_ms))
        mads = fm[names[dom]] * MADS_PER_FPMUL * n
        achieved = mads / (phase_ms[dom] * 1e-3)
        total_mads = sum(fm.values()) * MADS_PER_FPMUL * n
        out = {
            "metric": "verified credentials/sec (msg_count=6); pairings/sec = 2x",
            "value": round(value, 1),
            "unit": "credentials/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (Fp 12x32-bit Montgomery limbs, integer-only)",
            "data": "synthetic (seeded; sigma = k*G2, k*(x+sum y m)*G2 built on the GPU; 1/16 corrupted)",
            "config": {"workload": "config2: batch of 65,536 Signature::verify per GPU, msg_count=6, "
                                   "shared aggregated verkey, SigG2 (reference default)",
                       "credentials_per_gpu": n, "msg_count": q, "parallelism": f"shard-by-credential x{world}"},
            "pairings_per_s": round(2 * value, 1),
            "phase_ms": {k: round(float(v), 3) for k, v in zip(names, phase_ms)},
            "roofline": {"bound": "valu-int", "kernel": names[dom], "achieved": round(achieved / 1e12, 3),
                         "peak": PEAK_MAD_PER_S / 1e12, "unit": "Tmad/s (v_mad_u64_u32)",
                         "frac": round(achieved / PEAK_MAD_PER_S, 4),
                         "traffic": pmc_traffic("k_" + names[dom]), "traffic_unit": "bytes per launch (PMC, "
                         "profiles/r01_final/pmc_summary.json: register-spill/call-frame scratch, not algorithmic)",
                         "algorithmic_mads_per_credential": round(fm[names[dom]] * MADS_PER_FPMUL),
                         "whole_step_frac": round(total_mads / (ms_per_step * 1e-3) / PEAK_MAD_PER_S, 4),
                         "hbm_view_GBs": round(n * (2 * 192 + q * 48 + 1) / (ms_per_step * 1e-3) / 1e9, 3),
                         "hbm_peak_GBs": HBM_PEAK_GBS},
            "setup": {"verkey_tables_ms": round(vk_ms, 1), "synthetic_data_s": round(setup_s, 2)},
        }
        if not args.no_cpu_baseline and world == 1:
            thr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 8, 16)
            thr = max(1, min(thr, 16))
            out["cpu_baseline"] = cpu_baseline(batch, q, thr)
            out["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
