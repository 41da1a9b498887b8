#!/usr/bin/env python3
"""bench.py — batched Coconut Signature::verify throughput on MI355X (BASELINE.json `metric`).

Default workload (BASELINE.json configs[1]): a batch of 65,536 independent
msg_count = 6 credential verifies per GPU against one shared aggregated verkey, reference default
group assignment (SigG2: sigma in G2, verkey in G1).  1/16 of the credentials are corrupted
(sigma_2 + G), so the kernels see the reject path too.  A "step" is one pass of the hot path over the
whole batch — decode + verkey MSM -> 2-pair Miller loop -> final exponentiation -> verdicts — with
the serialized inputs already resident in HBM (cc_verify_batch_device).

Other modes (one JSON line each; the headline is the default):
  --mode verify-g1   config 2 in the literal "G2 MSM" layout (SigG1: sigma in G1, verkey in G2)
  --mode verify-pervk  config 2's size with a distinct verkey per credential (per-call Signature::verify)
  --mode rlc         config 3: q = 16, 131,072 credentials per GPU, RLC batch mode, RCCL all-gather
  --mode aggregate   config 4: Signature::aggregate + Verkey::aggregate, t = 67 of n = 100, 10k creds
  --mode pok         config 5: PoKOfSignatureProof::verify, q = 32, revealed {3,5,7,11,13,17,19,23}

Synthetic data: group elements are k*G for known scalars k, built by the product's own GPU
fixed-base multiplication (cc_fixed_base_mul), never by the oracle.

Multi-GPU: `--gpus N` without a torch.distributed environment relaunches itself under
torch.distributed.run (before any GPU call) with one process per GPU; each rank owns its own batch
(weak scaling, no data-path collective except the RLC all-gather); value = all credentials /
max-over-ranks time.

cpu_baseline: the C restatement in oracle/ (test infrastructure, kind "port") timed on this host on a
bounded sample of the same inputs (rank 0, N = 1 only): the threads this box grants (its CPU share)
and one thread, with nproc and the CPU model.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "coconut-rust_amd"))

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
MADS_PER_M = 288   # one Montgomery multiplication: 12x12 a*b + 12x12 m*p 32x32->64 products
# Peak v_mad_u64_u32 issue rate: the highest sustained rate tools/ubench_int.hip has measured on
# MI355X (profiles/r02_ubench_int.jsonl; plain-C chains at 8 waves/SIMD).
UBENCH = os.path.join(ROOT, "profiles", "r02_ubench_int.jsonl")
HBM_PEAK_GBS = 8000.0
OPCOUNT = os.path.join(ROOT, "tests", "fixtures", "opcount.json")
# per-mode rocprofv3 evidence of the current build (tools/gpu_modes_prof.sh): kernel-trace stats and the
# PMC passes of one bench step, summarised per kernel by tools/pmc_summary.py
PROFILE_DIR = os.path.join(ROOT, "profiles", "r06", "modes")


def peak_mad_per_s():
    best = 3.132e13  # profiles/r01_ubench_int.jsonl, one chain at 8 waves/SIMD
    try:
        with open(UBENCH) as f:
            for line in f:
                d = json.loads(line)
                if d.get("instr", "").startswith("v_mad_u64_u32"):
                    best = max(best, d["lane_ops_per_s"])
    except OSError:
        pass
    return best


# Verkey-table window width each bench mode opts into (cc_set_table_bits).  The library's own default
# stays within 4 GiB of HBM a context (18 bits at q = 6, 16 at q = 16); the bench asks for the widths
# the round-3 numbers were measured with, and names the width and the GiB in its config.
BENCH_VK_BITS = {"verify": 22, "verify-g1": 22, "rlc": 22, "pok": 20, "pok-g1": 20}


def vk_bits_for(args):
    return args.vk_bits if args.vk_bits is not None else BENCH_VK_BITS.get(args.mode, 0)


def table_config(ctx, q):
    """The verkey tables a context holds: window bits, GiB of HBM (q + 2 bases, fixed.h layout) and
    whether the width was the bench's explicit choice or the library default."""
    bits = ctx.table_bits()[0]
    entry = 96 if int(ctx.mode) == 0 else 192  # affine OtherGroup entry: G1 (SigG2) / G2 (SigG1)
    gib = (q + 2) * ((256 + bits - 1) // bits) * ((1 << bits) - 1) * entry / 2**30 if bits else 0.0
    return {"verkey_table_bits": bits, "verkey_table_GiB": round(gib, 2)}


def lib_info():
    import coconut
    return {"library": coconut.version(), "src_hash": coconut.source_hash()}


def opcounts(key):
    with open(OPCOUNT) as f:
        return json.load(f)["configs"][key]["M_per_credential"]


def pmc(kernel_key, mode=None):
    """Per-launch PMC figures of the same build (profiles/r06/modes/<mode>/pmc_summary.json; separate
    rocprofv3 --pmc passes, tools/pmc_summary.py; none if that mode has no committed summary): HBM bytes =
    2 x FETCH_SIZE (gfx950 counts half of wide reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, and VALU
    wave-instructions per CU per clock."""
    d = None
    for path in [os.path.join(PROFILE_DIR, mode, "pmc_summary.json")] if mode else []:
        try:
            with open(path) as f:
                d = json.load(f)
            break
        except (OSError, ValueError):
            continue
    if d is None:
        return {}
    for name, c in d.items():
        if kernel_key in name:
            out = {}
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                out["traffic_bytes"] = round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            if "SQ_INSTS_VALU" in c and c.get("GRBM_GUI_ACTIVE"):
                out["valu_issue_per_cu_clk"] = round(c["SQ_INSTS_VALU"] / 256 / (c["GRBM_GUI_ACTIVE"] / 8), 3)
            return out
    return {}


def kernel_pmc_report(mode):
    """North_star's per-kernel rocprof report for one bench mode: every product kernel's average
    duration (rocprofv3 --kernel-trace --stats), HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE,
    MI355X_MICROARCH.md gfx950 correction), achieved HBM GB/s, VALU issue (wave-instructions per CU per
    clock; 1.0 = every SIMD issuing a wave64 VALU op every 4 clocks) and the fraction of wave-cycles
    waiting.  Read from profiles/r06/modes/<mode>/ (committed evidence of the same build)."""
    import csv
    d = os.path.join(PROFILE_DIR, mode)
    try:
        with open(os.path.join(d, "pmc_summary.json")) as f:
            pm = json.load(f)
        with open(os.path.join(d, "rocprof_kernel_stats.csv")) as f:
            st = {r["Name"]: r for r in csv.DictReader(f)}
    except (OSError, ValueError):
        return None
    out = {}
    for name, c in pm.items():
        if not any(k in name for k in ("k_", "cc::")) or "k_table" in name or "k_decode_points" in name \
                or "k_fixed_mul" in name or "k_subgroup<" in name:
            continue  # setup kernels (tables, synthetic data) are outside the timed step
        r = st.get(name)
        if not r:
            continue
        ms = float(r["AverageNs"]) / 1e6
        row = {"avg_ms": round(ms, 4), "calls": int(r["Calls"])}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            tb = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            row["hbm_bytes_per_launch"] = round(tb)
            row["hbm_GB_s"] = round(tb / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
            row["hbm_frac"] = round(tb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ms > 0 else None
        if "SQ_INSTS_VALU" in c and c.get("GRBM_GUI_ACTIVE"):
            row["valu_issue_per_cu_clk"] = round(c["SQ_INSTS_VALU"] / 256 / (c["GRBM_GUI_ACTIVE"] / 8), 3)
        if c.get("SQ_WAVE_CYCLES"):
            row["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
        short = name.split("(")[0].replace("void ", "")
        out[short] = row
    return {"source": f"profiles/r06/modes/{mode}/ (rocprofv3 kernel stats + PMC passes)", "kernels": out}


def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return model, os.cpu_count() or 1, aff


def host_threads():
    """Threads this box grants: OMP_NUM_THREADS (16 per GPU on the pool), else the affinity set."""
    _, _, aff = cpu_info()
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    except ValueError:
        n = 0
    return max(1, min(n or aff, aff))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


BACKEND = os.environ.get("COCONUT_BENCH_BACKEND", "nccl")  # bench.py --backend


def _dist_setup():
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        if BACKEND == "nccl":  # RCCL over xGMI: one GPU per rank
            torch.cuda.set_device(local)
        else:
            # gloo: a rehearsal of the multi-rank path (barriers, max over ranks, RLC all-gather through host
            # memory); with fewer GPUs than ranks the ranks share them (device_count touches no GPU here)
            local = local % max(1, torch.cuda.device_count())
        dist.init_process_group(BACKEND)
    return world, rank, local, dist


def _max_over_ranks(x, dist, dev):
    if not dist:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=dev if BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def default_tables_leg(args, ctx, rebind, step, check, n, dev, dist, unit="credentials/s", table_kind="verkey",
                       run_k=None):
    """The rate a drop-in caller gets with the library's DEFAULT table widths (cc_set_table_bits(0, 0):
    verkey tables <= 4 GiB, issuer tables <= 16 GiB), measured in the same run after the headline's
    timed region: rebind the tables at the default width, one warmup step, then min(args.steps, 10) timed
    steps bracketed like the headline's (synchronize + barrier, max over ranks); the outputs are checked
    again (check() must return True).  run_k(k), when given, runs k steps itself (the RLC's pipelined
    loop) in place of k calls of step()."""
    import torch
    world = dist.get_world_size() if dist else 1
    ctx.set_table_bits(0, 0)
    t = time.perf_counter()
    rebind()
    build_ms = (time.perf_counter() - t) * 1e3
    k = max(1, min(args.steps, 10))
    if run_k is None:
        def run_k(kk):
            for _ in range(kk):
                step()
    run_k(1)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run_k(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dist, dev)
    if not check():
        raise SystemExit("default-table outputs disagree with construction — refusing to report a number")
    bits = ctx.table_bits()
    return {"value": round(n * world * k / el, 1), "unit": unit, "steps": k, "ms_per_step": round(el / k * 1e3, 3),
            "table_bits": bits[0] if table_kind == "verkey" else bits[1], "tables": table_kind,
            "table_build_ms": round(build_ms, 1),
            "note": "library default widths (cc_set_table_bits(0, 0)): what a drop-in caller gets without opting in"}


def latency_of(ctx, launch, expect, dev, ns=(1, 256), reps=5, what="credentials"):
    """Single-call latency of a device entry point (what a drop-in caller waiting on ONE call sees):
    launch(nn, d_verdicts, stream_handle) on the first nn items of the bench batch, inputs resident, one
    call + synchronize, median of `reps` after a warmup; per-phase times from cc_last_timing."""
    import numpy as np
    import torch
    sh = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out = {}
    for nn in ns:
        d_v = torch.zeros(nn, dtype=torch.uint8, device=dev)
        launch(nn, d_v, sh)
        torch.cuda.synchronize(dev)
        ms = []
        for _ in range(reps):
            t0 = time.perf_counter()
            launch(nn, d_v, sh)
            torch.cuda.synchronize(dev)
            ms.append((time.perf_counter() - t0) * 1e3)
        if not np.array_equal(d_v.cpu().numpy(), expect[:nn]):
            raise SystemExit("latency-leg verdicts disagree with construction — refusing to report a number")
        ctx.timing(True)
        launch(nn, d_v, sh)
        ph = ctx.last_timing()
        ctx.timing(False)
        out[str(nn)] = {"ms": round(float(np.median(ms)), 3), "phase_ms": {"prep": round(ph[0], 3),
                        "miller": round(ph[1], 3), "fexp": round(ph[2], 3)}}
    return {what: out, "note": "one device call + synchronize on resident inputs, median of %d; batches of "
                               "<= 4,096 run the one-wave-per-pair Miller loop (<= 2,048: one-wave fexp and verify prep; "
                               "PoK / per-verkey preps: <= 1,024)" % reps}


def latency_leg(ctx, d_s1, d_s2, d_m, q, expect, dev, ns=(1, 256), reps=5):
    """latency_of for cc_verify_batch_device (shared verkey): one Signature::verify, a batch of 256."""
    import coconut
    lib = coconut._lib.lib

    def launch(nn, d_v, sh):
        st = lib.cc_verify_batch_device(ctx.h, nn, q, ctypes.c_void_p(d_s1.data_ptr()), ctypes.c_void_p(d_s2.data_ptr()),
                                        ctypes.c_void_p(d_m.data_ptr()), ctypes.c_void_p(d_v.data_ptr()), None, sh)
        if st != 0:
            raise RuntimeError(f"cc_verify_batch_device: {lib.cc_status_str(st).decode()}")
    return latency_of(ctx, launch, expect, dev, ns, reps)


# ---------------------------------------------------------------- synthetic data (on the GPU)
def rand_fr(rng):
    return int.from_bytes(rng.bytes(32), "big") % R_ORDER


CORRUPT_KINDS = ("sigma2+G", "msg+1", "swapped", "sigma1=O", "sigma2=O", "wrong vk")


def make_verify_batch(ctx, mode, n, q, seed, bad_every=16, key_seed=None):
    """one shared verkey AGGREGATED 3-of-5 (Shamir-shared issuer keys, the
    product's Verkey::aggregate on the GPU, checked against x g~ before use); per-credential messages
    uniform; sigma_1 = k G, sigma_2 = k (x + sum y_j m_j) G.  Every bad_every-th credential is corrupted,
    the kinds split evenly over CORRUPT_KINDS: sigma_2 + G, one m_j + 1, sigma_1 <-> sigma_2 swapped,
    sigma_1 = O, sigma_2 = O, signed under another verkey.  mode 0 = SigG2 (sigma in G2), 1 = SigG1.
    bad_every = 0: all valid.  key_seed: the issuer keys and g~ drawn from their own seed (the ranks of an
    RLC job verify under ONE verkey: every rank's finish pairs the gathered window sums with its own g~),
    the credentials from `seed`."""
    import numpy as np
    import coconut
    rng = np.random.default_rng(seed if key_seed is None else key_seed)
    og, sg = (1, 2) if mode == 0 else (2, 1)
    gen = {1: coconut.G1_GENERATOR, 2: coconut.G2_GENERATOR}
    ob, sb = (97, 192) if mode == 0 else (192, 97)
    # 3-of-5 Shamir keygen (reference keygen.rs:48-72 trusted_party_SSS_keygen): degree-2 polynomials
    fx = [rand_fr(rng) for _ in range(3)]
    fy = [[rand_fr(rng) for _ in range(3)] for _ in range(q)]
    ev = lambda c, i: (c[0] + c[1] * i + c[2] * i * i) % R_ORDER  # noqa: E731
    x, y = fx[0], [c[0] for c in fy]
    gk = rand_fr(rng) or 1
    ids = [1, 2, 3, 4, 5]
    sc = b"".join(v.to_bytes(48, "big") for i in ids for v in [ev(fx, i) * gk % R_ORDER] +
                  [ev(c, i) * gk % R_ORDER for c in fy])
    keys = coconut.fixed_base_mul(ctx, og, gen[og], sc)
    g_tilde = coconut.fixed_base_mul(ctx, og, gen[og], gk.to_bytes(48, "big"))
    use = [0, 2, 4]  # issuers 1, 3, 5
    kX = b"".join(keys[(u * (q + 1)) * ob:(u * (q + 1) + 1) * ob] for u in use)
    kY = b"".join(keys[(u * (q + 1) + 1) * ob:(u * (q + 1) + 1 + q) * ob] for u in use)
    X, Y = coconut.verkey_aggregate_batch(ctx, 1, 3, 3, q, [[ids[u] for u in use]], kX, kY)
    want = coconut.fixed_base_mul(ctx, og, gen[og], b"".join(v.to_bytes(48, "big") for v in
                                                              [x * gk % R_ORDER] + [v * gk % R_ORDER for v in y]))
    if X + Y != want:
        raise SystemExit("aggregated verkey differs from g~ * master secret — refusing to build the batch")
    if key_seed is not None:
        rng = np.random.default_rng(seed)
    m = [[rand_fr(rng) for _ in range(q)] for _ in range(n)]
    ks = [rand_fr(rng) or 1 for _ in range(n)]
    x_other = (x + 0x5EED) % R_ORDER
    e1, e2 = [], []
    expect = np.ones(n, dtype=np.uint8)
    kind = [None] * n
    for i in range(n):
        e = ks[i] * ((x + sum(yj * mj for yj, mj in zip(y, m[i]))) % R_ORDER) % R_ORDER
        k1 = ks[i]
        if bad_every and i % bad_every == bad_every - 1:
            kd = CORRUPT_KINDS[(i // bad_every) % len(CORRUPT_KINDS)]
            kind[i] = kd
            expect[i] = 0
            if kd == "sigma2+G":
                e = (e + 1) % R_ORDER
            elif kd == "msg+1":
                m[i][0] = (m[i][0] + 1) % R_ORDER
            elif kd == "swapped":
                k1, e = e, k1
            elif kd == "sigma1=O":
                k1 = 0
            elif kd == "sigma2=O":
                e = 0
            else:  # wrong vk
                e = ks[i] * ((x_other + sum(yj * mj for yj, mj in zip(y, m[i]))) % R_ORDER) % R_ORDER
        e1.append(k1.to_bytes(48, "big"))
        e2.append(e.to_bytes(48, "big"))
    s1 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(e1))
    s2 = coconut.fixed_base_mul(ctx, sg, gen[sg], b"".join(e2))
    msgs = b"".join(v.to_bytes(48, "big") for row in m for v in row)
    return dict(X=X, Y=Y, g_tilde=g_tilde, s1=s1, s2=s2, msgs=msgs, expect=expect, mode=mode, q=q, n=n, kind=kind)


def to_dev(b, dev):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)


# ---------------------------------------------------------------- CPU baseline (oracle/c, test infra)
def _oracle():
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle", "c")])
    return ctypes.CDLL(so)


def cpu_verify_rate(batch, threads, target_s):
    """oc_verify_batch (64-bit Montgomery, AMCL-class algorithm) on `threads` threads over a sample
    of the same credentials sized to ~target_s of wall time; returns (creds/s, sample, seconds)."""
    import numpy as np
    oc = _oracle()
    mode, q = batch["mode"], batch["q"]
    sb = 192 if mode == 0 else 97
    ob = 97 if mode == 0 else 192
    pervk = 1 if batch.get("per_vk") else 0  # one verkey per credential (X: n x ob, Y: n x q x ob)
    vk = lambda k: (batch["X"][:k * ob], batch["Y"][:k * q * ob]) if pervk else (batch["X"], batch["Y"])  # noqa: E731
    k0 = max(2, threads * 2)
    ver = ctypes.create_string_buffer(k0)
    t = time.perf_counter()
    oc.oc_verify_batch(mode, ctypes.c_size_t(k0), ctypes.c_size_t(q), batch["s1"][:k0 * sb], batch["s2"][:k0 * sb],
                       batch["msgs"][:k0 * q * 48], *vk(k0), pervk, batch["g_tilde"], ver, None, threads)
    per = (time.perf_counter() - t) / k0
    k = int(min(batch["n"], max(threads * 4, target_s / max(per, 1e-6))))
    k = max(threads, (k // threads) * threads)
    ver = ctypes.create_string_buffer(k)
    t = time.perf_counter()
    oc.oc_verify_batch(mode, ctypes.c_size_t(k), ctypes.c_size_t(q), batch["s1"][:k * sb], batch["s2"][:k * sb],
                       batch["msgs"][:k * q * 48], *vk(k), pervk, batch["g_tilde"], ver, None, threads)
    dt = time.perf_counter() - t
    agree = bool(np.array_equal(np.frombuffer(ver.raw, np.uint8), batch["expect"][:k]))
    return k / dt, k, dt, agree


def cpu_baseline_verify(batch, value, what="shared vk"):
    """The CPU path timed on this box's host cores in the same run.  The pool grants one GPU's job a
    share of the host (OMP_NUM_THREADS = 16 CPUs per GPU; it kills jobs that run wider), so the timed
    figure is that share; the whole host (nproc CPUs) is single_thread x nproc scaled by the measured
    per-thread efficiency of the share — an extrapolation, labelled as one.  gpu_over_cpu compares with
    that whole-host figure (the conservative ratio); gpu_over_cpu_share with the timed share."""
    model, nproc, aff = cpu_info()
    thr = host_threads()
    v_mt, k_mt, dt_mt, ok_mt = cpu_verify_rate(batch, thr, target_s=2.0)
    v_1, k_1, dt_1, ok_1 = cpu_verify_rate(batch, 1, target_s=3.0)
    eff = min(1.0, v_mt / (thr * v_1)) if thr > 1 else 1.0
    host = v_1 * nproc * eff
    layout = "SigG2" if batch["mode"] == 0 else "SigG1"
    return {
        "value": round(v_mt, 1), "unit": "credentials/s", "cores": thr, "kind": "port",
        "sample": f"{k_mt} credentials of the timed batch (q={batch['q']}, {what}, {layout}) on {thr} threads "
                  f"in {dt_mt:.2f} s, plus {k_1} on 1 thread in {dt_1:.2f} s; oracle/c bls_oracle.c oc_verify_batch "
                  f"(per-credential verify, test infrastructure); verdicts agree with construction: {ok_mt and ok_1}",
        "single_thread": round(v_1, 1),
        "per_thread_efficiency": round(eff, 3),
        "nproc": nproc, "affinity_cpus": aff, "cpu_model": model,
        "threads_note": f"timed on the {thr}-CPU share this box grants per GPU (OMP_NUM_THREADS); the pool's rules "
                        f"cap a one-GPU job at that share (worker pools sized to it; nproc = {nproc} counts the whole "
                        "machine), so all cores are NOT timed: the whole host is extrapolated as single_thread x nproc "
                        "x per_thread_efficiency (all_cores_extrapolated), and gpu_over_cpu quotes that conservative "
                        "ratio",
        "all_cores_extrapolated": round(host, 1),
        "gpu_over_cpu": round(value / host, 2),
        "gpu_over_cpu_share": round(value / v_mt, 1),
    }


def cpu_pool_rate(fn, n_avail, threads, target_s):
    """Rate of fn(i) (one oracle call on item i; ctypes releases the GIL, so the calls run in parallel)
    over a sample of the first items sized to ~target_s of wall time on `threads` threads.  Returns
    (items/s, items, seconds, results)."""
    from concurrent.futures import ThreadPoolExecutor
    t = time.perf_counter()
    fn(0)
    per = max(time.perf_counter() - t, 1e-6)
    k = int(min(n_avail, max(threads * 2, target_s * threads / per)))
    k = max(min(threads, n_avail), (k // threads) * threads) if k >= threads else k
    with ThreadPoolExecutor(max_workers=threads) as ex:
        t = time.perf_counter()
        res = list(ex.map(fn, range(k)))
        dt = time.perf_counter() - t
    return k / dt, k, dt, res


def cpu_report(value, unit, what, mt, one, thr, agree):
    """cpu_baseline object from a `thr`-thread sample and a one-thread sample (cpu_pool_rate results):
    the whole host is extrapolated as single thread x nproc x the share's per-thread efficiency, as in
    cpu_baseline_verify."""
    model, nproc, aff = cpu_info()
    v_mt, k_mt, dt_mt = mt[:3]
    v_1, k_1, dt_1 = one[:3]
    eff = min(1.0, v_mt / (thr * v_1)) if thr > 1 else 1.0
    host = v_1 * nproc * eff
    return {
        "value": round(v_mt, 2), "unit": unit, "cores": thr, "kind": "port",
        "sample": f"{k_mt} items of the timed batch on {thr} threads in {dt_mt:.2f} s, plus {k_1} on 1 thread in "
                  f"{dt_1:.2f} s; {what} (oracle/c, test infrastructure); outputs agree with construction: {agree}",
        "single_thread": round(v_1, 2), "per_thread_efficiency": round(eff, 3),
        "nproc": nproc, "affinity_cpus": aff, "cpu_model": model,
        "all_cores_extrapolated": round(host, 1),
        "gpu_over_cpu": round(value / host, 2), "gpu_over_cpu_share": round(value / v_mt, 1),
    }


# ---------------------------------------------------------------- modes
def kernel_table(phase_ms, n, counts, in_bytes_per_cred, peak, prep_kernel="k_prep_sigg2_pair", mode=None):
    """Per-kernel roofline: algorithmic M (tests/fixtures/opcount.json) x 288 mads x n / kernel time.
    PMC columns only where the committed summary holds that exact kernel (prep_kernel names it)."""
    out = {}
    names = ["prep", "miller", "fexp"]
    for k, ms in zip(names, phase_ms):
        mads = counts[k] * MADS_PER_M * n
        ach = mads / (ms * 1e-3) if ms > 0 else 0.0
        row = {"ms": round(float(ms), 3), "mads_per_launch": round(mads), "achieved_Tmad_s": round(ach / 1e12, 3),
               "frac": round(ach / peak, 4)}
        if k == "prep":
            row["input_GB_s"] = round(n * in_bytes_per_cred / (ms * 1e-3) / 1e9, 2)
        # the batch kernels by exact name stem: the small-batch paths' k_miller_wide / k_fexp1 (the latency
        # legs) appear in the same profiles
        mk = "lz::k_miller<1, false>" if mode and mode.endswith("g1") else "lz::k_miller<2, false>"
        row.update(pmc({"prep": prep_kernel + "(", "miller": mk, "fexp": "lz::k_fexp_q("}[k], mode))
        out[k] = row
    return out


def bench_verify(args, mode, sub=None):
    """sub: None for a mode's own line; else (world, rank, local, dist) of the running headline, and this
    call is its same-run SigG1 leg: the same workload, batches in flight and verdict check, returned as a
    compact dict (no PCIe / default-table / latency / CPU legs) for the line's `sigg1` object."""
    import numpy as np
    import torch
    import coconut
    world, rank, local, dist = sub if sub else _dist_setup()
    dev = torch.device("cuda", local)
    n, q = args.n or 65536, 6
    ctx = coconut.Context(local, coconut.GroupMode(mode))
    t_setup = time.perf_counter()
    batch = make_verify_batch(ctx, mode, n, q, seed=1000 + rank + 100 * mode)
    ctx.set_params(batch["g_tilde"])
    t_vk = time.perf_counter()
    ctx.set_table_bits(args.vk_bits if args.vk_bits is not None else BENCH_VK_BITS["verify" if mode == 0 else "verify-g1"], 0)
    ctx.set_verkey(batch["X"], batch["Y"])
    vk_ms = (time.perf_counter() - t_vk) * 1e3
    # --inflight K: K batches in flight on ONE context (cc_set_concurrency: K workspace slots, one set of
    # verkey tables) and K streams, steps issued round-robin, so one batch's kernel tails overlap the
    # next batch's kernels
    K = max(1, args.inflight)
    KK = [K]  # slots the steps rotate over (the per-kernel pass below uses one)
    ctx.set_concurrency(K)
    setup_s = time.perf_counter() - t_setup
    d_s1, d_s2, d_m = to_dev(batch["s1"], dev), to_dev(batch["s2"], dev), to_dev(batch["msgs"], dev)
    d_vs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(K)]
    d_v = d_vs[0]
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    for s_ in streams:
        s_.wait_stream(torch.cuda.current_stream(dev))
    shs = [ctypes.c_void_p(s_.cuda_stream) for s_ in streams]
    sh = shs[0]
    lib = coconut._lib.lib
    rr = [0]

    def step():
        k = rr[0] % KK[0]
        rr[0] += 1
        st = lib.cc_verify_batch_device(ctx.h, n, q, ctypes.c_void_p(d_s1.data_ptr()),
                                        ctypes.c_void_p(d_s2.data_ptr()), ctypes.c_void_p(d_m.data_ptr()),
                                        ctypes.c_void_p(d_vs[k].data_ptr()), None, shs[k])
        if st != 0:
            raise RuntimeError(f"cc_verify_batch_device: {lib.cc_status_str(st).decode()}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # phase timing (events + a host wait per call) only with one batch in flight: it would serialize them
    timed_phases = K == 1
    if timed_phases:
        ctx.timing(True)
    phase = np.zeros(3)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if timed_phases:
            phase += np.array(ctx.last_timing())
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.timing(False)
    if args.steps + args.warmup == 0:
        step()
        torch.cuda.synchronize(dev)
    for k in range(K):
        if rr[0] > k and not np.array_equal(d_vs[k].cpu().numpy(), batch["expect"]):
            raise SystemExit("verdicts disagree with construction — refusing to report a number")
    ctx.set_concurrency(1)
    KK[0] = 1
    rr[0] = 0
    if not timed_phases:  # the per-kernel table from a separate single-batch pass
        ctx.timing(True)
        for _ in range(min(args.steps, 5)):
            step()
            phase += np.array(ctx.last_timing())
        ctx.timing(False)
        phase *= args.steps / max(min(args.steps, 5), 1)
    elapsed = _max_over_ranks(elapsed, dist, dev)
    value = n * world * args.steps / elapsed
    opt_in = table_config(ctx, q)
    if sub:
        kt = kernel_table(phase / max(args.steps, 1), n, opcounts("verify_sigg1_q6_shared_vk"), 97 * 2 + q * 48,
                          peak_mad_per_s(), "k_prep_sigg1_pair", "verify-g1")
        ctx.close()
        return {"layout": "SigG1 (BASELINE config 2 wording: 'G2 MSM + 2-pairing check': verkey MSM in G2, "
                          "sigma in G1)",
                "value": round(value, 1), "unit": "credentials/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                "steps": args.steps, "warmup": args.warmup, "batches_in_flight": K, "credentials_per_gpu": n,
                "verdicts_checked": "against construction (1/16 corrupted), every slot", **opt_in,
                "kernels": kt, "rocprof_kernels": kernel_pmc_report("verify-g1")}
    # PCIe-inclusive rate: the host-buffer entry point (H2D of the serialized batch + D2H of verdicts);
    # --no-pcie skips it (profiling runs: then every launch of the trace is a warmup or a timed step)
    pcie_rate = None
    if not args.no_pcie:
        v = coconut.verify_batch(ctx, n, q, batch["s1"], batch["s2"], batch["msgs"])  # sizes the host path's buffers
        assert np.array_equal(v, batch["expect"])
        reps = 3
        t = time.perf_counter()
        for _ in range(reps):
            v = coconut.verify_batch(ctx, n, q, batch["s1"], batch["s2"], batch["msgs"])
        pcie_rate = n * reps / (time.perf_counter() - t)
        assert np.array_equal(v, batch["expect"])
    # the library-default tables at the headline's batches in flight
    def rebind_dflt():
        ctx.set_verkey(batch["X"], batch["Y"])
        ctx.set_concurrency(K)
        KK[0] = K
        rr[0] = 0

    def check_dflt():
        ok = all(np.array_equal(d_vs[k].cpu().numpy(), batch["expect"]) for k in range(min(K, rr[0])))
        ctx.set_concurrency(1)
        return ok
    dflt = default_tables_leg(args, ctx, rebind_dflt, step, check_dflt, n, dev, dist)
    dflt["batches_in_flight"] = K
    dflt.update(table_config(ctx, q))
    latency = latency_leg(ctx, d_s1, d_s2, d_m, q, batch["expect"], dev)
    sigg1 = None
    if mode == 0 and not args.no_sigg1:  # BASELINE config 2's own wording, same run, same K
        ctx.close()
        ctx = None
        del d_s1, d_s2, d_m, d_vs, d_v
        torch.cuda.empty_cache()
        sigg1 = bench_verify(args, 1, sub=(world, rank, local, dist))
    if rank == 0:
        key = "verify_sigg2_q6_shared_vk" if mode == 0 else "verify_sigg1_q6_shared_vk"
        counts = opcounts(key)
        peak = peak_mad_per_s()
        phase_ms = phase / max(args.steps, 1)
        sb = 192 if mode == 0 else 97
        mname = "verify" if mode == 0 else "verify-g1"
        kt = kernel_table(phase_ms, n, counts, 2 * sb + q * 48, peak,
                          "k_prep_sigg2_pair" if mode == 0 else "k_prep_sigg1_pair", mname)
        dom = max(kt, key=lambda k: kt[k]["ms"])
        ms_per_step = elapsed / args.steps * 1e3
        total_mads = sum(counts.values()) * MADS_PER_M * n
        layout = "SigG2 (reference default: sigma in G2, verkey MSM in G1)" if mode == 0 else \
            "SigG1 (BASELINE config 2 wording: verkey MSM in G2, sigma in G1)"
        out = {
            "metric": "verified credentials/sec (msg_count=6); pairings/sec = 2x" + ("" if mode == 0 else " [SigG1]"),
            "value": round(value, 1), "unit": "credentials/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "int32/u32 (pairing kernels: 14 signed 28-bit-radix limbs, lazy; elsewhere 12x32-bit Montgomery; integer-only)",
            "data": "synthetic (seeded, SURVEY.md §8d config 2: verkey aggregated 3-of-5 on the GPU; sigma = k*G, "
                    "k*(x+sum y m)*G built on the GPU; 1/16 corrupted, split evenly over " + ", ".join(CORRUPT_KINDS) + ")",
            "config": {"workload": f"config2: batch of {n:,} Signature::verify per GPU, msg_count=6, shared "
                                   f"aggregated verkey, {layout}",
                       "credentials_per_gpu": n, "msg_count": q, "parallelism": f"shard-by-credential x{world}",
                       "batches_in_flight": max(1, args.inflight),
                       **opt_in, "verkey_tables": "opt-in width (bench); library default <= 4 GiB"},
            **lib_info(),
            "pairings_per_s": round(2 * value, 1),
            "default_tables": dflt,
            "latency": latency,
            "roofline": {"bound": "valu-int", "kernel": dom, "achieved": kt[dom]["achieved_Tmad_s"],
                         "peak": round(peak / 1e12, 3), "unit": "Tmad/s (v_mad_u64_u32, 32x32->64)",
                         "frac": kt[dom]["frac"], "traffic": kt[dom].get("traffic_bytes"),
                         "traffic_unit": "HBM-side bytes per launch (PMC, 2 x FETCH_SIZE + WRITE_SIZE)",
                         "algorithmic_mads_per_credential": round(counts[dom] * MADS_PER_M),
                         "opcount_fixture": "tests/fixtures/opcount.json (tools/opcount.py)",
                         "whole_step_frac": round(total_mads / (ms_per_step * 1e-3) / peak, 4),
                         "hbm_view_GBs": round(n * (2 * sb + q * 48 + 1) / (ms_per_step * 1e-3) / 1e9, 3),
                         "hbm_peak_GBs": HBM_PEAK_GBS},
            "kernels": kt,
            "rocprof_kernels": kernel_pmc_report(mname),
            "pcie_inclusive": {"value": round(pcie_rate, 1) if pcie_rate else None, "unit": "credentials/s",
                               "note": "cc_verify_batch with host buffers, one call at a time (after one "
                                       "untimed call that sizes its buffers): H2D of the serialized batch + D2H "
                                       "of verdicts included (not `value`)"},
            "setup": {"verkey_tables_ms": round(vk_ms, 1), "verkey_table_bits": opt_in["verkey_table_bits"],
                      "synthetic_data_s": round(setup_s, 2)},
        }
        if sigg1:
            out["sigg1"] = sigg1
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline_verify(batch, value)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if ctx is not None:
        ctx.close()


def bench_rlc(args):
    """BASELINE config 3: q = 16 credentials verified in RLC batch mode.  Each rank owns 131,072
    credentials (2^20 over 8 GPUs); a step = per-rank partial (delta-weighted Miller product of the
    slice) -> RCCL all-gather of the 3,716-byte partials -> one final exponentiation on every rank ->
    accept.  All credentials are valid, so the accept path is timed; the reject path (one corrupted
    credential -> every rank rejects -> per-credential fallback) is checked after the timed region."""
    import numpy as np
    import torch
    import coconut
    from coconut.dist import DeviceEngine, gather_partials
    world, rank, local, dist = _dist_setup()
    dev = torch.device("cuda", local)
    n, q = args.n or 131072, 16
    ctx = coconut.Context(local, coconut.GroupMode.SIG_G2)
    batch = make_verify_batch(ctx, 0, n, q, seed=3000 + rank, bad_every=0, key_seed=2999)
    ctx.set_params(batch["g_tilde"])
    ctx.set_table_bits(vk_bits_for(args), 0)
    ctx.set_verkey(batch["X"], batch["Y"])
    d_s1, d_s2, d_m = to_dev(batch["s1"], dev), to_dev(batch["s2"], dev), to_dev(batch["msgs"], dev)
    # --inflight K: K engines (own streams and partial buffers) take turns on ONE context whose
    # cc_set_concurrency(K) gives successive partials their own workspace slots, so batch i + 1's partial
    # can start while batch i's is still draining (its last waves) and batch i's finish runs
    K = max(1, args.rlc_inflight)
    engs = [DeviceEngine(ctx, n, q, d_s1, d_s2, d_m, base_index=rank * n) for _ in range(K)]
    eng = engs[0]

    # batches are pipelined: batch i's single final exponentiation (one wave, latency-bound) runs on the
    # engine's finish stream while batch i+1's partial runs (DeviceEngine.finish_async)
    def run(k_steps, phase=None, k_eng=1):
        ok = True
        cur = engs[0]
        part = cur.partial()
        if phase is not None:
            phase += np.array(ctx.last_timing())
        for s in range(k_steps):
            allp, k = gather_partials(part)
            decision = cur.finish_async(allp, k)
            if s + 1 < k_steps:
                cur = engs[(s + 1) % k_eng]
                part = cur.partial()
                if phase is not None:
                    phase += np.array(ctx.last_timing())
            ok &= decision()
        return ok

    # per-phase times come from a single-slot pass (the phase events of overlapping batches would overlap)
    phase = np.zeros(3)
    if args.steps:
        ctx.timing(True)
        assert run(min(args.steps, 5), phase)
        torch.cuda.synchronize(dev)
        ctx.timing(False)
        phase *= args.steps / min(args.steps, 5)
    ctx.set_concurrency(K)
    if args.warmup:
        assert run(args.warmup, k_eng=K)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ok = run(args.steps, k_eng=K)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_concurrency(1)
    if not ok:
        raise SystemExit("RLC rejected an all-valid batch — refusing to report a number")
    bad = d_s2.clone()
    if rank == 0:
        bad[:192] = d_s2[192:384]
    eng_bad = DeviceEngine(ctx, n, q, d_s1, bad, d_m, base_index=rank * n)
    pb, k = gather_partials(eng_bad.partial())
    if eng_bad.finish(pb, k):
        raise SystemExit("RLC accepted a corrupted batch — refusing to report a number")
    elapsed = _max_over_ranks(elapsed, dist, dev)
    value = n * world * args.steps / elapsed
    opt_in = table_config(ctx, q)
    # one NON-pipelined decision, as a single cc_verify_batch(..., rlc=1) call pays it: partial -> all-gather
    # -> finish -> accept on the host, nothing overlapped (the finish's one-wave kernels on the critical path)
    lat = []
    for _ in range(3 if args.steps else 0):
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        allp, k = gather_partials(eng.partial())
        if not eng.finish(allp, k):
            raise SystemExit("RLC rejected an all-valid batch — refusing to report a number")
        lat.append(time.perf_counter() - t1)
    single_ms = _max_over_ranks(min(lat), dist, dev) * 1e3 if lat else None

    ok_dflt = [True]

    def run_dflt(k_steps):
        ctx.set_concurrency(K)
        ok_dflt[0] &= run(k_steps, k_eng=K)
        ctx.set_concurrency(1)
    dflt = default_tables_leg(args, ctx, lambda: ctx.set_verkey(batch["X"], batch["Y"]), None,
                              lambda: ok_dflt[0], n, dev, dist, run_k=run_dflt)
    dflt.update(table_config(ctx, q))
    dflt["note"] += "; pipelined as the headline (finish of batch i under the partial of batch i + 1)"
    if rank == 0:
        phase_ms = phase / max(args.steps, 1)
        out = {
            "metric": "verified credentials/sec, RLC batch mode (msg_count=16)",
            "value": round(value, 1), "unit": "credentials/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32/u32 (pairing kernels: 14 signed 28-bit-radix limbs, lazy; elsewhere 12x32-bit Montgomery; integer-only)",
            "data": "synthetic (seeded; all valid, reject path checked after timing)",
            "config": {"workload": "config3: RLC batch verify, msg_count=16, shared verkey, SigG2",
                       "credentials_per_gpu": n, "msg_count": q,
                       "parallelism": f"shard-by-credential x{world} + RCCL all-gather of Fp12 partials",
                       "batches_in_flight": K,
                       **opt_in, "verkey_tables": "opt-in width (bench); library default <= 4 GiB"},
            **lib_info(),
            "single_call_ms": round(single_ms, 3) if single_ms else None,
            "single_call_note": "one non-pipelined RLC decision over the rank's credentials (partial -> "
                                "all-gather -> finish -> host accept; best of 3): the latency a single "
                                "cc_verify_batch(..., rlc=1) call pays",
            "default_tables": dflt,
            "phase_ms": {"prep": round(phase_ms[0], 3), "miller": round(phase_ms[1], 3),
                         "reduce": round(phase_ms[2], 3)},
            "us_per_credential": round(elapsed / args.steps / n * 1e6, 4),
        }
        counts = opcounts("rlc_sigg2_q16")
        peak = peak_mad_per_s()
        kt = {}
        for k, ms in zip(("prep", "miller", "reduce"), phase_ms):
            ach = counts[k] * MADS_PER_M * n / (ms * 1e-3) if ms > 0 else 0.0
            kt[k] = {"ms": round(float(ms), 3), "achieved_Tmad_s": round(ach / 1e12, 3), "frac": round(ach / peak, 4)}
        out["kernels"] = kt
        rk = kernel_pmc_report("rlc")
        out["rocprof_kernels"] = rk
        mk = next((v for k, v in (rk or {}).get("kernels", {}).items() if "k_miller4" in k), {})
        out["roofline"] = {"bound": "valu-int", "kernel": "miller (k_miller4: four credentials per shared-squaring loop)",
                           "achieved": kt["miller"]["achieved_Tmad_s"], "peak": round(peak / 1e12, 3),
                           "unit": "Tmad/s (v_mad_u64_u32, 32x32->64)", "frac": kt["miller"]["frac"],
                           "traffic": mk.get("hbm_bytes_per_launch"),
                           "traffic_unit": "HBM-side bytes per launch of the credentials' Miller kernel (PMC)",
                           "algorithmic_mads_per_credential": round(counts["miller"] * MADS_PER_M),
                           "opcount_fixture": "tests/fixtures/opcount.json rlc_sigg2_q16",
                           "note": "the batch's one final exponentiation (single element, latency-bound) and the "
                                   "all-gather are outside the three phases but inside ms_per_step"}
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline_verify(batch, value, "shared vk, per-credential verify")
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


def bench_stub(args):
    """The multi-rank skeleton without a GPU (tests/test_bench_cli.py): relaunch, rendezvous, barrier,
    timed loop of a CPU stub step, max over ranks, one JSON line from rank 0.  Not a measurement."""
    import numpy as np
    world, rank, local, dist = _dist_setup()
    a = np.arange(1 << 16, dtype=np.uint64)
    for _ in range(args.warmup):
        a = (a * 6364136223846793005 + 1) & 0xFFFFFFFF
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = (a * 6364136223846793005 + 1) & 0xFFFFFFFF
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dist, "cpu")
    if rank == 0:
        print(json.dumps({"metric": "stub (CPU skeleton check, not a measurement)", "value": None, "unit": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4), "backend": BACKEND,
                          "scaling": "weak"}), flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    global BACKEND
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None,
                    help="torch.distributed backend for --gpus N (default nccl = RCCL; gloo: CPU skeleton tests)")
    ap.add_argument("--steps", type=int, default=100)  # ~2.3 s timed at config 2: long enough to see from outside
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=0, help="credentials per GPU per step (0 = the config's size)")
    ap.add_argument("--iss-bits", type=int, default=None,
                    help="issuer table window width for the aggregate modes (cc_set_table_bits; 0 = the "
                         "library's <= 16 GiB choice; default: bench_modes.BENCH_ISS_BITS = 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) rate")
    ap.add_argument("--no-sigg1", action="store_true",
                    help="default verify line: skip its same-run SigG1 leg (the `sigg1` object)")
    ap.add_argument("--vk-bits", type=int, default=None,
                    help="verkey table window width (cc_set_table_bits; 0 = the library's <= 4 GiB default; "
                         "unset = the mode's opt-in width, BENCH_VK_BITS)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="verify modes: batches in flight on one context (cc_set_concurrency slots) and as many "
                         "streams, issued round-robin; 1 = each batch ordered after the previous one")
    ap.add_argument("--rlc-inflight", type=int, default=1,
                    help="RLC mode: engines (own streams, partial buffers) taking cc_set_concurrency slots in "
                         "turn; 1 = the pipelined single engine (measured the same as 2 and 3: "
                         "profiles/r05/modes2; with pinned seed staging again 5.68 / 5.68 M/s: profiles/r06/base)")
    ap.add_argument("--mode", choices=["verify", "verify-g1", "verify-pervk", "verify-pervk-g1", "rlc", "aggregate",
                                       "aggregate-g1", "pok", "pok-g1", "stub"], default="verify")
    # a relaunched rank takes the launching command's arguments from the environment (see below)
    relaunched = os.environ.get("COCONUT_BENCH_ARGV") if "WORLD_SIZE" in os.environ else None
    args = ap.parse_args(json.loads(relaunched) if relaunched else None)
    if args.backend:
        BACKEND = args.backend
        os.environ["COCONUT_BENCH_BACKEND"] = args.backend  # inherited by the relaunched ranks
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run BEFORE any GPU call (no exec from a
        # process that touched the GPU: this one has not), and exit with its status
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
        # the bench's own arguments travel in the environment: torch.distributed.run's parser reads the
        # words after the script too, and rejects an abbreviation of its own options (`--n`) there
        env = dict(os.environ, COCONUT_BENCH_ARGV=json.dumps(sys.argv[1:]))
        return subprocess.call(cmd, env=env)
    if args.mode == "stub":
        return bench_stub(args)
    if args.mode == "verify":
        return bench_verify(args, 0)
    if args.mode == "verify-g1":
        return bench_verify(args, 1)
    if args.mode == "rlc":
        return bench_rlc(args)
    if args.mode in ("verify-pervk", "verify-pervk-g1"):
        from bench_modes import bench_pervk
        return bench_pervk(args)
    if args.mode in ("aggregate", "aggregate-g1"):
        from bench_modes import bench_aggregate
        return bench_aggregate(args)
    from bench_modes import bench_pok
    return bench_pok(args)


if __name__ == "__main__":
    sys.exit(main() or 0)
