"""Single-call latency of the verify path against batch size (round 5): what a drop-in caller that
verifies ONE credential (the reference's `Signature::verify`, src/signature.rs:473-478) or a small batch
waits for, per phase (cc_last_timing: prep / Miller / final exponentiation), on the device path and
through the host-buffer entry point.  One JSON line per (mode, n).

    python tools/latency_probe.py [--modes 0,1] [--ns 1,2,16,256,4096,65536] [--reps 7]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coconut-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--ns", default="1,2,16,256,4096,65536")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--q", type=int, default=6)
    args = ap.parse_args()
    import numpy as np
    import torch
    import coconut
    import bench
    dev = torch.device("cuda", 0)
    lib = coconut._lib.lib
    for mode in [int(m) for m in args.modes.split(",")]:
        ctx = coconut.Context(0, coconut.GroupMode(mode))
        nmax = max(int(x) for x in args.ns.split(","))
        batch = bench.make_verify_batch(ctx, mode, nmax, args.q, seed=77 + mode, bad_every=0)
        ctx.set_params(batch["g_tilde"])
        ctx.set_verkey(batch["X"], batch["Y"])
        d_s1, d_s2, d_m = (bench.to_dev(batch[k], dev) for k in ("s1", "s2", "msgs"))
        for n in [int(x) for x in args.ns.split(",")]:
            d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
            st = torch.cuda.current_stream(dev)
            sh = ctypes.c_void_p(st.cuda_stream)

            def call():
                r = lib.cc_verify_batch_device(ctx.h, n, args.q, ctypes.c_void_p(d_s1.data_ptr()),
                                               ctypes.c_void_p(d_s2.data_ptr()), ctypes.c_void_p(d_m.data_ptr()),
                                               ctypes.c_void_p(d_v.data_ptr()), None, sh)
                if r != 0:
                    raise RuntimeError(lib.cc_status_str(r).decode())
            call()
            torch.cuda.synchronize(dev)
            wall, phases = [], []
            for _ in range(args.reps):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                call()
                torch.cuda.synchronize(dev)
                wall.append((time.perf_counter() - t0) * 1e3)
            ctx.timing(True)
            for _ in range(3):
                call()
                phases.append(ctx.last_timing())
            ctx.timing(False)
            torch.cuda.synchronize(dev)
            ok = bool(d_v.cpu().numpy().all())
            host_ms = None
            if n <= 256:
                sb = ctx.mode.sig_bytes
                s1, s2 = batch["s1"][:n * sb], batch["s2"][:n * sb]
                m = batch["msgs"][:n * args.q * 48]
                hs = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    v = coconut.signature.verify_batch(ctx, n, args.q, s1, s2, m)
                    hs.append((time.perf_counter() - t0) * 1e3)
                    ok = ok and bool(np.asarray(v).all())
                host_ms = round(float(np.median(hs)), 3)
            ph = np.median(np.array(phases), axis=0)
            print(json.dumps({"mode": "SigG2" if mode == 0 else "SigG1", "n": n, "q": args.q, "ok": ok,
                              "device_ms_median": round(float(np.median(wall)), 3),
                              "device_ms_min": round(float(np.min(wall)), 3),
                              "host_ms_median": host_ms,
                              "phase_ms": {"prep": round(float(ph[0]), 3), "miller": round(float(ph[1]), 3),
                                           "fexp": round(float(ph[2]), 3)},
                              "per_credential_us": round(float(np.min(wall)) * 1e3 / n, 3)}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
