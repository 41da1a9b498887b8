"""GPU debugging aid for the RLC path: accept flag for single / multi partials on valid batches."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "coconut-rust_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import coconut
from coconut.dist import DeviceEngine
from test_gpu_parity import _gen_batch
for mode in (0, 1):
    ctx = coconut.Context(0, coconut.GroupMode(mode))
    sb = 192 if mode == 0 else 97
    for n in (1, 8):
        b = _gen_batch(mode, n, 6, seed=5, bad_every=n + 1)
        ctx.set_params(b["g_tilde"]); ctx.set_verkey(b["X"], b["Y"])
        dev = torch.device("cuda", 0)
        t = lambda x: torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)
        s1, s2, ms = t(b["s1"]), t(b["s2"]), t(b["msgs"])
        vh = coconut.verify_batch(ctx, n, 6, b["s1"], b["s2"], b["msgs"])
        e = DeviceEngine(ctx, n, 6, s1, s2, ms, base_index=0, seed=bytes(32))
        print("host-path verdicts", vh.tolist()[:8], "device-path before rlc", e.per_credential().tolist()[:8])
        p = e.partial().clone()
        gt = torch.zeros(576, dtype=torch.uint8, device=dev)
        ok = e.finish(p.reshape(1, -1), 1)
        print("mode", mode, "n", n, "accept", ok, "flag", int(p[144]), "perc", e.per_credential().tolist()[:8])
        # two partials of the halves
        if n >= 2:
            h = n // 2
            e0 = DeviceEngine(ctx, h, 6, s1[:h*sb], s2[:h*sb], ms[:h*6*48], base_index=0, seed=bytes(32))
            p0 = e0.partial().clone()
            e1 = DeviceEngine(ctx, n-h, 6, s1[h*sb:], s2[h*sb:], ms[h*6*48:], base_index=h, seed=bytes(32))
            p1 = e1.partial().clone()
            print("   split accept", e1.finish(torch.stack([p0, p1]), 2))
