"""How much does per-lane divergence cost the verify kernels?  Times the three verify phases (prep,
Miller, final exponentiation) of a 65,536-credential config-2 batch of distinct credentials against a
batch of 65,536 copies of ONE credential, where every lane of every wave follows the same path (the
divstep inversions of the final exponentiation diverge across lanes on distinct inputs).  GPU tool
(run on the GPU box from the repository root); prints one JSON line.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "coconut-rust_amd"))


def main():
    import torch
    import coconut
    from bench import make_verify_batch, to_dev
    n, q, steps = 65536, 6, 5
    dev = torch.device("cuda", 0)
    ctx = coconut.Context(0, coconut.GroupMode.SIG_G2)
    b = make_verify_batch(ctx, 0, n, q, seed=77, bad_every=0)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    lib = coconut._lib.lib
    out = {}
    for name, (s1, s2, m) in {"distinct": (b["s1"], b["s2"], b["msgs"]),
                              "identical": (b["s1"][:192] * n, b["s2"][:192] * n, b["msgs"][:q * 48] * n)}.items():
        d1, d2, dm = to_dev(s1, dev), to_dev(s2, dev), to_dev(m, dev)
        v = torch.zeros(n, dtype=torch.uint8, device=dev)
        st = torch.cuda.Stream(dev)
        sh = ctypes.c_void_p(st.cuda_stream)

        def step():
            r = lib.cc_verify_batch_device(ctx.h, n, q, ctypes.c_void_p(d1.data_ptr()), ctypes.c_void_p(d2.data_ptr()),
                                           ctypes.c_void_p(dm.data_ptr()), ctypes.c_void_p(v.data_ptr()), None, sh)
            assert r == 0
        step()
        torch.cuda.synchronize(dev)
        ctx.timing(True)
        ph = np.zeros(3)
        for _ in range(steps):
            step()
            ph += np.array(ctx.last_timing())
        ctx.timing(False)
        torch.cuda.synchronize(dev)
        assert int(v.sum().item()) == n, "every credential of the batch is valid"
        out[name] = dict(zip(("prep_ms", "miller_ms", "fexp_ms"), np.round(ph / steps, 3).tolist()))
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
