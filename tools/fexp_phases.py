"""Phase breakdown of the quad-lane final exponentiation (k_fexp_q) from its CC_FEXP_PROF build.

Build (CPU container):  make -C coconut-rust_amd BUILD=build_prof LIB=libcoconut_hip_prof.so \
                            FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DCC_FEXP_PROF"
Run (GPU box):          python tools/fexp_phases.py > gpurun_out/fexp_phases.json
Runs one config-2 verify batch (65,536 credentials) and prints per-phase shader-clock means over the
kernel's waves (lane 0 of each wave stores its totals; the last launch's values are read)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["COCONUT_HIP_LIB"] = os.path.join(ROOT, "coconut-rust_amd", "libcoconut_hip_prof.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "coconut-rust_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import coconut  # noqa: E402

NAMES = ["in", "easy_part", "powx_squarings", "powx_decompress", "powx_tail", "chain_steps", "out", "q12_inv (inside easy_part)"]


def main():
    n, q = 65536, 6
    ctx = coconut.Context(0, coconut.GroupMode(0))
    b = bench.make_verify_batch(ctx, 0, n, q, seed=1000)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    dev = torch.device("cuda", 0)
    d = {k: torch.frombuffer(bytearray(b[k]), dtype=torch.uint8).to(dev) for k in ("s1", "s2", "msgs")}
    v = torch.zeros(n, dtype=torch.uint8, device=dev)
    lib = coconut._lib.lib
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    for _ in range(3):
        st = lib.cc_verify_batch_device(ctx.h, n, q, P(d["s1"]), P(d["s2"]), P(d["msgs"]), P(v), None, None)
        assert st == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), b["expect"])
    nw = (4 * n + 63) // 64
    buf = np.zeros((nw, 8), dtype=np.uint64)
    lib.cck_fexp_prof_read.restype = ctypes.c_int
    lib.cck_fexp_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.cck_fexp_prof_read(buf.ctypes.data_as(ctypes.c_void_p), nw) == 0
    mean = buf.astype(np.float64).mean(axis=0)
    total = mean[:7].sum()
    out = {"waves": nw, "total_clk_per_wave": total, "phases": {}}
    for k in range(8):
        out["phases"][NAMES[k]] = {"clk": round(mean[k]), "frac": round(mean[k] / total, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
