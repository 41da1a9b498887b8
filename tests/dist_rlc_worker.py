"""One rank of tests/test_gpu_dist.py (started as a child process BEFORE it touches the GPU): builds
a DeviceEngine on GPU 0 over its half of a q = 16 batch, all-gathers the real 929-word RLC partials
over gloo (host memory), finishes with one final exponentiation, falls back per credential on
reject, and writes its verdicts + fallback flag to <out>/r<rank>.npy.

argv: out_dir corrupt(0/1)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "coconut-rust_amd"))


def main():
    out, corrupt = sys.argv[1], sys.argv[2] == "1"
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import coconut
        from bench import make_verify_batch, to_dev
        from coconut.dist import DeviceEngine, rlc_accept, shard_bounds
        dev = torch.device("cuda", 0)
        ctx = coconut.Context(0, coconut.GroupMode.SIG_G2)
        n, q = 1024, 16
        b = make_verify_batch(ctx, 0, n, q, seed=77, bad_every=0)  # every rank builds the same batch
        ctx.set_params(b["g_tilde"])
        ctx.set_verkey(b["X"], b["Y"])
        s2 = bytearray(b["s2"])
        expect = b["expect"].copy()
        if corrupt:  # credential 700 (rank 1's slice) gets credential 701's sigma_2
            s2[700 * 192:701 * 192] = b["s2"][701 * 192:702 * 192]
            expect[700] = 0
        lo, hi = shard_bounds(n, world, rank)
        e = DeviceEngine(ctx, hi - lo, q, to_dev(b["s1"][lo * 192:hi * 192], dev), to_dev(bytes(s2[lo * 192:hi * 192]), dev),
                         to_dev(b["msgs"][lo * q * 48:hi * q * 48], dev), base_index=lo)
        acc = rlc_accept(e)  # partial -> gloo all-gather of the partials -> one final exponentiation
        v = np.ones(hi - lo, np.uint8) if acc else e.per_credential()  # coconut.dist.verify_sharded
        np.save(os.path.join(out, f"r{rank}.npy"),
                np.concatenate([v.astype(np.int64), expect[lo:hi].astype(np.int64), [int(acc)]]))
        ctx.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
