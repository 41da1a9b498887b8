"""bench.py's multi-GPU launcher on CPU: `--gpus 2` relaunches itself under torch.distributed.run
(before any GPU call) into 2 ranks, which rendezvous on 127.0.0.1, run the barrier / timed loop /
max-over-ranks skeleton, and rank 0 prints ONE JSON line with n_gpus = 2.  The stub step and the gloo
backend replace the GPU step and RCCL (the 8-GPU run is the driver's)."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_gpus2_relaunch_reports_two_ranks():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--mode", "stub", "--steps", "3", "--warmup", "1",
                        # `--n` abbreviates several of torch.distributed.run's options: the relaunch must
                        # not hand it to that parser (bench.py passes its arguments in the environment)
                        "--n", "64"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["backend"] == "gloo"
