"""bench.py's multi-rank path on the one GPU a test box has: `--gpus 2 --backend gloo` relaunches the
bench under torch.distributed.run (two ranks, 127.0.0.1), both ranks on the same GPU.  This is the
path the driver's multi-GPU scaling run takes with RCCL (one rank per GPU): the relaunch before any GPU
call, the barriers and the max-over-ranks clock, the SigG1 leg under a live process group, and in RLC
mode the all-gather of the per-rank partials followed by every rank's finish — which must accept the
all-valid batch of BOTH ranks under the one verkey of the job (a per-rank key once made it reject,
profiles/r06/rehearsal_gloo2).  Small batches and 16-bit tables keep each run to tens of seconds."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(*args):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-pcie", "--vk-bits", "16", *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints, once
    return json.loads(lines[0])


def test_bench_verify_two_ranks():
    d = _bench("--n", "8192")
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["config"]["credentials_per_gpu"] == 8192
    assert d["sigg1"]["value"] > 0  # the SigG1 leg ran under the process group, verdicts checked


def test_bench_rlc_two_ranks():
    d = _bench("--mode", "rlc", "--n", "8192")
    assert d["n_gpus"] == 2 and d["value"] > 0


@pytest.mark.parametrize("mode,n", [("verify-pervk", "4096"), ("aggregate", "256"), ("pok", "4096")])
def test_bench_other_modes_two_ranks(mode, n):
    """The other sharded modes (bench_modes.py) through the same relaunch and clock."""
    extra = ["--iss-bits", "8"] if mode == "aggregate" else []
    d = _bench("--mode", mode, "--n", n, *extra)
    assert d["n_gpus"] == 2 and d["value"] > 0
