"""The multi-process RLC path on a real GPU: two rank
processes, started as children BEFORE either touches the GPU, each drive a DeviceEngine on GPU 0 over
half of a q = 16 batch, all-gather the REAL 929-word partials over gloo (host memory: one box has
one GPU, so RCCL over xGMI between two GPUs is unmeasured on hardware here), and finish with one final
exponentiation each.  Valid batch: both ranks accept.  One swapped sigma_2 in rank 1's slice: both
ranks reject (one gathered decision) and the per-credential fallback verdicts equal construction."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
WORLD = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, corrupt):
    port = _port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_rlc_worker.py"),
                                       str(tmp_path), "1" if corrupt else "0"], env=env))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * WORLD
    outs = [np.load(tmp_path / f"r{r}.npy") for r in range(WORLD)]
    v = np.concatenate([o[:(len(o) - 1) // 2] for o in outs])
    e = np.concatenate([o[(len(o) - 1) // 2:-1] for o in outs])
    return v, e, [bool(o[-1]) for o in outs]


def test_two_process_rlc_accepts_valid_batch(tmp_path):
    v, e, acc = _run(tmp_path, corrupt=False)
    assert acc == [True] * WORLD
    assert e.all() and v.all() and len(v) == 1024


def test_two_process_rlc_rejects_and_falls_back_exactly(tmp_path):
    v, e, acc = _run(tmp_path, corrupt=True)
    assert acc == [False] * WORLD
    assert np.array_equal(v, e) and int(e.sum()) == 1023 and e[700] == 0
