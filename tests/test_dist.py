"""Multi-rank control flow of coconut/dist.py on CPU: world sizes 2 and 4 over the gloo backend.

The device engine is replaced by a CPU engine whose per-credential verdicts come from the C oracle
(test infrastructure) and whose PARTIAL_WORDS-word partial carries the shard's "not all valid" flag, so these
tests exercise exactly the production sharding, all-gather and collective accept/fallback logic
(`verify_sharded`, `rlc_accept`, `gather_partials`) without a GPU.  The GPU form of the same flow
(real partials, one final exponentiation) is tests/test_gpu_parity.py::test_rlc_partials_*.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import golden, oracle_lib

WORLDS = (2, 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_verdicts(d, idx):
    oc = oracle_lib()
    cr = [d["creds"][i] for i in idx]
    cat = lambda hs: b"".join(bytes.fromhex(h) for h in hs)  # noqa: E731
    ver = ctypes.create_string_buffer(max(len(cr), 1))
    oc.oc_verify_batch(0 if d["mode"] == "G2" else 1, ctypes.c_size_t(len(cr)), ctypes.c_size_t(d["q"]),
                       cat(c["sigma1"] for c in cr), cat(c["sigma2"] for c in cr),
                       cat(m for c in cr for m in c["msgs"]), bytes.fromhex(d["vk"]["X"]),
                       cat(d["vk"]["Y"]), 0, bytes.fromhex(d["g_tilde"]), ver, None, 1)
    return np.frombuffer(ver.raw[:len(cr)], np.uint8).copy()


class OracleEngine:
    """CPU stand-in for DeviceEngine over one rank's slice."""

    def __init__(self, verdicts):
        self.n = len(verdicts)
        self._v = verdicts
        self.fell_back = False

    def partial(self):
        from coconut.dist import PARTIAL_FLAG, PARTIAL_WORDS
        t = torch.zeros(PARTIAL_WORDS, dtype=torch.int32)
        t[:self.n] = torch.from_numpy(self._v.astype(np.int32))[:PARTIAL_FLAG]
        t[PARTIAL_FLAG] = 0 if self._v.all() else 1
        return t

    def finish(self, allp, k):
        from coconut.dist import PARTIAL_FLAG, PARTIAL_WORDS
        assert tuple(allp.shape) == (k, PARTIAL_WORDS)
        return bool((allp[:, PARTIAL_FLAG] == 0).all())

    def per_credential(self):
        self.fell_back = True
        return self._v


def _worker(rank, world, port, idx, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from coconut.dist import shard_bounds, verify_sharded
        d = golden("verify_g2_q6.json")
        lo, hi = shard_bounds(len(idx), world, rank)
        eng = OracleEngine(_oracle_verdicts(d, idx[lo:hi]))
        v = verify_sharded(eng, rlc=True)
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.concatenate([v, [int(eng.fell_back)]]))
    finally:
        dist.destroy_process_group()


def _run(idx, tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), idx, str(tmp_path)), nprocs=world, join=True)
    outs = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    return np.concatenate([o[:-1] for o in outs]), [bool(o[-1]) for o in outs]


def test_shard_bounds_cover_batch():
    from coconut.dist import shard_bounds
    for n in (0, 1, 7, 65536, 1 << 20):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))


@pytest.mark.parametrize("world", WORLDS)
def test_rlc_all_valid_batch_accepted_by_every_rank(tmp_path, world):
    d = golden("verify_g2_q6.json")
    idx = [i for i, c in enumerate(d["creds"]) if c["verdict"] == 1]
    assert len(idx) >= 2
    v, fell = _run(idx, tmp_path, world)
    assert v.all() and len(v) == len(idx)
    assert fell == [False] * world


@pytest.mark.parametrize("world", WORLDS)
def test_rlc_reject_is_collective_and_fallback_exact(tmp_path, world):
    """A bad credential in ONE rank's slice makes EVERY rank fall back (one gathered decision), and
    the concatenated per-credential verdicts equal the fixture's."""
    d = golden("verify_g2_q6.json")
    good = [i for i, c in enumerate(d["creds"]) if c["verdict"] == 1]
    bad = [i for i, c in enumerate(d["creds"]) if c["verdict"] == 0]
    idx = good + bad[:1]  # the bad one lands in the last rank's slice
    v, fell = _run(idx, tmp_path, world)
    assert list(v) == [d["creds"][i]["verdict"] for i in idx]
    assert fell == [True] * world


def test_rlc_more_ranks_than_credentials(tmp_path):
    """Three credentials over four ranks: one rank's shard is empty (a neutral partial), the decision
    is still collective, and a bad credential still makes every rank fall back."""
    d = golden("verify_g2_q6.json")
    good = [i for i, c in enumerate(d["creds"]) if c["verdict"] == 1]
    bad = [i for i, c in enumerate(d["creds"]) if c["verdict"] == 0]
    v, fell = _run(good[:3], tmp_path, 4)
    assert v.all() and len(v) == 3 and fell == [False] * 4
    idx = good[:2] + bad[:1]
    v, fell = _run(idx, tmp_path, 4)
    assert list(v) == [d["creds"][i]["verdict"] for i in idx]
    assert fell == [True] * 4
