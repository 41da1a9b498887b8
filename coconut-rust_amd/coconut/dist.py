"""Multi-GPU batch verification: one process per GPU over torch.distributed (backend "nccl" is RCCL
on ROCm, riding xGMI between the GPUs of a node).  SURVEY.md §8e.

The batch shards by credential (credentials are independent):

* per-credential mode — every rank verifies its own contiguous slice; no collective on the data
  path (verdicts stay with the rank that owns the slice);
* RLC mode — every rank reduces its slice to one 929-word partial (the Fp12 Miller product of its
  delta-weighted pairs, a fall-back flag and its 16 fold window sums, ``cc_rlc_partial_device``); ONE
  all-gather of the partials (3,716 B per rank) is the only exchange; every rank pairs the gathered
  window sums with the fixed multiples of g~, multiplies everything and runs the single final
  exponentiation (``cc_rlc_finish_device``), so all ranks reach the same accept/reject
  decision without a second collective.  On reject every rank falls back to per-credential
  verification of its own slice, so verdicts always equal the reference's
  (``Signature::verify``, reference src/signature.rs:473-478, per credential).

Engines decouple this control flow from the device: ``DeviceEngine`` drives libcoconut_hip.so on
device-resident tensors; tests substitute a CPU engine to exercise the same sharding, gather and
decision logic over the gloo backend.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

# 144 Fp12 Montgomery words, fall-back flag, 16 x (48-word affine window sum + identity flag):
# CC_RLC_PARTIAL_WORDS of include/coconut_hip.h (= cc_rlc_partial_words(), checked by tests/test_capi.py)
PARTIAL_WORDS = 929
PARTIAL_FLAG = 144


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous slice [lo, hi) of an n-credential batch owned by `rank` of `world`."""
    return n * rank // world, n * (rank + 1) // world


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def gather_partials(part, group=None):
    """All-gather the per-rank partials (one tensor of PARTIAL_WORDS int32 each) -> (stacked, k).
    Over RCCL ("nccl") the device tensors are gathered in place (3,716 B per rank over xGMI); over gloo
    (CPU transport: tests, hosts without RCCL) a device partial crosses through host memory and the
    gathered partials return to its device."""
    import torch
    dist = _dist()
    world = dist.get_world_size(group) if dist else 1
    if world == 1:
        return part.reshape(1, -1), 1
    dev = part.device
    host = dev.type != "cpu" and dist.get_backend(group) == "gloo"
    src = part.cpu() if host else part
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    out = torch.stack(parts)
    return (out.to(dev) if host else out), world


def rlc_accept(engine, group=None) -> bool:
    """One RLC decision for the whole (sharded) batch: partial -> all-gather -> finish."""
    part = engine.partial()
    allp, k = gather_partials(part, group)
    return engine.finish(allp, k)


def verify_sharded(engine, rlc: bool = True, group=None) -> np.ndarray:
    """Verdicts (uint8) for this rank's slice; RLC first when requested, per-credential fallback."""
    if rlc and rlc_accept(engine, group):
        return np.ones(engine.n, dtype=np.uint8)
    return engine.per_credential()


class DeviceEngine:
    """One rank's slice, resident in HBM as torch tensors, checked through the C ABI."""

    def __init__(self, ctx, n: int, q: int, d_s1, d_s2, d_msgs, base_index: int = 0,
                 seed: Optional[bytes] = None, stream=None):
        import torch
        from ._lib import lib
        self.lib, self.ctx, self.n, self.q = lib, ctx, n, q
        self.d_s1, self.d_s2, self.d_msgs = d_s1, d_s2, d_msgs
        self.base_index = base_index
        self.seed = seed
        self.dev = d_s1.device
        # a real (non-null) stream: a NULL handle would select the context's own non-blocking stream,
        # which is not ordered against torch's default stream
        self.stream = stream if stream is not None else torch.cuda.Stream(self.dev)
        self._sh = ctypes.c_void_p(self.stream.cuda_stream)
        # two partial / accept buffers: a pipelined caller's finish of batch i (finish_async, on its own
        # stream) may still read one while the next partial writes the other.  A third partial issued
        # before batch i's finish has run reuses batch i's slot: partial() then makes the engine's stream
        # wait (on the device) for that finish's event, so the slot is never overwritten while read.
        self._parts = [torch.empty(PARTIAL_WORDS, dtype=torch.int32, device=self.dev) for _ in range(2)]
        self._accepts = [torch.zeros(1, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        self._slot_ev = [None, None]
        self._slot = 0
        self.part = self._parts[0]
        self.accept = self._accepts[0]
        self._fin_stream = None
        self.verdicts = torch.zeros(n, dtype=torch.uint8, device=self.dev)

    def _enter(self):
        import torch
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))

    def _leave(self):
        import torch
        torch.cuda.current_stream(self.dev).wait_stream(self.stream)

    def _check(self, st, what):
        if st != 0:
            from .errors import CoconutError
            raise CoconutError(st, f"{what}: {self.lib.cc_status_str(st).decode()}")

    def partial(self):
        seed = self.seed if self.seed is not None else os.urandom(32)
        self._slot ^= 1
        self.part = self._parts[self._slot]
        self._enter()
        if self._slot_ev[self._slot] is not None:  # a finish_async still reading this slot
            self.stream.wait_event(self._slot_ev[self._slot])
            self._slot_ev[self._slot] = None
        self._check(self.lib.cc_rlc_partial_device(self.ctx.h, self.n, self.q, self.base_index, seed,
                                                   ctypes.c_void_p(self.d_s1.data_ptr()),
                                                   ctypes.c_void_p(self.d_s2.data_ptr()),
                                                   ctypes.c_void_p(self.d_msgs.data_ptr()),
                                                   ctypes.c_void_p(self.part.data_ptr()), self._sh),
                    "cc_rlc_partial_device")
        self._leave()
        return self.part

    def finish(self, allp, k: int, sync: bool = True):
        allp = allp.contiguous()
        self._enter()
        self._check(self.lib.cc_rlc_finish_device(self.ctx.h, k, ctypes.c_void_p(allp.data_ptr()),
                                                  ctypes.c_void_p(self.accept.data_ptr()), None, self._sh),
                    "cc_rlc_finish_device")
        self._leave()
        if not sync:
            return None
        return bool(self.accept.item())

    def finish_async(self, allp, k: int):
        """cc_rlc_finish_device on the engine's second stream, NOT ordered before later work on the
        engine's main stream: the next batch's partial() can overlap this batch's final exponentiation.
        Returns a callable that waits for the decision and returns it.  Any number of finishes may be
        outstanding: the library runs the finishes of one context in call order, and a partial() that
        reuses the slot of an unfinished batch waits for that batch's finish on the device."""
        import torch
        if self._fin_stream is None:
            # high priority: the finish's latency-bound launches (16 waves of window pairs per partial, the
            # product tree, one final exponentiation) take wave slots ahead of the next partial's full
            # launches instead of queueing behind them
            self._fin_stream = torch.cuda.Stream(self.dev, priority=-1)
        fs = self._fin_stream
        allp = allp.contiguous()
        fs.wait_stream(torch.cuda.current_stream(self.dev))  # the gathered partials are ready
        fs.wait_stream(self.stream)
        allp.record_stream(fs)
        acc = self._accepts[self._slot]
        self._check(self.lib.cc_rlc_finish_device(self.ctx.h, k, ctypes.c_void_p(allp.data_ptr()),
                                                  ctypes.c_void_p(acc.data_ptr()), None,
                                                  ctypes.c_void_p(fs.cuda_stream)), "cc_rlc_finish_device")
        # the decision is copied out on the finish stream, so a later batch reusing this slot cannot
        # change what result() returns
        host = torch.empty(1, dtype=torch.uint8, pin_memory=True)
        with torch.cuda.stream(fs):
            host.copy_(acc, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(fs)
        self._slot_ev[self._slot] = ev

        def result() -> bool:
            ev.synchronize()
            return bool(host[0].item())
        return result

    def per_credential(self) -> np.ndarray:
        self._enter()
        self._check(self.lib.cc_verify_batch_device(self.ctx.h, self.n, self.q,
                                                    ctypes.c_void_p(self.d_s1.data_ptr()),
                                                    ctypes.c_void_p(self.d_s2.data_ptr()),
                                                    ctypes.c_void_p(self.d_msgs.data_ptr()),
                                                    ctypes.c_void_p(self.verdicts.data_ptr()), None, self._sh),
                    "cc_verify_batch_device")
        self._leave()
        return self.verdicts.cpu().numpy()
