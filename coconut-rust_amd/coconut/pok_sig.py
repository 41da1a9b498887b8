"""PoKOfSignatureProof::verify — host mirror of the ps_sig 0.1.2 API [EXT] the reference exercises
in src/pok_sig.rs:85-105 (`proof.verify(&ps_verkey, &ps_params, revealed_msgs, &chal)`).

Responses are ordered as ps_sig builds them: [r2 for g~, m_i for each hidden i ascending]
(pok_sig init bases g~, Y~_hidden).  The revealed map is keyed by message index; iteration order
does not matter (the sum is order-independent), so indices are sorted here.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, List, Union

import numpy as np

from ._lib import buf, check, lib, need
from .errors import CoconutError
from .signature import GT_BYTES, Context, Params, Verkey, fr_bytes


@dataclass
class PoKOfSignatureProof:
    sigma_1: bytes          # sigma'_1 (SignatureGroup)
    sigma_2: bytes          # sigma'_2
    J: bytes                # OtherGroup
    commitment: bytes       # Schnorr commitment T (OtherGroup)
    responses: List[bytes]  # 48-byte Fr each

    def verify(self, vk: Verkey, params: Params, revealed_msgs: Dict[int, Union[int, bytes]],
               chal: Union[int, bytes], ctx: Context = None) -> bool:
        ctx = ctx or Context.default()
        ctx.set_params(params.g_tilde)
        ctx.set_verkey(vk.X_tilde, vk.Y_tilde)
        idx = sorted(revealed_msgs)
        v = pok_verify_batch(ctx, 1, len(vk.Y_tilde), idx, len(self.responses), self.sigma_1, self.sigma_2,
                             self.J, self.commitment, b"".join(self.responses), fr_bytes(chal),
                             b"".join(fr_bytes(revealed_msgs[i]) for i in idx))
        return bool(v[0])


def pok_verify_batch(ctx: Context, n: int, q: int, revealed_idx, nresp: int, sigma1: bytes, sigma2: bytes,
                     J: bytes, T: bytes, responses: bytes, chal: bytes, revealed_msgs: bytes,
                     want_gt: bool = False):
    """Batch PoK verify against the context's params and shared verkey."""
    r = len(revealed_idx)
    sb, ob = ctx.mode.sig_bytes, ctx.mode.other_bytes
    for v, nb, what in ((sigma1, n * sb, "sigma'_1"), (sigma2, n * sb, "sigma'_2"), (J, n * ob, "J"),
                        (T, n * ob, "commitment"), (responses, n * nresp * 48, "responses"),
                        (chal, n * 48, "challenges"), (revealed_msgs, n * r * 48, "revealed messages")):
        need(v, nb, what)
    idx = np.ascontiguousarray(np.asarray(revealed_idx, dtype=np.uint64)) if r else np.zeros(1, np.uint64)
    verdicts = np.zeros(max(n, 1), dtype=np.uint8)
    gts = np.zeros(max(n, 1) * GT_BYTES, dtype=np.uint8) if want_gt else None
    keep = [buf(x) for x in (sigma1, sigma2, J, T, responses, chal, revealed_msgs)]
    ptrs = [k[0] for k in keep]
    st = lib.cc_pok_verify_batch(ctx.h, n, q, r, nresp, ptrs[0], ptrs[1], ptrs[2], ptrs[3], ptrs[4], ptrs[5],
                                 ctypes.c_void_p(idx.ctypes.data), ptrs[6], ctypes.c_void_p(verdicts.ctypes.data),
                                 ctypes.c_void_p(gts.ctypes.data) if want_gt else None)
    if st != 0:
        raise CoconutError(st, lib.cc_status_str(st).decode())
    if want_gt:
        return verdicts[:n], gts[:n * GT_BYTES].tobytes()
    return verdicts[:n]
