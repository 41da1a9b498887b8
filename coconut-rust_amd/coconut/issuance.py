"""Issuer-side batch entry points — host mirror of reference src/signature.rs:124-444 (SURVEY.md
§8(f) row 3): BlindSignature::new (382-433) and SignatureRequestProof::verify (324-377) for whole
batches of signature requests, through include/coconut_hip.h."""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import numpy as np

from ._lib import buf, check, lib, need
from .signature import Context


def blind_sign_batch(ctx: Context, q: int, k: int, commitments: Sequence[bytes], known: Sequence[Sequence[bytes]],
                     ciphertexts: Sequence[Sequence[tuple]], x: bytes, y: Sequence[bytes]):
    """Per request: (h, c~1, c~2) = BlindSignature::new(request, Sigkey{x, y}); returns three lists."""
    n = len(commitments)
    sb = ctx.mode.sig_bytes
    cm = b"".join(commitments)
    kn = b"".join(m for row in known for m in row)
    ct = b"".join(a + b for row in ciphertexts for a, b in row)
    yb = b"".join(y)
    for v, nb, what in ((cm, n * sb, "commitments"), (kn, n * max(q - k, 0) * 48, "known messages"),
                        (ct, n * k * 2 * sb, "ciphertexts"), (x, 48, "x"), (yb, q * 48, "y")):
        need(v, nb, what)
    outs = [np.zeros(max(n, 1) * sb, dtype=np.uint8) for _ in range(3)]
    keep = [buf(v) for v in (cm, kn, ct, x, yb)]
    check(lib.cc_blind_sign_batch(ctx.h, n, q, k, keep[0][0], keep[1][0] if kn else None, keep[2][0] if ct else None,
                                  keep[3][0], keep[4][0], *[ctypes.c_void_p(o.ctypes.data) for o in outs]),
          "cc_blind_sign_batch")
    raw = [o.tobytes() for o in outs]
    return tuple([r[i * sb:(i + 1) * sb] for i in range(n)] for r in raw)


def sigreq_verify_batch(ctx: Context, q: int, k: int, g: bytes, h: Sequence[bytes], commitments: Sequence[bytes],
                        known: Sequence[Sequence[bytes]], ciphertexts: Sequence[Sequence[tuple]],
                        elgamal_pks: Sequence[bytes], proofs: Sequence[bytes], chals: Sequence[bytes]) -> np.ndarray:
    """SignatureRequestProof::verify per request; proofs packed as cc_sigreq_proof_bytes describes."""
    n = len(commitments)
    pb = lib.cc_sigreq_proof_bytes(ctx.h, k)
    if any(len(p) != pb for p in proofs):
        raise ValueError(f"each proof must be {pb} bytes")
    kn = b"".join(m for row in known for m in row)
    ct = b"".join(a + b for row in ciphertexts for a, b in row)
    sb = ctx.mode.sig_bytes
    parts = (g, b"".join(h[:k]), b"".join(commitments), kn, ct, b"".join(elgamal_pks), b"".join(proofs),
             b"".join(chals))
    for v, nb, what in zip(parts, (sb, k * sb, n * sb, n * max(q - k, 0) * 48, n * k * 2 * sb, n * sb, n * pb,
                                   n * 48),
                           ("g", "h", "commitments", "known messages", "ciphertexts", "ElGamal keys", "proofs",
                            "challenges")):
        need(v, nb, what)
    keep = [buf(v) for v in parts]
    v = np.zeros(max(n, 1), dtype=np.uint8)
    ptr = [kp[0] for kp in keep]
    check(lib.cc_sigreq_verify_batch(ctx.h, n, q, k, ptr[0], ptr[1] if k else None, ptr[2], ptr[3] if kn else None,
                                     ptr[4] if ct else None, ptr[5], ptr[6], ptr[7], ctypes.c_void_p(v.ctypes.data)),
          "cc_sigreq_verify_batch")
    return v[:n]


def vss_verify_batch(ctx: Context, t: int, g: bytes, h: bytes, commitment_sets: Sequence[Sequence[bytes]],
                     set_of: Sequence[int], ids: Sequence[int], shares: Sequence[tuple]) -> np.ndarray:
    """PedersenVSS::verify_share for a batch of (id, (s, s')) against their dealer's commitments (G1)."""
    n = len(ids)
    cm = b"".join(c for cs in commitment_sets for c in cs)
    so = np.ascontiguousarray(np.asarray(set_of, dtype=np.uint32))
    iv = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64))
    sh = b"".join(a + b for a, b in shares)
    for v, nb, what in ((g, 97, "g"), (h, 97, "h"), (cm, len(commitment_sets) * t * 97, "commitments"),
                        (sh, n * 96, "shares")):
        need(v, nb, what)
    if len(so) < n:
        need(None, n, "set_of")
    keep = [buf(v) for v in (g, h, cm, sh)]
    v = np.zeros(max(n, 1), dtype=np.uint8)
    check(lib.cc_vss_verify_batch(ctx.h, n, t, keep[0][0], keep[1][0], keep[2][0], len(commitment_sets),
                                  ctypes.c_void_p(so.ctypes.data), ctypes.c_void_p(iv.ctypes.data), keep[3][0],
                                  ctypes.c_void_p(v.ctypes.data)), "cc_vss_verify_batch")
    return v[:n]
