"""Signature / Verkey / Params — host mirror of reference src/signature.rs (verifier side).

The reference API (signature.rs:448-526) is kept name-for-name:

* ``Signature.verify(messages, vk, params)``              -> signature.rs:473-478
* ``Signature.aggregate(threshold, [(id, Signature)])``   -> signature.rs:448-470
* ``Verkey.aggregate(threshold, [(id, Verkey)])``         -> signature.rs:483-526

plus batch entry points (``verify_batch``, ``signature_aggregate_batch``,
``verkey_aggregate_batch``) that hand whole batches to the GPU through the C ABI
(include/coconut_hip.h).  Group elements are carried as amcl_wrapper ``to_bytes`` encodings
(G1 97 B, G2 192 B), scalars as 48-byte big-endian Fr.  Where the reference panics (assert!,
unwrap on PSError) these raise ``CoconutError`` with the matching kind.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple, Union

import numpy as np

from ._lib import need, buf, check, lib
from .errors import CoconutError

FR_BYTES = 48
G1_BYTES = 97
G2_BYTES = 192
GT_BYTES = 576
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class GroupMode(enum.IntEnum):
    """Reference src/lib.rs:3-4 feature mutex; SIG_G2 is the default build."""
    SIG_G2 = 0  # sigma, g, h in G2; X~, Y~, g~ in G1
    SIG_G1 = 1  # sigma, g, h in G1; X~, Y~, g~ in G2

    @property
    def sig_bytes(self) -> int:
        return G2_BYTES if self == GroupMode.SIG_G2 else G1_BYTES

    @property
    def other_bytes(self) -> int:
        return G1_BYTES if self == GroupMode.SIG_G2 else G2_BYTES


def fr_bytes(m: Union[int, bytes]) -> bytes:
    if isinstance(m, (bytes, bytearray)):
        if len(m) != FR_BYTES:
            raise CoconutError(-4, "Fr must be 48 bytes")
        return bytes(m)
    return int(m % R_ORDER).to_bytes(FR_BYTES, "big")


@dataclass
class Params:
    """signature.rs:13-17.  Only g_tilde is read on the verify path."""
    g: bytes
    g_tilde: bytes
    h: List[bytes] = field(default_factory=list)

    def msg_count(self) -> int:
        return len(self.h)


@dataclass
class Verkey:
    """signature.rs:46-49."""
    X_tilde: bytes
    Y_tilde: List[bytes]

    @staticmethod
    def aggregate(threshold: int, keys: Sequence[Tuple[int, "Verkey"]], ctx: "Context" = None) -> "Verkey":
        """signature.rs:483-526 (q+1 Lagrange-weighted MSMs over the first `threshold` keys)."""
        ctx = ctx or Context.default()
        if len(keys) < threshold:
            raise CoconutError(-3, "keys.len() < threshold")
        q = len(keys[0][1].Y_tilde)
        for _, vk in keys[1:]:
            if len(vk.Y_tilde) != q:
                raise CoconutError(-3, "ragged verkeys (reference assert_eq! at signature.rs:486-488)")
        ids = np.array([[i for i, _ in keys]], dtype=np.uint64)
        X = b"".join(vk.X_tilde for _, vk in keys)
        Y = b"".join(y for _, vk in keys for y in vk.Y_tilde)
        oX, oY = verkey_aggregate_batch(ctx, 1, len(keys), threshold, q, ids, X, Y)
        ob = ctx.mode.other_bytes
        return Verkey(oX, [oY[j * ob:(j + 1) * ob] for j in range(q)])


@dataclass
class Signature:
    """signature.rs:68-71."""
    sigma_1: bytes
    sigma_2: bytes

    @staticmethod
    def aggregate(threshold: int, sigs: Sequence[Tuple[int, "Signature"]], ctx: "Context" = None) -> "Signature":
        """signature.rs:448-470: sigma_1 from entry 0, sigma_2 = sum l_i(0) sigma_2_i over the first t."""
        ctx = ctx or Context.default()
        if len(sigs) < threshold or not sigs:
            raise CoconutError(-3, "sigs.len() < threshold")
        ids = np.array([[i for i, _ in sigs]], dtype=np.uint64)
        s1 = b"".join(s.sigma_1 for _, s in sigs)
        s2 = b"".join(s.sigma_2 for _, s in sigs)
        o1, o2 = signature_aggregate_batch(ctx, 1, len(sigs), threshold, ids, s1, s2)
        return Signature(o1, o2)

    def verify(self, messages: Sequence[Union[int, bytes]], vk: Verkey, params: Params,
               ctx: "Context" = None) -> bool:
        """signature.rs:473-478 -> ps_sig Signature::verify: one credential through the batch path."""
        ctx = ctx or Context.default()
        if len(vk.Y_tilde) != len(messages):
            raise CoconutError(-1, f"Verkey valid for {len(vk.Y_tilde)} messages but given {len(messages)}")
        ctx.set_params(params.g_tilde)
        msgs = b"".join(fr_bytes(m) for m in messages)
        v = verify_batch(ctx, 1, len(messages), self.sigma_1, self.sigma_2, msgs,
                         vk=(vk.X_tilde, b"".join(vk.Y_tilde)))
        return bool(v[0])


class Context:
    """One cc_ctx: a HIP device, a stream and device-resident params/verkey tables."""

    _default = {}

    def __init__(self, device: int = 0, mode: GroupMode = GroupMode.SIG_G2, devices: Sequence[int] = None):
        """devices=[...] makes a device-set context (cc_ctx_create_multi): cc_verify_batch shards the
        batch over those GPUs, RLC mode gathers the per-GPU partials with RCCL inside the library."""
        self.mode = GroupMode(mode)
        self.device = device if devices is None else devices[0]
        h = ctypes.c_void_p()
        if devices is None:
            check(lib.cc_ctx_create(device, int(self.mode), ctypes.byref(h)), "cc_ctx_create")
        else:
            mask = 0
            for d in devices:
                mask |= 1 << int(d)
            check(lib.cc_ctx_create_multi(mask, int(self.mode), ctypes.byref(h)), "cc_ctx_create_multi")
        self.h = h
        self._gtilde = None
        self._vk = None
        self._timing = False
        self._iss_q = 0

    @classmethod
    def default(cls, device: int = 0, mode: GroupMode = GroupMode.SIG_G2) -> "Context":
        key = (device, int(mode))
        if key not in cls._default:
            cls._default[key] = Context(device, mode)
        return cls._default[key]

    def close(self):
        if self.h:
            lib.cc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, g_tilde: bytes):
        if self._gtilde == g_tilde:
            return
        need(g_tilde, self.mode.other_bytes, "g_tilde")
        p, keep = buf(g_tilde)
        self._gtilde = None
        try:
            check(lib.cc_set_params(self.h, p), "cc_set_params")
        except Exception:
            self._vk = None  # a failed table rebuild leaves the C context without a verkey
            raise
        self._gtilde = g_tilde

    def set_verkey(self, X: bytes, Y: Sequence[bytes]):
        Yb = b"".join(Y) if not isinstance(Y, (bytes, bytearray)) else bytes(Y)
        key = (bytes(X), Yb)
        if self._vk == key:
            return
        q = len(Yb) // self.mode.other_bytes
        need(X, self.mode.other_bytes, "X~")
        px, k1 = buf(X)
        py, k2 = buf(Yb)
        self._vk = None  # a failed call leaves the context without a verkey
        check(lib.cc_set_verkey(self.h, px, py, q), "cc_set_verkey")
        self._vk = key

    def set_issuers(self, ids, X: bytes, Y: bytes, q: int):
        """Issuer verkey table (cc_set_issuers): ids[k] is issuer k's signer id, X n x OtherGroup,
        Y n x q x OtherGroup; then verkey_aggregate_ids takes id lists only."""
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64))
        ob = self.mode.other_bytes
        need(X, len(ids) * ob, "issuer X~")
        need(Y, len(ids) * q * ob, "issuer Y~")
        px, k1 = buf(X)
        py, k2 = buf(Y)
        check(lib.cc_set_issuers(self.h, len(ids), q, ctypes.c_void_p(ids.ctypes.data), px, py), "cc_set_issuers")
        self._iss_q = q

    def set_concurrency(self, slots: int):
        """cc_set_concurrency: K verify batches in flight on K caller streams (workspace slots taken
        round-robin by the *_device verify calls; 1 = every call ordered against every other)."""
        check(lib.cc_set_concurrency(self.h, int(slots)), "cc_set_concurrency")

    def concurrency(self) -> int:
        v = ctypes.c_int(0)
        check(lib.cc_concurrency(self.h, ctypes.byref(v)), "cc_concurrency")
        return v.value

    def set_table_bits(self, verkey_bits: int = 0, issuer_bits: int = 0):
        """Window widths of the tables later set_verkey / set_issuers calls build (0: by memory)."""
        check(lib.cc_set_table_bits(self.h, verkey_bits, issuer_bits), "cc_set_table_bits")
        self._vk = None  # the next set_verkey rebuilds its tables at the new width, even for the same key

    def table_bits(self):
        """(verkey table bits, issuer table bits) of the current tables (0: none)."""
        v, i = ctypes.c_int(), ctypes.c_int()
        check(lib.cc_table_bits(self.h, ctypes.byref(v), ctypes.byref(i)), "cc_table_bits")
        return v.value, i.value

    def device_error(self, stream=None) -> int:
        """CC_DEVERR_* bits raised by *_device calls since the last read (synchronises the stream)."""
        v = ctypes.c_uint32()
        check(lib.cc_device_error(self.h, stream, ctypes.byref(v)), "cc_device_error")
        return v.value

    def num_devices(self) -> int:
        n = ctypes.c_int()
        check(lib.cc_ctx_num_devices(self.h, ctypes.byref(n)), "cc_ctx_num_devices")
        return n.value

    def timing(self, enabled: bool = True):
        check(lib.cc_set_timing(self.h, int(enabled)))
        self._timing = bool(enabled)

    def last_timing(self):
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        check(lib.cc_last_timing(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value


def verify_batch(ctx: Context, n: int, q: int, sigma1: bytes, sigma2: bytes, msgs: bytes, vk=None,
                 want_gt: bool = False, rlc: bool = False):
    """Batch Signature::verify.  vk=None uses the context's shared verkey (cc_set_verkey);
    vk=(X_bytes, Y_bytes) gives one verkey per credential (n*ob, n*q*ob) or a single verkey
    that is broadcast when len(X) == ob.  Returns verdicts (uint8[n]) [, gts (n*576 bytes)]."""
    ob = ctx.mode.other_bytes
    if vk is not None and len(vk[0]) == ob and n != 1:
        ctx.set_verkey(vk[0], vk[1])
        vk = None
    sb = ctx.mode.sig_bytes
    need(sigma1, n * sb, "sigma_1")
    need(sigma2, n * sb, "sigma_2")
    need(msgs, n * q * 48, "messages")
    if vk is not None:
        need(vk[0], n * ob, "X~ per credential")
        need(vk[1], n * q * ob, "Y~ per credential")
    verdicts = np.zeros(max(n, 1), dtype=np.uint8)
    gts = np.zeros(max(n, 1) * GT_BYTES, dtype=np.uint8) if want_gt else None
    p1, k1 = buf(sigma1)
    p2, k2 = buf(sigma2)
    pm, k3 = buf(msgs)
    px, k4 = buf(vk[0]) if vk is not None else (None, None)
    py, k5 = buf(vk[1]) if vk is not None else (None, None)
    check(lib.cc_verify_batch(ctx.h, n, q, p1, p2, pm, px, py,
                              ctypes.c_void_p(verdicts.ctypes.data),
                              ctypes.c_void_p(gts.ctypes.data) if want_gt else None, int(rlc)),
          "cc_verify_batch")
    if want_gt:
        return verdicts[:n], gts[:n * GT_BYTES].tobytes()
    return verdicts[:n]


def signature_aggregate_batch(ctx: Context, n: int, length: int, t: int, ids, sigma1: bytes, sigma2: bytes):
    sb = ctx.mode.sig_bytes
    ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64).reshape(n, length))
    need(sigma1, n * length * sb, "sigma_1")
    need(sigma2, n * length * sb, "sigma_2")
    o1 = np.zeros(max(n, 1) * sb, dtype=np.uint8)
    o2 = np.zeros(max(n, 1) * sb, dtype=np.uint8)
    p1, k1 = buf(sigma1)
    p2, k2 = buf(sigma2)
    check(lib.cc_signature_aggregate_batch(ctx.h, n, length, t, ctypes.c_void_p(ids.ctypes.data), p1, p2,
                                           ctypes.c_void_p(o1.ctypes.data), ctypes.c_void_p(o2.ctypes.data)),
          "cc_signature_aggregate_batch")
    return o1[:n * sb].tobytes(), o2[:n * sb].tobytes()


def verkey_aggregate_batch(ctx: Context, n: int, length: int, t: int, q: int, ids, X: bytes, Y: bytes):
    ob = ctx.mode.other_bytes
    ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64).reshape(n, length))
    oX = np.zeros(max(n, 1) * ob, dtype=np.uint8)
    oY = np.zeros(max(n * q, 1) * ob, dtype=np.uint8)
    need(X, n * length * ob, "X~")
    need(Y, n * length * q * ob, "Y~")
    px, k1 = buf(X)
    py, k2 = buf(Y)
    check(lib.cc_verkey_aggregate_batch(ctx.h, n, length, t, q, ctypes.c_void_p(ids.ctypes.data), px, py,
                                        ctypes.c_void_p(oX.ctypes.data), ctypes.c_void_p(oY.ctypes.data)),
          "cc_verkey_aggregate_batch")
    return oX[:n * ob].tobytes(), oY[:n * q * ob].tobytes()


def verkey_aggregate_ids(ctx: Context, n: int, length: int, t: int, ids):
    """Verkey::aggregate for n credentials from the issuer table (cc_verkey_aggregate_ids)."""
    ob, q = ctx.mode.other_bytes, ctx._iss_q
    ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64).reshape(n, length))
    oX = np.zeros(max(n, 1) * ob, dtype=np.uint8)
    oY = np.zeros(max(n * q, 1) * ob, dtype=np.uint8)
    check(lib.cc_verkey_aggregate_ids(ctx.h, n, length, t, ctypes.c_void_p(ids.ctypes.data),
                                      ctypes.c_void_p(oX.ctypes.data), ctypes.c_void_p(oY.ctypes.data)),
          "cc_verkey_aggregate_ids")
    return oX[:n * ob].tobytes(), oY[:n * q * ob].tobytes()


def _pack(msgs):
    offs = np.zeros(len(msgs) + 1, dtype=np.uint64)
    for i, m in enumerate(msgs):
        offs[i + 1] = offs[i] + len(m)
    return b"".join(msgs), offs


def hash_to_curve(ctx: Context, group: int, msgs: Sequence[bytes]) -> List[bytes]:
    """amcl_wrapper `from_msg_hash` for a batch of messages on the GPU (cc_hash_to_curve)."""
    eb = G1_BYTES if group == 1 else G2_BYTES
    data, offs = _pack(msgs)
    out = np.zeros(max(len(msgs), 1) * eb, dtype=np.uint8)
    p, k = buf(data)
    check(lib.cc_hash_to_curve(ctx.h, group, len(msgs), p, ctypes.c_void_p(offs.ctypes.data),
                               ctypes.c_void_p(out.ctypes.data)), "cc_hash_to_curve")
    raw = out.tobytes()
    return [raw[i * eb:(i + 1) * eb] for i in range(len(msgs))]


def hash_msg(ctx: Context, msgs: Sequence[bytes]) -> List[bytes]:
    data, offs = _pack(msgs)
    out = np.zeros(max(len(msgs), 1) * 48, dtype=np.uint8)
    p, k = buf(data)
    check(lib.cc_hash_msg(ctx.h, len(msgs), p, ctypes.c_void_p(offs.ctypes.data), ctypes.c_void_p(out.ctypes.data)),
          "cc_hash_msg")
    raw = out.tobytes()
    return [raw[i * 48:(i + 1) * 48] for i in range(len(msgs))]


def params_new(ctx: Context, msg_count: int, label: bytes) -> Params:
    """Params::new (src/signature.rs:22-32) in one batch per group."""
    sg = 2 if ctx.mode == GroupMode.SIG_G2 else 1
    sig = hash_to_curve(ctx, sg, [label + b" : g"] + [label + b" : y" + str(i).encode() for i in range(msg_count)])
    gt = hash_to_curve(ctx, 3 - sg, [label + b" : g_tilde"])[0]
    return Params(g=sig[0], g_tilde=gt, h=sig[1:])


def subgroup_check(ctx: Context, group: int, points: bytes):
    """Per point: 0 identity / invalid encoding, 1 on-curve outside the subgroup, 2 in G1/G2."""
    eb = G1_BYTES if group == 1 else G2_BYTES
    n = len(points) // eb
    st = np.zeros(max(n, 1), dtype=np.uint8)
    p, k = buf(points)
    check(lib.cc_subgroup_check(ctx.h, group, n, p, ctypes.c_void_p(st.ctypes.data)), "cc_subgroup_check")
    return st[:n]


# Standard BLS12-381 generators (amcl_wrapper encodings) — public curve constants.
G1_GENERATOR = bytes.fromhex(
    "04"
    "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"
    "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1")
G2_GENERATOR = bytes.fromhex(
    "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8"
    "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
    "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801"
    "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be")


def fixed_base_mul(ctx: Context, group: int, base: bytes, scalars: bytes) -> bytes:
    """out_i = k_i * base on the GPU (group 1 = G1, 2 = G2); scalars n x 48 B big-endian."""
    n = len(scalars) // FR_BYTES
    eb = G1_BYTES if group == 1 else G2_BYTES
    need(base, eb, "base point")
    out = np.zeros(max(n, 1) * eb, dtype=np.uint8)
    pb, k1 = buf(base)
    ps, k2 = buf(scalars)
    check(lib.cc_fixed_base_mul(ctx.h, group, pb, n, ps, ctypes.c_void_p(out.ctypes.data)), "cc_fixed_base_mul")
    return out[:n * eb].tobytes()
