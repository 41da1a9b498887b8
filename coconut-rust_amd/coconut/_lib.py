"""Loads libcoconut_hip.so (built in-tree by `make -C coconut-rust_amd`) and declares the C ABI
of include/coconut_hip.h.  No fallback: a missing library is an ImportError."""
import ctypes
import os

from .errors import CoconutError

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("COCONUT_HIP_LIB", os.path.join(os.path.dirname(_HERE), "libcoconut_hip.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libcoconut_hip.so not built at {LIB_PATH}: run `make -C coconut-rust_amd` "
                      "(or __graft_entry__.build()); there is no CPU fallback")

# torch ships its own libamdhip64.so.7 (built for an older ROCm) with the same SONAME as
# /opt/rocm's. Whichever is loaded first serves both, and torch's own device init fails against
# the newer one ("No HIP GPUs are available"). Load torch first so that this library binds to
# torch's runtime. Tensors handed across the ABI then live in the same HIP context.
try:
    import torch  # noqa: F401
except ImportError:  # the C ABI itself needs no torch
    pass

lib = ctypes.CDLL(LIB_PATH)

c_sz = ctypes.c_size_t
c_p = ctypes.c_void_p
c_int = ctypes.c_int
u8p = ctypes.c_char_p

_SIGS = {
    "cc_status_str": (ctypes.c_char_p, [c_int]),
    "cc_version": (ctypes.c_char_p, []),
    "cc_ctx_create": (c_int, [c_int, c_int, ctypes.POINTER(c_p)]),
    "cc_ctx_create_multi": (c_int, [ctypes.c_uint64, c_int, ctypes.POINTER(c_p)]),
    "cc_ctx_num_devices": (c_int, [c_p, ctypes.POINTER(c_int)]),
    "cc_ctx_destroy": (c_int, [c_p]),
    "cc_ctx_mode": (c_int, [c_p, ctypes.POINTER(c_int)]),
    "cc_set_params": (c_int, [c_p, c_p]),
    "cc_set_verkey": (c_int, [c_p, c_p, c_p, c_sz]),
    "cc_set_table_bits": (c_int, [c_p, c_int, c_int]),
    "cc_table_bits": (c_int, [c_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "cc_set_concurrency": (c_int, [c_p, c_int]),
    "cc_concurrency": (c_int, [c_p, ctypes.POINTER(c_int)]),
    "cc_device_error": (c_int, [c_p, c_p, ctypes.POINTER(ctypes.c_uint32)]),
    "cc_verify_batch": (c_int, [c_p, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int]),
    "cc_verify_batch_device": (c_int, [c_p, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_verify_batch_pervk_device": (c_int, [c_p, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_signature_aggregate_batch": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p]),
    "cc_verkey_aggregate_batch": (c_int, [c_p, c_sz, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p]),
    "cc_pok_verify_batch": (c_int, [c_p, c_sz, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                    c_p, c_p]),
    "cc_pok_verify_batch_device": (c_int, [c_p, c_sz, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                           c_p, c_p, c_p]),
    "cc_signature_aggregate_batch_device": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_set_issuers": (c_int, [c_p, c_sz, c_sz, c_p, c_p, c_p]),
    "cc_verkey_aggregate_ids": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p]),
    "cc_verkey_aggregate_ids_device": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p]),
    "cc_aggregate_credential_batch_device": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_subgroup_check": (c_int, [c_p, c_int, c_sz, c_p, c_p]),
    "cc_hash_to_curve": (c_int, [c_p, c_int, c_sz, c_p, c_p, c_p]),
    "cc_hash_msg": (c_int, [c_p, c_sz, c_p, c_p, c_p]),
    "cc_blind_sign_batch": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_sigreq_proof_bytes": (c_sz, [c_p, c_sz]),
    "cc_sigreq_verify_batch": (c_int, [c_p, c_sz, c_sz, c_sz, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_vss_verify_batch": (c_int, [c_p, c_sz, c_sz, c_p, c_p, c_p, c_sz, c_p, c_p, c_p, c_p]),
    "cc_fixed_base_mul": (c_int, [c_p, c_int, c_p, c_sz, c_p, c_p]),
    "cc_rlc_partial_words": (c_int, []),
    "cc_rlc_partial_device": (c_int, [c_p, c_sz, c_sz, ctypes.c_uint64, c_p, c_p, c_p, c_p, c_p, c_p]),
    "cc_rlc_finish_device": (c_int, [c_p, c_sz, c_p, c_p, c_p, c_p]),
    "cc_last_timing": (c_int, [c_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                               ctypes.POINTER(ctypes.c_float)]),
    "cc_set_timing": (c_int, [c_p, c_int]),
    "cc_selftest_lazy": (c_int, [c_int, c_sz, c_p, c_p, c_p, c_p, c_p]),
}

for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def version() -> str:
    """cc_version(): library version and the source hash it was built from (tools/src_hash.py)."""
    return lib.cc_version().decode()


def source_hash() -> str:
    """The 16-hex-digit source hash embedded at build time ("unknown" for a build outside the Makefile)."""
    v = version()
    return v.split(" src ", 1)[1].strip() if " src " in v else "unknown"


def check(status: int, what: str = ""):
    if status != 0:
        raise CoconutError(status, f"{what}: {lib.cc_status_str(status).decode()}")


def buf(b):
    """bytes/bytearray/numpy -> (ctypes pointer, keepalive)."""
    if b is None:
        return None, None
    import numpy as np
    if isinstance(b, (bytes, bytearray)):
        if not len(b):
            cb = ctypes.create_string_buffer(1)
            return ctypes.cast(cb, c_p), cb
        # no copy: every buffer this passes is a `const` input of the C ABI (read during the call only)
        a = np.frombuffer(b, dtype=np.uint8)
        return ctypes.c_void_p(a.ctypes.data), a
    a = np.ascontiguousarray(b)
    return ctypes.c_void_p(a.ctypes.data), a


def need(b, nbytes: int, what: str):
    """The byte count the C ABI will read from `b` (it trusts the caller's counts): a shorter buffer
    is CC_ERR_DECODE here instead of a read past its end there."""
    if nbytes > 0 and (b is None or len(b) < nbytes):
        from .errors import CoconutError
        got = 0 if b is None else len(b)
        raise CoconutError(-4, f"{what}: {got} bytes, the call reads {nbytes}")
