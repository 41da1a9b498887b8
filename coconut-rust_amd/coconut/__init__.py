"""coconut (MI355X) — host-side mirror of the reference crate's verifier API over the HIP C ABI.

Mirrors 3for/coconut-rust (`/root/reference/src/lib.rs:26-31` module list) for the hot path only:
`signature` (Signature::verify / aggregate, Verkey::aggregate + batch entry points), `pok_sig`
(PoKOfSignatureProof::verify), `errors`.  Every computation runs in libcoconut_hip.so on the GPU;
importing this package on a machine without the built library raises immediately.
"""
from .errors import CoconutError, CoconutErrorKind  # noqa: F401
from ._lib import version, source_hash  # noqa: F401
from .signature import (GroupMode, Params, Verkey, Signature, Context, verify_batch,  # noqa: F401
                        signature_aggregate_batch, verkey_aggregate_batch, verkey_aggregate_ids, fixed_base_mul, subgroup_check, hash_to_curve, hash_msg, params_new,
                        G1_GENERATOR, G2_GENERATOR)
from .pok_sig import PoKOfSignatureProof, pok_verify_batch  # noqa: F401
from .issuance import blind_sign_batch, sigreq_verify_batch, vss_verify_batch  # noqa: F401
