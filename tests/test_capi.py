"""CPU tests of the drop-in boundary: libcoconut_hip.so loads and exports every symbol that
include/coconut_hip.h declares; host-side argument checking; no compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "coconut_hip.h")
LIB = os.path.join(ROOT, "coconut-rust_amd", "libcoconut_hip.so")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cc_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("cc_ctx_create", "cc_set_params", "cc_set_verkey", "cc_verify_batch", "cc_verify_batch_device",
              "cc_signature_aggregate_batch", "cc_verkey_aggregate_batch", "cc_pok_verify_batch"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: make -C coconut-rust_amd"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_status_strings_and_version():
    from coconut._lib import lib
    assert lib.cc_status_str(0) == b"ok"
    assert lib.cc_status_str(-1) == b"UnsupportedNoOfMessages"
    assert lib.cc_status_str(-2) == b"UnequalNoOfBasesExponents"
    assert b"gfx950" in lib.cc_version()


def test_rlc_partial_size_agrees_with_the_python_side():
    """The partial's size (rlc_part.h: Fp12 product, flag, 16 window sums) as the library exports it is the
    one coconut/dist.py gathers and the header declares."""
    from coconut._lib import lib
    from coconut.dist import PARTIAL_WORDS
    hdr = open(os.path.join(ROOT, "include", "coconut_hip.h")).read()
    assert lib.cc_rlc_partial_words() == PARTIAL_WORDS == int(re.search(r"CC_RLC_PARTIAL_WORDS (\d+)", hdr).group(1))


def test_null_and_bad_arguments_rejected_without_gpu():
    from coconut._lib import lib
    assert lib.cc_ctx_create(0, 7, None) == -4        # bad mode / null out
    assert lib.cc_verify_batch(None, 1, 6, None, None, None, None, None, None, None, 0) == -4
    assert lib.cc_set_params(None, None) == -4
    assert lib.cc_set_concurrency(None, 2) == -4
    assert lib.cc_concurrency(None, None) == -4


def test_ctx_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from coconut import Context, CoconutError
    with pytest.raises(CoconutError):
        Context(0)


def test_package_import_requires_built_library(tmp_path):
    import subprocess
    import sys
    env = dict(os.environ, COCONUT_HIP_LIB=str(tmp_path / "missing.so"))
    r = subprocess.run([sys.executable, "-c", "import coconut"], cwd=os.path.join(ROOT, "coconut-rust_amd"),
                       env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "no CPU fallback" in r.stderr


def _makefile_flags():
    mk = open(os.path.join(ROOT, "coconut-rust_amd", "Makefile")).read()
    flags = re.search(r"^FLAGS \?= (.*)$", mk, flags=re.M).group(1)
    arch = re.search(r"^ARCH \?= (.*)$", mk, flags=re.M).group(1).strip()
    return flags.replace("$(ARCH)", arch)


def test_version_carries_the_source_hash_of_this_tree():
    """cc_version() embeds tools/src_hash.py's hash of csrc/, the header, the Makefile and the flags: the
    loaded library was built from exactly these sources (the default build)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from src_hash import src_hash
    import coconut
    h = src_hash(_makefile_flags())
    assert len(h) == 16
    assert coconut.source_hash() == h, (coconut.version(), h)


def test_source_hash_changes_with_the_sources(tmp_path):
    import shutil
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from src_hash import src_hash
    root = tmp_path / "tree"
    shutil.copytree(os.path.join(ROOT, "coconut-rust_amd", "csrc"), root / "coconut-rust_amd" / "csrc")
    shutil.copy(os.path.join(ROOT, "coconut-rust_amd", "Makefile"), root / "coconut-rust_amd" / "Makefile")
    (root / "include").mkdir()
    shutil.copy(HDR, root / "include" / "coconut_hip.h")
    flags = _makefile_flags()
    h0 = src_hash(flags, str(root))
    assert h0 == src_hash(flags, ROOT)
    f = root / "coconut-rust_amd" / "csrc" / "fexp_q.hip"
    f.write_bytes(f.read_bytes() + b"\n")
    h1 = src_hash(flags, str(root))
    assert h1 != h0
    assert src_hash(flags + " -DX", ROOT) != h0
