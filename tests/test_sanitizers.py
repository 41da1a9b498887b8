"""Host sanitizers (SURVEY.md §5 "Race detection / sanitizers"), CPU only.

* The C oracle built with -fsanitize=address,undefined (oracle/c `make san`, tests/san_oracle.py) runs the
  oracle's golden-fixture tests (tests/test_oracle.py) and the multi-rank gloo tests (tests/test_dist.py,
  whose CPU engine takes its verdicts from the oracle) — in a child pytest with CC_ORACLE_SAN=1, so no
  sanitizer runtime is loaded into this process.
* The concurrency-slot bookkeeping of the C ABI (coconut-rust_amd/csrc/slots.h, the code capi.cpp runs over
  HIP streams and events) is compiled with the same sanitizers against a simulated device timeline
  (tests/host/test_slots.cpp): a workspace set missing a member must be refused, a slot's buffers must not
  be reallocated while its batch is queued, and a launch failing half-way must still fence its slot.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def _san_env():
    return dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


def test_slot_bookkeeping_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "test_slots")
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", *SAN, "-I",
                           os.path.join(ROOT, "coconut-rust_amd", "csrc"),
                           os.path.join(ROOT, "tests", "host", "test_slots.cpp"), "-o", exe])
    p = subprocess.run([exe], capture_output=True, text=True, env=_san_env())
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all checks passed" in p.stdout
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr


def test_sanitized_oracle_catches_an_overread(tmp_path):
    """The sanitized driver has teeth: a verify call whose message buffer is one byte short aborts with
    a heap-buffer-overflow report."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import san_oracle
    from conftest import golden
    san_oracle.build()
    d = golden("verify_g2_q6.json")
    c = d["creds"][0]
    cat = lambda hs: b"".join(bytes.fromhex(h) for h in hs)  # noqa: E731
    o = san_oracle.SanOracle()
    import ctypes
    ver = ctypes.create_string_buffer(1)
    args = [0, 1, d["q"], bytes.fromhex(c["sigma1"]), bytes.fromhex(c["sigma2"]), cat(c["msgs"]),
            bytes.fromhex(d["vk"]["X"]), cat(d["vk"]["Y"]), 0, bytes.fromhex(d["g_tilde"]), ver, None, 1]
    o.oc_verify_batch(*args)
    assert ver.raw[0] == c["verdict"]
    args[5] = args[5][:-1]
    with pytest.raises(AssertionError, match="heap-buffer-overflow"):
        o.oc_verify_batch(*args)


def test_oracle_and_gloo_suites_under_asan_ubsan(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import san_oracle
    san_oracle.build()
    log = tmp_path / "calls.log"
    env = dict(_san_env(), CC_ORACLE_SAN="1", CC_ORACLE_SAN_LOG=str(log))
    p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle.py"), os.path.join(ROOT, "tests", "test_dist.py")],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=1500)
    assert p.returncode == 0, p.stdout[-6000:] + p.stderr[-3000:]
    ops = log.read_text().split()
    # every oracle entry point the suites use went through the sanitized build
    assert {"verify", "pairing", "lagrange", "sigagg", "vkagg", "pok"} <= set(ops), sorted(set(ops))
