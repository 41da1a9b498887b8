"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (test infrastructure only).

`SanOracle` has the ctypes surface of `oracle/build/liboracle.so` that the CPU tests use (oc_verify_batch,
oc_pairing, oc_lagrange, oc_signature_aggregate, oc_verkey_aggregate, oc_pok_verify, oc_gen_mul[_mt]),
but runs every call in `oracle/build/san_driver` (oracle/c/san_driver.c, built by `make -C oracle/c san`
with -fsanitize=address,undefined -fno-sanitize-recover=all): each argument is copied into a heap block
of exactly the caller's length, so a read past an input is a heap-buffer-overflow report, and any
sanitizer report fails the call.  conftest.oracle_lib() returns it when CC_ORACLE_SAN=1
(tests/test_sanitizers.py runs test_oracle.py and the gloo tests that way).
"""
import ctypes
import os
import struct
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "oracle", "build", "san_driver")
LOG = os.environ.get("CC_ORACLE_SAN_LOG")


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle", "c"), "san"])
    return DRIVER


def _blob(a):
    if isinstance(a, (bytes, bytearray)):
        b = bytes(a)
    elif isinstance(a, int):
        b = struct.pack("<q", a) if a < 0 else struct.pack("<Q", a)
    elif isinstance(a, (ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64, ctypes.c_int64)):
        b = struct.pack("<Q", a.value & (2 ** 64 - 1))
    elif isinstance(a, ctypes.Array):
        b = bytes(a)
    else:
        raise TypeError(f"san_oracle: unsupported argument {type(a)}")
    return struct.pack("<Q", len(b)) + b


def _val(a):
    return a.value if hasattr(a, "value") and not isinstance(a, ctypes.Array) else int(a)


class SanOracle:
    """Drop-in for the ctypes oracle library; every call is one sanitized process."""

    def __init__(self):
        if not os.path.exists(DRIVER):
            build()
        self.calls = 0

    def _run(self, op, args, out_lens):
        with tempfile.TemporaryDirectory() as d:
            fin, fout = os.path.join(d, "in"), os.path.join(d, "out")
            with open(fin, "wb") as f:
                for a in args:
                    f.write(_blob(a))
            env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
                       UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
            p = subprocess.run([DRIVER, op, fin, fout], capture_output=True, text=True, env=env)
            if p.returncode != 0 or "runtime error" in p.stderr or "Sanitizer" in p.stderr:
                raise AssertionError(f"san_driver {op} failed (rc {p.returncode}):\n{p.stderr[-4000:]}")
            with open(fout, "rb") as f:
                data = f.read()
        self.calls += 1
        if LOG:
            with open(LOG, "a") as f:
                f.write(op + "\n")
        outs, off = [], 0
        for n in out_lens:
            outs.append(data[off:off + n])
            off += n
        rc = struct.unpack("<i", data[off:off + 4])[0]
        return outs, rc

    @staticmethod
    def _put(buf, data):
        if buf is not None and data:
            ctypes.memmove(buf, data, len(data))

    def oc_verify_batch(self, mode, n, q, s1, s2, msgs, X, Y, per, g, ver, gts, nthreads):
        n = _val(n)
        want = gts is not None
        (v, gt), rc = self._run("verify", [_val(mode), n, _val(q), s1, s2, msgs, X, Y, _val(per), g, _val(nthreads),
                                           int(want)], [n, 576 * n if want else 0])
        self._put(ver, v)
        if want:
            self._put(gts, gt)
        return rc

    def oc_pairing(self, P, Q, out):
        (gt,), rc = self._run("pairing", [P, Q], [576])
        self._put(out, gt)
        return rc

    def oc_lagrange(self, t, ids, out):
        t = _val(t)
        (l,), rc = self._run("lagrange", [t, ids], [48 * t])
        self._put(out, l)
        return rc

    def oc_signature_aggregate(self, mode, L, t, ids, s1, s2, o1, o2):
        sb = 192 if _val(mode) == 0 else 97
        (a, b), rc = self._run("sigagg", [_val(mode), _val(L), _val(t), ids, s1, s2, sb], [sb, sb])
        self._put(o1, a)
        self._put(o2, b)
        return rc

    def oc_verkey_aggregate(self, mode, L, t, q, ids, X, Y, oX, oY):
        ob = 97 if _val(mode) == 0 else 192
        q = _val(q)
        (a, b), rc = self._run("vkagg", [_val(mode), _val(L), _val(t), q, ids, X, Y, ob], [ob, ob * q])
        self._put(oX, a)
        self._put(oY, b)
        return rc

    def oc_pok_verify(self, mode, q, r, s1, s2, J, T, resp, nresp, chal, idx, rev_msgs, X, Y, g, gt):
        (o,), rc = self._run("pok", [_val(mode), _val(q), _val(r), s1, s2, J, T, resp, _val(nresp), chal, idx, rev_msgs,
                                     X, Y, g], [576])
        self._put(gt, o)
        return rc

    def oc_gen_mul_mt(self, group, n, ks, out, nthreads=4):
        n = _val(n)
        ob = 97 if _val(group) == 1 else 192
        (o,), rc = self._run("gen_mul", [_val(group), n, ks], [n * ob])
        self._put(out, o)
        return rc

    def oc_gen_mul(self, group, n, ks, out):
        return self.oc_gen_mul_mt(group, n, ks, out)
