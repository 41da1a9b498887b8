#!/usr/bin/env python3
"""Source hash of the product library (embedded in cc_version() by coconut-rust_amd/Makefile).

sha256 over the library's sources — every file in coconut-rust_amd/csrc/, include/coconut_hip.h and
the Makefile, each as its path relative to the repository root and its bytes, in sorted path order —
and the compile flags, first 16 hex digits.  A library built from other sources or flags reports
another hash, so a bench line or a smoke log names exactly the tree its binary came from.

Usage: src_hash.py "<flags>"   (prints the hash; the Makefile passes its FLAGS + HOT_FLAGS)
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root=ROOT):
    csrc = os.path.join(root, "coconut-rust_amd", "csrc")
    files = [os.path.join(csrc, f) for f in os.listdir(csrc) if os.path.isfile(os.path.join(csrc, f))]
    files += [os.path.join(root, "include", "coconut_hip.h"), os.path.join(root, "coconut-rust_amd", "Makefile")]
    return sorted(os.path.relpath(f, root) for f in files)


def src_hash(flags, root=ROOT):
    h = hashlib.sha256()
    for rel in source_files(root):
        with open(os.path.join(root, rel), "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    h.update(b"flags\0" + " ".join(flags.split()).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_hash(sys.argv[1] if len(sys.argv) > 1 else ""))
