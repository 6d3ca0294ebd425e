#!/usr/bin/env python3
"""Content hash of the native sources (csrc/*.hip, csrc/*.h, include/*.h): the Makefile compiles
it into libacehip.so (acehip_build_hash) and acehip._ffi refuses a library whose hash differs from
the tree it is loaded from, so the binary on the GPU box is provably built from these sources."""
import glob
import hashlib
import os
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # ace-step-1.5_amd/
ROOT = os.path.dirname(PKG)


def native_hash(pkg: str = PKG) -> str:
    root = os.path.dirname(pkg)
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.h")) +
                   glob.glob(os.path.join(root, "include", "*.h")))
    h = hashlib.sha256()
    for f in files:
        rel = os.path.relpath(f, root).replace(os.sep, "/")
        rel = rel.split("/", 1)[1] if rel.startswith(os.path.basename(pkg) + "/") else rel
        h.update(rel.encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(native_hash())
