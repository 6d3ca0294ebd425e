"""Content hash of the product sources (the HIP kernels, the C-ABI header, the Python host):
lets bench.py tell whether counter passes recorded in profiles/ came from the same product code
as the run that splices them in, on a box that receives the tree without its git metadata."""
import glob
import hashlib
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # ace-step-1.5_amd/
_REPO = os.path.dirname(_PKG)


def product_hash() -> str:
    files = sorted(glob.glob(os.path.join(_PKG, "csrc", "*.hip")) + glob.glob(os.path.join(_PKG, "csrc", "*.h")) +
                   glob.glob(os.path.join(_PKG, "acehip", "*.py")) + glob.glob(os.path.join(_REPO, "include", "*.h")))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, _REPO).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
