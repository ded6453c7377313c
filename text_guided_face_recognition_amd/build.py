"""Build libtgfr_hip.so (the C-ABI kernel library) in-tree for gfx950.

    python -m text_guided_face_recognition_amd.build [--verbose]

The library is a plain hipcc shared object; nothing here depends on torch.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libtgfr_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TGFR_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def build(force=False, verbose=False, extra=()):
    """Compile every csrc/*.hip into one shared library; returns its path."""
    if not force and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-fgpu-rdc" if False else "-fno-gpu-rdc", "-Wno-unused-result",
           "-I", CSRC, *extra, "-o", tmp, *sources()]
    if verbose:
        cmd.insert(3, "-Rpass-analysis=kernel-resource-usage")
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"hipcc failed ({res.returncode})")
    if verbose:
        sys.stderr.write(res.stderr)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose="--verbose" in sys.argv))
