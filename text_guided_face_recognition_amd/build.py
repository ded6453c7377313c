"""Build libtgfr_hip.so (the C-ABI kernel library) in-tree for gfx950.

    python -m text_guided_face_recognition_amd.build [--verbose]

Each csrc/*.hip compiles to its own object (in parallel, with per-file
flags), then hipcc links the shared library.  Nothing here depends on torch.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
LIB = os.path.join(LIB_DIR, "libtgfr_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TGFR_ARCH", "gfx950")

# Per-file flags.  The word<->region kernels interleave f32 VALU with MFMAs by
# hand: SLP vectorisation would pack adjacent f32 adds/multiplies into
# v_pk_*_f32, which cost more than two plain ops beside MFMAs
# (MI355X_MICROARCH.md, 'price of one filler beside MFMAs').
FILE_FLAGS = {
    "tgfr_wr.hip": ["-fno-slp-vectorize", "-mllvm", "-pragma-unroll-threshold=1000000"],
}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.abspath(__file__)]
    return any(os.path.getmtime(p) > t for p in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"hipcc failed ({res.returncode}): {' '.join(cmd[-3:])}")
    if verbose:
        sys.stderr.write(res.stderr)


def build(force=False, verbose=False, extra=()):
    """Compile every csrc/*.hip and link one shared library; returns its path."""
    if not force and not _stale():
        return LIB
    os.makedirs(OBJ_DIR, exist_ok=True)
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
              "-fno-gpu-rdc", "-Wno-unused-result", "-Wno-unused-value", "-I", CSRC, *extra]
    if verbose:
        common.append("-Rpass-analysis=kernel-resource-usage")
    jobs = []
    for src in sources():
        name = os.path.basename(src)
        obj = os.path.join(OBJ_DIR, name.replace(".hip", ".o"))
        jobs.append(([*common, *FILE_FLAGS.get(name, []), "-c", src, "-o", obj], obj))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(lambda j: _run(j[0], verbose), jobs))
    tmp = LIB + ".tmp"
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-fno-gpu-rdc", "-o", tmp,
          *[o for _, o in jobs]], verbose)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose="--verbose" in sys.argv))
