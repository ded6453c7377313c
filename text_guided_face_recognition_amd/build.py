"""Build libtgfr_hip.so (the C-ABI kernel library) in-tree for gfx950.

    python -m text_guided_face_recognition_amd.build [--verbose]

Each csrc/*.hip compiles to its own object (in parallel, with per-file
flags), then hipcc links the shared library.  Nothing here depends on torch.

The library is stamped with a hash of everything it is built from (sources,
headers, this file's flags): ``stale()`` compares the stamp with the tree, and
the loader (_hip.lib) rebuilds a stale or missing library before mapping it,
so a run never uses a binary built from other sources.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
LIB = os.path.join(LIB_DIR, "libtgfr_hip.so")
STAMP = LIB + ".sha256"
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
HIPCC = "/opt/rocm/bin/hipcc"
ARCH = "gfx950"

# Per-file flags.  The word<->region kernels interleave f32 VALU with MFMAs by
# hand: SLP vectorisation would pack adjacent f32 adds/multiplies into
# v_pk_*_f32, which cost more than two plain ops beside MFMAs
# (MI355X_MICROARCH.md, 'price of one filler beside MFMAs').
FILE_FLAGS = {
    "tgfr_wr.hip": ["-fno-slp-vectorize", "-mllvm", "-pragma-unroll-threshold=1000000"],
}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    """Every file the library is built from."""
    return sorted(sources() + glob.glob(os.path.join(CSRC, "*.h")) +
                  glob.glob(os.path.join(INCLUDE, "*.h")) + [os.path.abspath(__file__)])


def source_hash(extra=()):
    """Hash of every input of the build: the sources and headers, this file,
    the compiler, the target and any extra flags (a debug / experiment build
    never carries the default build's stamp)."""
    h = hashlib.sha256()
    h.update(f"{HIPCC}|{ARCH}|{' '.join(extra)}".encode())
    for p in deps():
        h.update(os.path.relpath(p, os.path.dirname(PKG)).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def stale():
    """True when the library is missing or was built from other sources."""
    if not (os.path.exists(LIB) and os.path.exists(STAMP)):
        return True
    with open(STAMP) as f:
        return f.read().strip() != source_hash()


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
    """Compile every csrc/*.hip and link one shared library; returns its path.
    Concurrent callers (test workers, ranks) serialise on a lock file."""
    if not force and not stale():
        return LIB
    import fcntl
    os.makedirs(LIB_DIR, exist_ok=True)
    with open(os.path.join(LIB_DIR, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and not stale():
            return LIB
        return _build_locked(verbose, extra)


def _build_locked(verbose, extra):
    digest = source_hash(tuple(extra))
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
    with open(STAMP, "w") as f:
        f.write(digest + "\n")
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose="--verbose" in sys.argv))
