"""Lab: build variants of the word<->region kernels by text substitution on
the product source (csrc/tgfr_wr.hip), each linked with the product's other
objects into tools/lab/build/lib_<name>.so.  Not part of the product: the
product library has no experiment switches; experiments live here.

    python tools/lab/variants.py            # builds every variant in VARIANTS
    python tools/lab/bench_variants.py      # (GPU) times each one
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from text_guided_face_recognition_amd import build as B  # noqa: E402

OUT = os.path.join(ROOT, "tools", "lab", "build")

# name -> list of (old, new) substitutions in tgfr_wr.hip
_OLD_PAD_SKIP = ("  // ---- prologue: G1 of caption 0\n",
            "  if (rt >= NRT) {       // the padding tile: only its share of the DMA\n"
            "    asm volatile(\"s_waitcnt vmcnt(0)\\n\\ts_waitcnt lgkmcnt(0)\\n\\ts_barrier\" ::: \"memory\");\n"
            "    const int T2p = (K + 2) & ~1;\n"
            "    for (int t = 0; t < T2p; ++t) { ring_barrier<0>(); stage_dma(t + 2); }\n"
            "    return;\n  }\n"
            "  // ---- prologue: G1 of caption 0\n")

# round 4: the two-role backward (wr_bwd_duo_kernel) against round 3's
# one-wave-per-SIMD pipe kernel
_DUO = ("""    if (const int e = allow_lds(wr_bwd_duo_kernel, BD_LDS)) return e;
    hipLaunchKernelGGL(wr_bwd_duo_kernel, dim3(grid), dim3(512), BD_LDS, s, Rhi, Whi, B_img,""")
_PIPE = ("""    if (const int e = allow_lds(wr_bwd_pipe_kernel, BP_LDS)) return e;
    hipLaunchKernelGGL(wr_bwd_pipe_kernel, dim3(grid), dim3(256), BP_LDS, s, Rhi, Whi, B_img,""")
VARIANTS = {
    "base": [],
    "pipe": [(_DUO, _PIPE)],
}


def build_variant(name, subs):
    if subs == "HEAD":          # the committed source, for A/B against the work tree
        src = subprocess.run(["git", "show", "HEAD:text_guided_face_recognition_amd/csrc/tgfr_wr.hip"],
                             cwd=ROOT, check=True, capture_output=True, text=True).stdout
        subs = []
    else:
        src = open(os.path.join(B.CSRC, "tgfr_wr.hip")).read()
    for old, new in subs:
        if old not in src:
            raise SystemExit(f"{name}: substitution not found: {old[:60]!r}")
        src = src.replace(old, new)
    os.makedirs(OUT, exist_ok=True)
    vsrc = os.path.join(OUT, f"tgfr_wr_{name}.hip")
    open(vsrc, "w").write(src)
    obj = os.path.join(OUT, f"tgfr_wr_{name}.o")
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-gpu-rdc",
           "-Wno-unused-result", "-Wno-unused-value", "-I", B.CSRC,
           *B.FILE_FLAGS["tgfr_wr.hip"], "-c", vsrc, "-o", obj]
    subprocess.run(cmd, check=True, capture_output=True)
    others = [os.path.join(B.OBJ_DIR, os.path.basename(s).replace(".hip", ".o"))
              for s in B.sources() if not s.endswith("tgfr_wr.hip")]
    lib = os.path.join(OUT, f"lib_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-fno-gpu-rdc",
                    "-o", lib, obj, *others], check=True, capture_output=True)
    return lib


def main(names=None):
    B.build()
    todo = {k: v for k, v in VARIANTS.items() if not names or k in names}
    with ThreadPoolExecutor(4) as ex:
        for lib in ex.map(lambda kv: build_variant(*kv), todo.items()):
            print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
