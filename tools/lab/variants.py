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
VARIANTS = {
    "base": [],
    "pf5": [("constexpr int PF_BWD = 3;", "constexpr int PF_BWD = 5;")],
    "nopref": [("constexpr int BU_NPF = 2; ", "constexpr int BU_NPF = 0; ")],
    # ablations (wrong results; timing only)
    "no_sm": [("      sm_chunk(m, tbs, A0, A1, Mo);", "      if (m == 63) { Mo[0] = Mo[1] = Mo[2] = Mo[3] = "
               "__builtin_bit_cast(bf16x8, A0n[0] > 1e30f ? rd[0] : rd[1]); }")],
    "no_dma": [("        if (t < K) stage_dma(n + 2);", "")],
    "no_g3rd": [("    auto read = [&](int m) { return m < 32 ? g3_read(m, x3) : g1_read(m - 32, x1); };",
                 "    auto read = [&](int m) { return m < 32 ? rd[(m + 5) & 7] : g1_read(m - 32, x1); };")],
    "no_rd": [("    auto read = [&](int m) { return m < 32 ? g3_read(m, x3) : g1_read(m - 32, x1); };",
               "    auto read = [&](int m) { return rd[(m + 5) & 7]; };")],
    "pure": [("      sm_chunk(m, tbs, A0, A1, Mo);", "      if (m == 63) { Mo[0] = Mo[1] = Mo[2] = Mo[3] = "
               "__builtin_bit_cast(bf16x8, A0n[0] > 1e30f ? rd[0] : rd[1]); }"),
             ("        if (t < K) stage_dma(n + 2);", ""),
             ("    auto read = [&](int m) { return m < 32 ? g3_read(m, x3) : g1_read(m - 32, x1); };",
              "    auto read = [&](int m) { return rd[(m + 5) & 7]; };")],
    # MFMA chains interleaved: G3 slot m -> (dt = m & 7, ks = m >> 3); G1 alternates A0 / A1
    "ilv": [("    const int dt = u >> 2, ks = u & 3;", "    const int dt = u & 7, ks = u >> 3;"),
            ("        const int ks = m & 3;\n        dR[m >> 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(\n"
             "            Mi[ks], __builtin_bit_cast(bf16x8, op), dR[m >> 2], 0, 0, 0);",
             "        const int ks = m >> 3;\n        dR[m & 7] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(\n"
             "            Mi[ks], __builtin_bit_cast(bf16x8, op), dR[m & 7], 0, 0, 0);"),
            ("    auto read = [&](int m) { return m < 32 ? g3_read(m, x3) : g1_read(m - 32, x1); };",
             "    auto ilv = [](int v) { return (v >> 1) + 16 * (v & 1); };\n"
             "    auto read = [&](int m) { return m < 32 ? g3_read(m, x3) : g1_read(ilv(m - 32), x1); };"),
            ("        g1_mfma(m - 32, op, A0n, A1n, init);", "        g1_mfma(ilv(m - 32), op, A0n, A1n, init);")],
    "nosb": [("      sm_chunk(m, tbs, A0, A1, Mo);\n      __builtin_amdgcn_sched_barrier(0);",
              "      sm_chunk(m, tbs, A0, A1, Mo);")],
    "sgb": [("      sm_chunk(m, tbs, A0, A1, Mo);\n      __builtin_amdgcn_sched_barrier(0);",
             "      sm_chunk(m, tbs, A0, A1, Mo);\n      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);\n"
             "      __builtin_amdgcn_sched_group_barrier(0x2, 4, 0);\n"
             "      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);")],
    # s_memtime stamps of the unit backward's phases into the workspace tail
    "stamps": [
        ("  if (N == 0) return;\n",
         "  if (N == 0) return;\n"
         "  unsigned long long* stamps_ = (unsigned long long*)(slab + (long long)G * "
         "max_contrib * 4 * BU_TILE) + (blockIdx.x * 4 + wid) * 16;\n"
         "#define STAMP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
         "if (lane == 0) stamps_[(k)] = t_; } while (0)\n"
         "  int seg_ = 0;\n  STAMP(0);\n"),
        ("  for (int ns = 0; ns < N;) {\n", "  STAMP(1);\n  for (int ns = 0; ns < N;) {\n"),
        ("    const int S = K + 1;  ", "    if (seg_ < 3) STAMP(2 + 4 * seg_);\n    const int S = K + 1;  "),
        ("    // ---- flush this segment's dR partial\n",
         "    if (seg_ < 3) STAMP(3 + 4 * seg_);\n    // ---- flush this segment's dR partial\n"),
        ("    ns += K;\n", "    if (seg_ < 3) { STAMP(4 + 4 * seg_); stamps_[5 + 4 * seg_] = K; }\n"
                          "    ++seg_;\n    ns += K;\n"),
        ("  // ---- last ticket, then the reductions this workgroup drew\n",
         "  STAMP(14);\n  // ---- last ticket, then the reductions this workgroup drew\n"),
        ("  n_red = min(red_count(), BU_MAXRED);\n",
         "  n_red = min(red_count(), BU_MAXRED);\n  STAMP(13);\n  if (lane == 0) stamps_[12] = n_red;\n"),
        ("          if (rt * 32 + r < NREG) dst[r * s_r + (dt * 32 + lr) * s_d] = acc[dt][gq][k];\n"
         "        }\n  }\n}\n",
         "          if (rt * 32 + r < NREG) dst[r * s_r + (dt * 32 + lr) * s_d] = acc[dt][gq][k];\n"
         "        }\n  }\n  STAMP(15);\n}\n"),
        ("    *floats = (long long)pl.G * pl.max_contrib * 4 * BU_TILE;",
         "    *floats = (long long)pl.G * pl.max_contrib * 4 * BU_TILE + 1024 * 16 * 2;"),
    ],
}


def build_variant(name, subs):
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
