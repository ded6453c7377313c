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
# round 4: the two-role backward (wr_bwd_duo_kernel) against round 3's
# one-wave-per-SIMD pipe kernel
_DUO = ("""    if (const int e = allow_lds(wr_bwd_duo_kernel, BD_LDS)) return e;
    hipLaunchKernelGGL(wr_bwd_duo_kernel, dim3(grid), dim3(512), BD_LDS, s, Rhi, Whi, B_img,""")
_PIPE = ("""    if (const int e = allow_lds(wr_bwd_pipe_kernel, BP_LDS)) return e;
    hipLaunchKernelGGL(wr_bwd_pipe_kernel, dim3(grid), dim3(256), BP_LDS, s, Rhi, Whi, B_img,""")
# ablations of the two-role backward (timing only: results are wrong)
_SM = ("""      sm_chunk(2 * n, tbs, A0, A1, Mo);
      sm_chunk(2 * n + 1, tbs, A0, A1, Mo);""")
_G3 = ("""          dR[n >> 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Mi[n & 3], rd[n & 7], dR[n >> 2],
                                                              0, 0, 0);""")
_DMA = ("""          if (bd_dma_slot(n) >= 0) dma_piece(t + 2, bd_dma_slot(n));""")
_SWAVE = ("""  // ================================================================== S wave
  const float gL = g1 * 1.4426950408889634f;""")
_MWAVE = ("""    // ================================================================ M wave
    // DMA pieces of one caption (bwd_stage's layout): M wave wid issues""")
VARIANTS = {
    "base": [],
    "head": "HEAD",
    "pipe": [(_DUO, _PIPE)],          # round 3's one-wave-per-SIMD backward
    # the second workgroup barrier per stage (before round 4's pairwise counter)
    "b2": [("""        if (lane == 0) lds_st_release(BD_CNT + 4 * wid, t + 1);""", ""),
           ("""        for (int j = 0; j < 9; ++j) dma_piece(t + 2, j);
      }
    }""", """        for (int j = 0; j < 9; ++j) dma_piece(t + 2, j);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    }"""),
           ("""    lds_wait_ge(BD_CNT + 4 * wid, t + 1);""",
            """    asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");"""),
           ("""    for (int t = 0; t < T2; ++t) asm volatile("s_barrier" ::: "memory");""",
            """    for (int t = 0; t < T2; ++t) asm volatile("s_barrier\\n\\ts_barrier" ::: "memory");""")],
    "nosm": [(_SM, """      asm volatile("" ::"v"(A0), "v"(A1));""")],
    "nog3": [(_G3, """          asm volatile("" ::"v"(Mi[n & 3]), "v"(rd[n & 7]));""")],
    "nodma": [(_DMA, "")],
    "prio_s": [(_SWAVE, _SWAVE + "\n  __builtin_amdgcn_s_setprio(1);")],
    "pf1_5": [("constexpr int BD_PF1 = 3;", "constexpr int BD_PF1 = 5;")],
    "pf3_6": [("constexpr int BD_PF3 = 4;", "constexpr int BD_PF3 = 6;")],
    "pf56": [("constexpr int BD_PF1 = 3;", "constexpr int BD_PF1 = 5;"),
             ("constexpr int BD_PF3 = 4;", "constexpr int BD_PF3 = 6;")],
    "dma_early": [("return (n >= 1 && n <= 17 && (n & 1) == 1) ? (n - 1) / 2 : -1;",
                   "return n < 9 ? n : -1;")],
    "prio_s2": [(_SWAVE, _SWAVE + "\n  __builtin_amdgcn_s_setprio(2);"),
                (_MWAVE, _MWAVE.replace("    // DMA", "    __builtin_amdgcn_s_setprio(0);\n    // DMA"))],
    "prio_m": [(_MWAVE, _MWAVE.replace("    // DMA", "    __builtin_amdgcn_s_setprio(1);\n    // DMA"))],
}


# variants of other sources: name -> (file, substitutions); the timing
# harness for these is the whole bench step (TGFR_LIB=<lib> bench.py)
FILE_VARIANTS = {
    # q/k/v projection (bf16 in / out): 512-workgroup budget instead of 256
    "gemm512": ("tgfr_gemm.hip", [("""  const int per_slice = std::max(1, std::min(m_tiles, 256 / n_slices));
  const int lds = WR_TN * K * 2 + WR_NS * WR_STG;
  auto fn = K == 256 ? &bgemm_wres_kernel<256, true, true> : &bgemm_wres_kernel<128, true, true>;""",
                                   """  const int per_slice = std::max(1, std::min(m_tiles, 512 / n_slices));
  const int lds = WR_TN * K * 2 + WR_NS * WR_STG;
  auto fn = K == 256 ? &bgemm_wres_kernel<256, true, true> : &bgemm_wres_kernel<128, true, true>;""")]),
    # optimiser: 2 float4 per thread (twice the workgroups) instead of 4
    "opt2": ("tgfr_optim.hip", [("VEC_PER_BLOCK = 4 * THREADS;", "VEC_PER_BLOCK = 2 * THREADS;")]),
    # BatchNorm normalise: 32 channels per workgroup (512 workgroups) instead of 64
    "bnct32": ("tgfr_bn.hip", [("constexpr int BN_CT = 64;", "constexpr int BN_CT = 32;")]),
    # IMIM weight gradients: the workgroup budget of the row-slice split
    # (512 kept in round 4; 256 and 128 measured slower)
    "dw768": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg);",
                                 "  dw_plan_n(rows, 4, NS, KS, 768, A, wsf, n_wg);")]),
    "dw256": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg);",
                                 "  dw_plan_n(rows, 4, NS, KS, 256, A, wsf, n_wg);")]),
}


def build_variant(name, subs, fname="tgfr_wr.hip"):
    if subs == "HEAD":          # the committed source, for A/B against the work tree
        src = subprocess.run(["git", "show", f"HEAD:text_guided_face_recognition_amd/csrc/{fname}"],
                             cwd=ROOT, check=True, capture_output=True, text=True).stdout
        subs = []
    else:
        src = open(os.path.join(B.CSRC, fname)).read()
    for old, new in subs:
        if old not in src:
            raise SystemExit(f"{name}: substitution not found: {old[:60]!r}")
        src = src.replace(old, new)
    os.makedirs(OUT, exist_ok=True)
    stem = fname[:-4]
    vsrc = os.path.join(OUT, f"{stem}_{name}.hip")
    open(vsrc, "w").write(src)
    obj = os.path.join(OUT, f"{stem}_{name}.o")
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-gpu-rdc",
           "-Wno-unused-result", "-Wno-unused-value", "-I", B.CSRC,
           *B.FILE_FLAGS.get(fname, []), "-c", vsrc, "-o", obj]
    subprocess.run(cmd, check=True, capture_output=True)
    others = [os.path.join(B.OBJ_DIR, os.path.basename(s).replace(".hip", ".o"))
              for s in B.sources() if not s.endswith(fname)]
    lib = os.path.join(OUT, f"lib_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-fno-gpu-rdc",
                    "-o", lib, obj, *others], check=True, capture_output=True)
    return lib


def main(names=None):
    B.build()
    todo = [(k, v, "tgfr_wr.hip") for k, v in VARIANTS.items() if not names or k in names]
    todo += [(k, v[1], v[0]) for k, v in FILE_VARIANTS.items() if names and k in names]
    with ThreadPoolExecutor(4) as ex:
        for lib in ex.map(lambda a: build_variant(*a), todo):
            print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
