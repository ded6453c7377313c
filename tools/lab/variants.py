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
# round 5: the two-role backward on the forward's stored scores
_SM = ("""        sm_chunk(bigc, c, tbs, spc, mc, Q, Mo);""")
_G3 = ("""          dR[n >> 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Mi[n & 3], rd[n & 7], dR[n >> 2],
                                                              0, 0, 0);""")
_DMA = ("""          if (bd_dma_slot(n) >= 0) dma_piece(t + 2, bd_dma_slot(n));""")
_G1 = ("""      g1_mfma(n, rd[n & 3], Qn);""")
_SWAVE = ("""  // ================================================================== S wave
  const float gL = g1 * 1.4426950408889634f;""")
_MWAVE = ("""    // ================================================================ M wave
    // DMA pieces of one caption: M wave wid issues pieces k = wid + 4 j""")
# per-stage s_memtime stamps (tools/lab/stamps.py reads them back through
# tgfr_lab_stamps): S wave after B1 / after its slot loop / after the M-slot
# wait; M wave after B1 / after its G3 loop
_STAMP_DECL = ("""constexpr int BD_NB = 4;                        // X ring depth""",
               """__device__ unsigned long long g_st[256 * 8 * 64 * 4];
#define STAMP(t, k) do { if (blockIdx.x < 256 && (t) < 64) \\
  g_st[((blockIdx.x * 8 + wv) * 64 + (t)) * 4 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
constexpr int BD_NB = 4;                        // X ring depth""")
_STAMPS = [
    _STAMP_DECL,
    ("""      ring_barrier<0>();                       // B1: X(t+1) landed; M(t-1) written
""", """      ring_barrier<0>();                       // B1: X(t+1) landed; M(t-1) written
      STAMP(t, 0);
"""),
    ("""          if (bd_dma_slot(n) >= 0) dma_piece(t + 2, bd_dma_slot(n));
          __builtin_amdgcn_sched_barrier(0);
        }
""", """          if (bd_dma_slot(n) >= 0) dma_piece(t + 2, bd_dma_slot(n));
          __builtin_amdgcn_sched_barrier(0);
        }
        STAMP(t, 1);
"""),
    ("""    ring_barrier<0>();                 // B1: X(t+1) landed everywhere
    sp_load(t + 1, spn, mn);""", """    ring_barrier<0>();                 // B1: X(t+1) landed everywhere
    STAMP(t, 0);
    sp_load(t + 1, spn, mn);"""),
    ("""    if (cnt < t + 1) lds_wait_ge(BD_CNT + 4 * wid, t + 1);
    asm volatile("" ::: "memory");""",
     """    STAMP(t, 1);
    if (cnt < t + 1) lds_wait_ge(BD_CNT + 4 * wid, t + 1);
    asm volatile("" ::: "memory");
    STAMP(t, 2);"""),
    ("""int tgfr_version(void) { return 510; }""",
     """int tgfr_version(void) { return 510; }
int tgfr_lab_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_st), sizeof(g_st), 0, hipMemcpyDeviceToHost);
}"""),
]
# per-stage s_memtime stamps of the T=64 backward (wr_bwd_wide2_kernel):
# stage head (after its barrier) / after G1 / before G3 / after G3
_WSTAMP_DECL = ("""constexpr int WPF = 4;      // wr_bwd_wide2_kernel's LDS operand prefetch distance (slots)""",
                """constexpr int WPF = 4;      // wr_bwd_wide2_kernel's LDS operand prefetch distance (slots)
__device__ unsigned long long g_wst[256 * 4 * 64 * 4];
#define WSTAMP(t, k) do { if (blockIdx.x < 256 && (t) < 64) \
  g_wst[((blockIdx.x * 4 + wid) * 64 + (t)) * 4 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)""")
_WSTAMPS = [
    _WSTAMP_DECL,
    ("""    const bool has_next = i + 1 < c1;
    const uint32_t nb = ((it + 1) & 1) * BUF;   // the next caption's slot""",
     """    const bool has_next = i + 1 < c1;
    WSTAMP(it, 0);
    const uint32_t nb = ((it + 1) & 1) * BUF;   // the next caption's slot"""),
    ("""    // ---- softmax over the 64 words (p = exp2(S'), bounded) and both backwards.""",
     """    WSTAMP(it, 1);
    // ---- softmax over the 64 words (p = exp2(S'), bounded) and both backwards."""),
    ("""      float rho = 0.f;
      uint32_t w2[8];""",
     """      float rho = 0.f;
      uint32_t w2[8];
      WSTAMP(it, 2);"""),
    ("""        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if (rt >= NRT) return;""", """        __builtin_amdgcn_sched_barrier(0);
      }
    }
    WSTAMP(it, 3);
  }
  if (rt >= NRT) return;"""),
    ("""int tgfr_version(void) { return 510; }""",
     """int tgfr_version(void) { return 510; }
int tgfr_lab_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wst), sizeof(g_wst), 0, hipMemcpyDeviceToHost);
}"""),
]
# per-pair-step s_memtime stamps of the T=64 forward (wr_fwd_res2_kernel):
# loop top / after GEMM1 / after the softmax sums / after the tile loop /
# after the epilogue barrier
_RSTAMP_DECL = ("""constexpr int RPF = 3;      // wr_fwd_res2_kernel's LDS operand prefetch distance (slots)""",
                """constexpr int RPF = 3;      // wr_fwd_res2_kernel's LDS operand prefetch distance (slots)
__device__ unsigned long long g_rst[256 * 4 * 64 * 8];
#define RSTAMP(t, k) do { if (blockIdx.x < 256 && (t) < 64) \
  g_rst[((blockIdx.x * 4 + wid) * 64 + (t)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)""")
_RSTAMPS = [
    _RSTAMP_DECL,
    ("""    const int tl = len_n - 32 * tt;              // valid words of this tile""",
     """    const int tl = len_n - 32 * tt;              // valid words of this tile
    RSTAMP(k, 0);"""),
    ("""    // ---- softmax over the caption's words, per region: max and sum over
    // both token tiles (partner wave = wid ^ 1)""", """    RSTAMP(k, 1);
    // ---- softmax over the caption's words, per region: max and sum over
    // both token tiles (partner wave = wid ^ 1)"""),
    ("""#pragma unroll
    for (int j = 0; j < NRT; ++j)
      sj[j] += lds_ldf(FR2_OFF_XS + ((wid ^ 1) * NRT + j) * 128 + lr * 4);""",
     """#pragma unroll
    for (int j = 0; j < NRT; ++j)
      sj[j] += lds_ldf(FR2_OFF_XS + ((wid ^ 1) * NRT + j) * 128 + lr * 4);
    RSTAMP(k, 2);"""),
    ("""    const float zr = rs16(zp, lr), nr = rs16(np, lr);
    if ((lr & 1) == 0) {
      const int t = acc_row(rs16_index(lr), h);
      lds_stf(tok + t * 4, zr);
      lds_stf(tok + 128 + t * 4, nr);
    }
    if (ATT && active && b + img_offset == i) {""",
     """    RSTAMP(k, 3);
    const float zr = rs16(zp, lr), nr = rs16(np, lr);
    if ((lr & 1) == 0) {
      const int t = acc_row(rs16_index(lr), h);
      lds_stf(tok + t * 4, zr);
      lds_stf(tok + 128 + t * 4, nr);
    }
    if (ATT && active && b + img_offset == i) {"""),
    ("""    ex += lds_ldf(FR2_OFF_XL + (wid ^ 1) * 4);
    // The stores are unconditional""", """    ex += lds_ldf(FR2_OFF_XL + (wid ^ 1) * 4);
    RSTAMP(k, 4);
    // The stores are unconditional"""),
    ("""int tgfr_version(void) { return 510; }""",
     """int tgfr_version(void) { return 510; }
int tgfr_lab_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rst), sizeof(g_rst), 0, hipMemcpyDeviceToHost);
}"""),
]
# per-caption s_memtime stamps of the T<=32 pipelined forward
# (wr_fwd_pipe_kernel): caption top / after the slot loop / before the stores / after
_PSTAMPS = [
    ("""constexpr float BIG_C = 10.f;""",
     """constexpr float BIG_C = 10.f;
__device__ unsigned long long g_pst[256 * 4 * 16 * 4];
#define PSTAMP(t, k) do { if (blockIdx.x < 256 && (t) < 16) \
  g_pst[((blockIdx.x * 4 + wid) * 16 + (t)) * 4 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)"""),
    ("""  auto caption = [&](auto bigc) {
    const int len = lens[i];""", """  auto caption = [&](auto bigc) {
    const int ci = (i - c0) / 4;
    PSTAMP(ci, 0);
    const int len = lens[i];"""),
    ("""    // ---- N per token: reduce-scatter over the region lanes -> LDS
    {
      const float nr = rs16(np, lr);""", """    PSTAMP(ci, 1);
    // ---- N per token: reduce-scatter over the region lanes -> LDS
    {
      const float nr = rs16(np, lr);"""),
    ("""    const float ex = half_sum(tvalid ? __expf(g2 * cosv) : 0.f);
    logits[(long long)b * ld_logits + i] = g3 * __logf(ex);""",
     """    const float ex = half_sum(tvalid ? __expf(g2 * cosv) : 0.f);
    PSTAMP(ci, 2);
    logits[(long long)b * ld_logits + i] = g3 * __logf(ex);"""),
    ("""    store_cq<MODE_BF16>(Chi, nullptr, pair, t, h, C);
    init = initn;""", """    store_cq<MODE_BF16>(Chi, nullptr, pair, t, h, C);
    PSTAMP(ci, 3);
    init = initn;"""),
    ("""int tgfr_version(void) { return 510; }""",
     """int tgfr_version(void) { return 510; }
int tgfr_lab_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_pst), sizeof(g_pst), 0, hipMemcpyDeviceToHost);
}"""),
]
VARIANTS = {
    "base": [],
    "pstamp": _PSTAMPS,
    "rstamp": _RSTAMPS,
    "wstamp": _WSTAMPS,
    "head": "HEAD",
    "stamp": _STAMPS,
    # ablations of the two-role backward (timing only: results are wrong)
    "nosm": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));""")],
    "nog3": [(_G3, """          asm volatile("" ::"v"(Mi[n & 3]), "v"(rd[n & 7]));""")],
    "nog1": [(_G1, """      asm volatile("" ::"v"(rd[n & 3]));""")],
    "nodma": [(_DMA, "")],
    # timing probes: the stored scores / the X images always from the chunk's
    # first caption (L2-resident: no HBM latency behind the loads)
    "spl2": [("""    const uint16_t* rec = spb + (long long)min(k, K - 1) * (NRT * SP_REC);""",
              """    const uint16_t* rec = spb;""")],
    "dmal2": [("""      const int kc = min(k, K - 1);
      const uint32_t base = (k % BD_NB) * BD_BUF;""", """      const int kc = 0;
      const uint32_t base = (k % BD_NB) * BD_BUF;""")],
    "skel": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));"""),
             (_G3, """          asm volatile("" ::"v"(Mi[n & 3]), "v"(rd[n & 7]));"""),
             (_G1, """      asm volatile("" ::"v"(rd[n & 3]));""")],
    "skel_nodma": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));"""),
                   (_G3, """          asm volatile("" ::"v"(Mi[n & 3]), "v"(rd[n & 7]));"""),
                   (_G1, """      asm volatile("" ::"v"(rd[n & 3]));"""), (_DMA, "")],
    "mfma_only": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));"""),
                  (_DMA, "")],
    "pf3_7": [("constexpr int BD_PF3 = 4;", "constexpr int BD_PF3 = 7;")],
    # the 64-token backward's LDS operand prefetch distance
    "wpf3": [("constexpr int WPF = 4;", "constexpr int WPF = 3;")],
    "wpf6": [("constexpr int WPF = 4;", "constexpr int WPF = 6;")],
    # the 64-token backward's phase-A window (slots a..a+31, 1/sum at a+32)
    "ph17": [("n >= 18 && n < 50", "n >= 17 && n < 49"),
             ("const int e = n - 18, uu", "const int e = n - 17, uu"),
             ("if (n == 50) {", "if (n == 49) {"),
             ("AX0 = 51", "AX0 = 50"),
             ("if (n == 46) f0b", "if (n == 45) f0b")],
    "ph16": [("n >= 18 && n < 50", "n >= 16 && n < 48"),
             ("const int e = n - 18, uu", "const int e = n - 16, uu"),
             ("if (n == 50) {", "if (n == 48) {"),
             ("AX0 = 51", "AX0 = 49"),
             ("if (n == 46) f0b", "if (n == 44) f0b")],
    "skel_l2": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));"""),
                (_G3, """          asm volatile("" ::"v"(Mi[n & 3]), "v"(rd[n & 7]));"""),
                (_G1, """      asm volatile("" ::"v"(rd[n & 3]));"""),
                ("""      const int kc = min(k, K - 1);
      const uint32_t base = (k % BD_NB) * BD_BUF;""", """      const int kc = 0;
      const uint32_t base = (k % BD_NB) * BD_BUF;""")],
    "skel_chat": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));"""),
                  (_G3, """          asm volatile("" ::"v"(Mi[n & 3]), "v"(rd[n & 7]));"""),
                  (_G1, """      asm volatile("" ::"v"(rd[n & 3]));"""),
                  ("""          if (bd_dma_slot(n) >= 0) dma_piece(t + 2, bd_dma_slot(n));""",
                   """          if (bd_dma_slot(n) >= 0 && (bd_dma_slot(n) % 4 >= 2 || bd_dma_slot(n) == 8)) dma_piece(t + 2, bd_dma_slot(n));""")],
    "skel_notr": [(_SM, """        asm volatile("" ::"v"(Q), "v"(spc[0].x), "v"(spc[1].x), "v"(mc));"""),
                  (_G3, """          asm volatile("" ::"v"(Mi[n & 3]));"""),
                  ("""          if (n + BD_PF3 < 32) rd[(n + BD_PF3) & 7] = g3_read(n + BD_PF3, x3);""", ""),
                  (_G1, """      asm volatile("" ::"v"(rd[n & 3]));""")],
    "fblead": [("      if (c == PB - 4 + 8 * g)", "      if (c == PB - 8 + 8 * g)")],
    "fblead2": [("      if (c == PB - 4 + 8 * g)", "      if (c == PB - 8 + 8 * g)"),
                ("      if (c == PC - 3 + 4 * g) {", "      if (c == PC - 4 + 4 * g) {")],
    "pf1_4": [("constexpr int BD_PF1 = 3; ", "constexpr int BD_PF1 = 4; "),
              ("    u32x4 rd[4];\n#pragma unroll\n    for (int n = 0; n < BD_PF1; ++n) rd[n] = g1_read(n, x1);",
               "    u32x4 rd[8];\n#pragma unroll\n    for (int n = 0; n < BD_PF1; ++n) rd[n] = g1_read(n, x1);"),
              ("      g1_mfma(n, rd[n & 3], Qn);\n      if (n + BD_PF1 < 16) rd[(n + BD_PF1) & 3] = g1_read(n + BD_PF1, x1);",
               "      g1_mfma(n, rd[n & 7], Qn);\n      if (n + BD_PF1 < 16) rd[(n + BD_PF1) & 7] = g1_read(n + BD_PF1, x1);")],
    # forward probes: one caption body only (big captions wrong: timing), no S' stores
    "fnobig": [("""    if (big_cur)
      caption(std::true_type{});
    else
      caption(std::false_type{});""", """    caption(std::false_type{});""")],
    "fnostore": [("""        *(uint4*)(spt + lane * 16 + (q & 8)) = make_uint4(spk[0], spk[1], spk[2], spk[3]);""",
                  """        asm volatile("" ::"v"(spk[0]), "v"(spk[1]), "v"(spk[2]), "v"(spk[3]));""")],
    "fnoboth": [("""    if (big_cur)
      caption(std::true_type{});
    else
      caption(std::false_type{});""", """    caption(std::false_type{});"""),
                ("""        *(uint4*)(spt + lane * 16 + (q & 8)) = make_uint4(spk[0], spk[1], spk[2], spk[3]);""",
                  """        asm volatile("" ::"v"(spk[0]), "v"(spk[1]), "v"(spk[2]), "v"(spk[3]));""")],
    "prio_s": [(_SWAVE, _SWAVE + "\n  __builtin_amdgcn_s_setprio(1);")],
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
    "opt1": ("tgfr_optim.hip", [("VEC_PER_BLOCK = 4 * THREADS;", "VEC_PER_BLOCK = 1 * THREADS;")]),
    # BatchNorm normalise: 32 channels per workgroup (512 workgroups) instead of 64
    "bnct32": ("tgfr_bn.hip", [("constexpr int BN_CT = 64;", "constexpr int BN_CT = 32;")]),
    # IMIM weight gradients: the workgroup budget of the row-slice split
    # (512 kept in round 4; 256 and 128 measured slower)
    "dw768": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, true);",
                                 "  dw_plan_n(rows, 4, NS, KS, 768, A, wsf, n_wg, true);")]),
    "dw1024": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, true);",
                                  "  dw_plan_n(rows, 4, NS, KS, 1024, A, wsf, n_wg, true);")]),
    "dw384": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, true);",
                                 "  dw_plan_n(rows, 4, NS, KS, 384, A, wsf, n_wg, true);")]),
    "dw256": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, true);",
                                 "  dw_plan_n(rows, 4, NS, KS, 256, A, wsf, n_wg, true);")]),
    # IMIM weight gradients with fp32 row-slice slabs (the pre-bf16-slab path)
    "dwf32slab": ("tgfr_tail.hip", [("  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, true);",
                                     "  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, false);")]),
    # the committed tail + LayerNorm sources (A/B of a work-tree change to both)
    "headtn": (("tgfr_tail.hip", "tgfr_norm.hip"), "HEAD"),
}


def build_variant(name, subs, fname="tgfr_wr.hip"):
    """fname: one source, or a tuple of sources when subs == "HEAD" (each
    taken at the committed revision)."""
    fnames = fname if isinstance(fname, tuple) else (fname,)
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for fn in fnames:
        if subs == "HEAD":      # the committed source, for A/B against the work tree
            src = subprocess.run(["git", "show", f"HEAD:text_guided_face_recognition_amd/csrc/{fn}"],
                                 cwd=ROOT, check=True, capture_output=True, text=True).stdout
        else:
            src = open(os.path.join(B.CSRC, fn)).read()
            for old, new in subs:
                if old not in src:
                    raise SystemExit(f"{name}: substitution not found: {old[:60]!r}")
                src = src.replace(old, new)
        stem = fn[:-4]
        vsrc = os.path.join(OUT, f"{stem}_{name}.hip")
        open(vsrc, "w").write(src)
        obj = os.path.join(OUT, f"{stem}_{name}.o")
        cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-gpu-rdc",
               "-Wno-unused-result", "-Wno-unused-value", "-I", B.CSRC,
               *B.FILE_FLAGS.get(fn, []), "-c", vsrc, "-o", obj]
        subprocess.run(cmd, check=True, capture_output=True)
        objs.append(obj)
    others = [os.path.join(B.OBJ_DIR, os.path.basename(s).replace(".hip", ".o"))
              for s in B.sources() if os.path.basename(s) not in fnames]
    lib = os.path.join(OUT, f"lib_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-fno-gpu-rdc",
                    "-o", lib, *objs, *others], check=True, capture_output=True)
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
