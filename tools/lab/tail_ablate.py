"""Ablations of the fused IMIM tail kernels: each variant of tgfr_tail.hip
(text substitution) is built into its own small .so and timed with HIP events
over back-to-back launches at the step's shape (12544 rows).
Usage (GPU box): python tools/lab/tail_ablate.py [variant ...]"""
import ctypes, os, subprocess, sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "text_guided_face_recognition_amd", "csrc", "tgfr_tail.hip")
BUILD = os.path.join(ROOT, "tools", "lab", "build")

VARIANTS = {
    "base": [],
    "noR": [("        o[0] = acc[mt][0][q] * iv;\n        o[32] = acc[mt][1][q] * iv;",
             "        if (iv == 12345.f) { o[0] = acc[mt][0][q]; o[32] = acc[mt][1][q]; }")],
    "nocopy": [("  copy_out<TH>(F_H1, H1b, TH, row0, rows, tid);\n", ""),
               ("  copy_out<TC>(F_H2, H2b, TC, row0, rows, tid);\n", "")],
    "noZb": [("      *(uint4*)(Zb + (long long)(row0 + m) * TC + 8 * c) = v;\n", "")],
    "l1only": [("  copy_out<TH>(F_H1, H1b, TH, row0, rows, tid);\n",
                "  copy_out<TH>(F_H1, H1b, TH, row0, rows, tid);\n  if (rows > 0) return;\n")],
    "zonly": [("  __syncthreads();\n\n  // layer 1, transposed", "  if (rows > 0) return;\n  __syncthreads();\n\n  // layer 1, transposed")],
    "now": [("w1f[s] = gld16(frag_ptr(pk, OFF_W1, TC, w, s, lane));",
             "w1f[s] = as_bf8(make_uint4(s, lr, h, w));"),
            ("w2f[s][jt] = gld16(frag_ptr(pk, OFF_W2, TH, 2 * w + jt, s, lane));",
             "w2f[s][jt] = as_bf8(make_uint4(s, lr, jt, w));"),
            ("wpf[s][nt] = gld16(frag_ptr(pk, OFF_WP, TC, 2 * w + nt, s, lane));",
             "wpf[s][nt] = as_bf8(make_uint4(s, lr, nt, h));")],
    # weight fragments loaded at each use instead of prefetched per layer
    # (fewer VGPRs: two waves per SIMD)
    "nopf": [
        ("""  bf16x8 w1f[TC / 16], w2f[TH / 16][2];
#pragma unroll
  for (int s = 0; s < TC / 16; ++s) w1f[s] = gld16(frag_ptr(pk, OFF_W1, TC, w, s, lane));
#pragma unroll
  for (int s = 0; s < TH / 16; ++s)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
      w2f[s][jt] = gld16(frag_ptr(pk, OFF_W2, TH, 2 * w + jt, s, lane));
""", ""),
        ("w1f[s]", "gld16(frag_ptr(pk, OFF_W1, TC, w, s, lane))"),
        ("w2f[s][jt]", "gld16(frag_ptr(pk, OFF_W2, TH, 2 * w + jt, s, lane))"),
        ("""  bf16x8 wpf[TC / 16][2];
#pragma unroll
  for (int s = 0; s < TC / 16; ++s)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      wpf[s][nt] = gld16(frag_ptr(pk, OFF_WP, TC, 2 * w + nt, s, lane));
""", ""),
        ("wpf[s][nt]", "gld16(frag_ptr(pk, OFF_WP, TC, 2 * w + nt, s, lane))"),
        ("""  bf16x8 wptf[TD / 16][2], w2tf[TC / 16];
#pragma unroll
  for (int s = 0; s < TD / 16; ++s)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
      wptf[s][jt] = gld16(frag_ptr(pk, OFF_WPT, TD, 2 * w + jt, s, lane));
#pragma unroll
  for (int s = 0; s < TC / 16; ++s)
    w2tf[s] = gld16(frag_ptr(pk, OFF_W2T, TC, w, s, lane));
""", ""),
        ("wptf[s][jt]", "gld16(frag_ptr(pk, OFF_WPT, TD, 2 * w + jt, s, lane))"),
        ("w2tf[s]", "gld16(frag_ptr(pk, OFF_W2T, TC, w, s, lane))"),
        ("""  bf16x8 w1tf[TH / 16][2];
#pragma unroll
  for (int s = 0; s < TH / 16; ++s)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      w1tf[s][ct] = gld16(frag_ptr(pk, OFF_W1T, TH, 2 * w + ct, s, lane));
""", ""),
        ("w1tf[s][ct]", "gld16(frag_ptr(pk, OFF_W1T, TH, 2 * w + ct, s, lane))"),
    ],
    "bwd_nocopy": [("  copy_out<TC>(B_DH2, dH2b, TC, row0, rows, tid);\n", ""),
                   ("  copy_out<TH>(B_DH1, dH1b, TH, row0, rows, tid);\n", "")],
    "bwd_nodz": [("        o[0] = acc[mt][0][q];\n        o[32] = acc[mt][1][q];",
                  "        if (acc[mt][0][q] == 12345.f) { o[0] = 1.f; o[32] = 1.f; }")],
}


def build(name):
    s = open(SRC).read()
    for a, b in VARIANTS[name]:
        assert a in s, (name, a[:60])
        s = s.replace(a, b)
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(BUILD, f"tail_{name}.hip")
    open(src, "w").write(s)
    so = os.path.join(BUILD, f"tail_{name}.so")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-shared", "-I", os.path.dirname(SRC), src, "-o", so])
    return so


def bench(so, rows=12544, reps=20):
    lib = ctypes.CDLL(so)
    P, L, I, F = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_float
    lib.tgfr_tail_fwd.argtypes = [P, L, I, P, P, P, P, F, P, L, P, P, P, P, P, P, I, I, I, P]
    lib.tgfr_tail_bwd.argtypes = [P, L, P, L, P, I, F, P, P, P, P, L, P, P, P, P]
    lib.tgfr_tail_pack.argtypes = [P, P, P, P, P]
    d = "cuda"
    z = torch.randn(rows, 256, device=d)
    w1, w2, wp = (torch.randn(*s, device=d) * .06 for s in ((128, 256), (256, 128), (256, 256)))
    b1, b2, bp = torch.zeros(128, device=d), torch.zeros(256, device=d), torch.zeros(256, device=d)
    pk = torch.empty(lib.tgfr_tail_pack_elems(), dtype=torch.int16, device=d)
    st = torch.cuda.current_stream().cuda_stream
    lib.tgfr_tail_pack(w1.data_ptr(), w2.data_ptr(), wp.data_ptr(), pk.data_ptr(), st)
    r = torch.empty(rows, 256, device=d)
    inv = torch.empty(rows, device=d)
    zb, h1, h2 = (torch.empty(rows, n, dtype=torch.int16, device=d) for n in (256, 128, 256))
    dz = torch.empty(rows, 256, device=d)
    dp, dh2, dh1 = (torch.empty(rows, n, dtype=torch.int16, device=d) for n in (256, 256, 128))
    dr = torch.randn(rows, 256, device=d)

    def fwd():
        lib.tgfr_tail_fwd(z.data_ptr(), 256, rows, pk.data_ptr(), b1.data_ptr(), b2.data_ptr(),
                          bp.data_ptr(), 1e-12, r.data_ptr(), 256, zb.data_ptr(), h1.data_ptr(),
                          h2.data_ptr(), inv.data_ptr(), None, None, 0, 0, 0, st)

    def bwd():
        lib.tgfr_tail_bwd(dr.data_ptr(), 256, r.data_ptr(), 256, inv.data_ptr(), rows, 1e-12,
                          pk.data_ptr(), h1.data_ptr(), h2.data_ptr(), dz.data_ptr(), 256,
                          dp.data_ptr(), dh2.data_ptr(), dh1.data_ptr(), st)
    out = {}
    for nm, fn in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[nm] = round(e0.elapsed_time(e1) / reps * 1000, 1)
    return out


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        print(n, bench(build(n)), flush=True)
