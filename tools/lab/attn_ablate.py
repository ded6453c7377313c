"""Ablations of the fused attention forward / backward (tgfr_attn.hip):
variants by text substitution, each built into its own .so and timed with
HIP events at the IMIM shape (B=64, HW=196).  Usage: python
tools/lab/attn_ablate.py [variant ...]"""
import ctypes, os, subprocess, sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "text_guided_face_recognition_amd", "csrc", "tgfr_attn.hip")
BUILD = os.path.join(ROOT, "tools", "lab", "build")

VARIANTS = {
    "base": [],
    # forward: no MFMAs in the S phase / PV phase
    "f_nos": [("        sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(buf, s, lane), qf[s], sc[kt], 0, 0, 0);",
               "        sc[kt][s] += (float)frag(buf, s, lane)[0];")],
    "f_nopv": [("          oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[kt][s2], vb, oacc[dt], 0, 0, 0);",
                "          oacc[dt][s2] += (float)vb[0] + (float)pf[kt][s2][1];")],
    "f_nodma": [("    glds16(src, base + p * 1024);", "    if (n < 0) glds16(src, base + p * 1024);")],
    "f_nostore": [("      if (qq < hw) Ob[(long long)qq * ldo + 32 * dt + lr] = oacc[dt][r];",
                   "      if (qq < 0) Ob[(long long)qq * ldo + 32 * dt + lr] = oacc[dt][r];")],
    "f_empty": [("  const int nt = (hw + 31) / 32, np = (nt + 1) / 2;\n  // the workgroups of one sample run on one XCD (its Kr / V stay in that L2)",
                 "  if (hw > 0) return;\n  const int nt = (hw + 31) / 32, np = (nt + 1) / 2;\n  // the workgroups of one sample run on one XCD (its Kr / V stay in that L2)")],
    "f_smalllds": [("constexpr int FWD_NS = 7;", "constexpr int FWD_NS = 2;")],
    # s_memtime stamps into the lse buffer (wave 0 of each workgroup; every
    # lane stores its own copy with a vector store): [wg][16] int64
    "f_stamps": [
        ("  const uint32_t qimg = w * IMG, ring = 2 * IMG;\n  const int n_st = 2 * nt;",
         "  const uint32_t qimg = w * IMG, ring = 2 * IMG;\n  const int n_st = 2 * nt;\n"
         "  long long* stp = (long long*)lse + (long long)blockIdx.x * 24; int nst = 0;\n"
         "  auto STAMP = [&]() { long long t = __builtin_amdgcn_s_memtime(); if (w == 0 && lane == nst && nst < 24) stp[nst] = t; ++nst; };\n"
         "  STAMP();"),
        ("  wait(0);                                           // also covers the Qr tile",
         "  wait(0);                                           // also covers the Qr tile\n  STAMP();"),
        ("    if (kt > 0) {\n      wait(sk);", "    if (kt > 0) {\n      STAMP();\n      wait(sk);\n      STAMP();"),
        ("    wait(sk + 1);", "    STAMP();\n    wait(sk + 1);"),
        ("  l = xhalf_sum(l);\n  mfma_drain();", "  STAMP();\n  l = xhalf_sum(l);\n  mfma_drain();"),
        ("  if (h == 0) lse[(long long)b * hw + q] = m * scale + __logf(l);", "  if (h == 0 && lse == nullptr) lse[0] = m;"),
    ],
    "f_noexp": [("      sc[kt][r] = exp2f((sc[kt][r] - m) * c);", "      sc[kt][r] = (sc[kt][r] - m) * c;")],
}


def build(name):
    s = open(SRC).read()
    for a, b in VARIANTS[name]:
        assert a in s, (name, a[:70])
        s = s.replace(a, b)
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(BUILD, f"attn_{name}.hip")
    open(src, "w").write(s)
    so = os.path.join(BUILD, f"attn_{name}.so")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-shared", "-I", os.path.dirname(SRC), src, "-o", so])
    return so


def bench(so, nb=64, hw=196, reps=20):
    lib = ctypes.CDLL(so)
    P, L, I, F = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_float
    lib.tgfr_attn_fwd.argtypes = [P, P, P, L, L, I, I, F, P, L, L, P, P]
    lib.tgfr_attn_bwd.argtypes = [P, P, P, L, L, I, I, F, P, P, L, L, P, P, P, P, L, L, P, P]
    lib.tgfr_attn_bwd_ws.argtypes = [I, I, P]
    d = "cuda"
    px = torch.randn(nb, hw, 768, device=d).to(torch.bfloat16).view(torch.int16)
    o = torch.empty(nb, hw, 256, device=d)
    lse = torch.empty(nb * hw, device=d)
    do = torch.randn(nb, hw, 256, device=d)
    g = torch.empty(nb, hw, 768, device=d)
    out = (ctypes.c_longlong * 1)()
    lib.tgfr_attn_bwd_ws(nb, hw, ctypes.addressof(out))
    ws = torch.empty(int(out[0]), dtype=torch.uint8, device=d)
    st = torch.cuda.current_stream().cuda_stream
    q, k, v = px.data_ptr(), px[..., 256:].data_ptr(), px[..., 512:].data_ptr()

    def fwd():
        lib.tgfr_attn_fwd(q, k, v, 768, hw * 768, nb, hw, 0.0625, o.data_ptr(), 256, hw * 256,
                          lse.data_ptr(), st)

    def bwd():
        lib.tgfr_attn_bwd(q, k, v, 768, hw * 768, nb, hw, 0.0625, o.data_ptr(), do.data_ptr(),
                          256, hw * 256, lse.data_ptr(), g.data_ptr(), g[..., 256:].data_ptr(),
                          g[..., 512:].data_ptr(), 768, hw * 768, ws.data_ptr(), st)
    res = {}
    for nm, fn in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[nm] = round(e0.elapsed_time(e1) / reps * 1000, 1)
    return res


if __name__ == "__main__":
    args = sys.argv[1:] or list(VARIANTS)
    if args[0] == "stamps":
        so = build("f_stamps")
        bench(so, nb=64, reps=1)
        lib = ctypes.CDLL(so)
        # rerun once and read the stamps
        nb, hw = 64, 196
        P, L, I, F = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_float
        lib.tgfr_attn_fwd.argtypes = [P, P, P, L, L, I, I, F, P, L, L, P, P]
        px = torch.randn(nb, hw, 768, device="cuda").to(torch.bfloat16).view(torch.int16)
        o = torch.empty(nb, hw, 256, device="cuda")
        lse = torch.zeros(nb * hw * 4, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        lib.tgfr_attn_fwd(px.data_ptr(), px[..., 256:].data_ptr(), px[..., 512:].data_ptr(), 768,
                          hw * 768, nb, hw, 0.0625, o.data_ptr(), 256, hw * 256, lse.data_ptr(), st)
        torch.cuda.synchronize()
        t = lse.view(torch.int64)[:256 * 24].view(256, 24).cpu()
        d = (t[:, 1:20] - t[:, 0:19]).float()
        print("median deltas", [round(float(x)) for x in d.median(0).values])
        print("wg 1", [round(float(x)) for x in d[1]])
    elif args[0] == "sweep":
        so = build("base")
        for nb in (8, 16, 32, 64, 128):
            print("B", nb, bench(so, nb=nb), flush=True)
    else:
        for n in args:
            print(n, bench(build(n)), flush=True)
