"""Ablations of the fused IMIM attention kernels (csrc/tgfr_attn.hip) at the
IMIM shape: variants by text substitution, each built on the GPU box into its
own .so under /tmp and timed with HIP events (forward, backward = prep + dK/dV
+ dQ).  Which phase of a latency-bound kernel holds its time shows as the
time a variant without it saves.
    python tools/attn_lab.py [variant ...]      (GPU box; 'sweep' = batch sweep)"""
import ctypes
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "text_guided_face_recognition_amd", "csrc", "tgfr_attn.hip")
BUILD = "/tmp/tgfr_attn_lab"

VARIANTS = {
    "base": [],
    # dK / dV: without the dV / dK MFMAs of each query tile
    "kv_nodkdv": [("        dv[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, obf, dv[t], 0, 0, 0);\n"
                   "        dk[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa, qbf, dk[t], 0, 0, 0);",
                   "        dv[t][0] += (float)obf[0] + (float)pa[1];\n"
                   "        dk[t][0] += (float)qbf[0] + (float)sa[1];")],
    # dK / dV: without the S / dP recompute MFMAs
    "kv_norecomp": [("      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(AI, s, lane), kf[s], acc0, 0, 0, 0);\n"
                     "      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(AI, s + 1, lane), kf[s + 1], acc1, 0,\n"
                     "                                                     0, 0);",
                     "      acc0[s] += (float)frag(AI, s, lane)[0] + (float)kf[s][1];\n"
                     "      acc1[s] += (float)frag(AI, s + 1, lane)[0] + (float)kf[s + 1][1];")],
    # dK / dV: without the dS stores
    "kv_nods": [("        if (qq < hw) dsb[(long long)qq * kp + key] = bf_bits(ds[r]);",
                 "        if (qq < 0) dsb[(long long)qq * kp + key] = bf_bits(ds[r]);")],
    # dK / dV: without the S / dP exchange barrier (wrong results, timing only)
    "kv_noxch": [("      __syncthreads();\n      f32x16 par;", "      f32x16 par;")],
    # forward: without the O^T += V^T P^T MFMAs
    "f_nopv": [("        oacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb[s2], oacc[t], 0, 0, 0);",
                "        oacc[t][0] += (float)va[0] + (float)pb[s2][1];")],
    # forward: without the S MFMAs
    "f_nos": [("      sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(kbuf, s, lane), qf[s], sc, 0, 0, 0);",
               "      sc[s] += (float)frag(kbuf, s, lane)[0] + (float)qf[s][1];")],
    # forward: every key tile read from stage 0 (wrong values): no DMA waits in the loop
    "f_nodmawait": [("      if (i + 1 < iters) {\n        ring_barrier<0>();\n        issue(i + 1);\n      } else {\n        ring_barrier<0>();\n      }",
                     "      __syncthreads();"),
                    ("  if (iters > 1) issue(1);\n", ""),
                    ("    const uint32_t kbuf = ring + (i & 1) * FWD_STAGE + (2 * half) * IMG, vbuf = kbuf + IMG;",
                     "    const uint32_t kbuf = ring + (2 * half) * IMG, vbuf = kbuf + IMG;")],
    # forward: without the O stores
    "f_nostore": [("      if (qv)\n        *(float4*)(orow + 32 * t + 8 * g + 4 * h) =",
                   "      if (q < 0)\n        *(float4*)(orow + 32 * t + 8 * g + 4 * h) =")],
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
    px = (torch.randn(nb, hw, 768, device=d) * 0.3).to(torch.bfloat16).view(torch.int16)
    o = torch.empty(nb, hw, 256, device=d)
    lse = torch.empty(nb * hw, device=d)
    do = torch.randn(nb, hw, 256, device=d)
    g = torch.empty(nb, hw, 768, dtype=torch.int16, device=d)
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
    if args[0] == "sweep":
        so = build("base")
        for nb in (8, 16, 32, 64, 128):
            print("B", nb, bench(so, nb=nb), flush=True)
    else:
        for n in args:
            print(n, bench(build(n)), flush=True)
