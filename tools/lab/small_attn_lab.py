"""Lab: phase ablation of the fused small attention (csrc/tgfr_attn.hip
attn_small_fwd / _bwd) at the FCFM shape (B = 256, HW = C' = C = 36).

    python tools/lab/small_attn_lab.py build     # CPU: tools/lab/build/small_<v>.so
    python tools/lab/small_attn_lab.py run       # GPU: times each variant

Each variant is the product source with one phase cut out by text
substitution (results are garbage; only the time matters)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "lab", "build")
SRC = os.path.join(ROOT, "text_guided_face_recognition_amd", "csrc", "tgfr_attn.hip")

VARIANTS = {
    "base": [],
    "noload": [("  small_load(ops);\n  __syncthreads();\n  small_product(sQ, lq, 1, sK",
                "  __syncthreads();\n  small_product(sQ, lq, 1, sK")],
    "noS": [("  small_product(sQ, lq, 1, sK, lq, 1, hw, hw, cq, 0,\n"
             "                [&](int i, int j, float v) { sP[i * lp + j] = v * scale; });\n", "")],
    "nosoft": [("  for (int i = threadIdx.x / 16; i < hw; i += SNT / 16) {\n    float* row = sP",
                "  for (int i = hw; i < hw; i += SNT / 16) {\n    float* row = sP")],
    "noPstore": [("  small_store(P + n * hw * hw, hw, sP, lp, hw, hw);\n", "")],
    "noPV": [("  small_product(sP, lp, 1, sV, 1, lv, hw, c, hw, 0,\n"
              "                [&](int i, int cc, float v) { o[i * sor + cc] = v; });\n", "")],
}


def build():
    from text_guided_face_recognition_amd import build as B
    os.makedirs(OUT, exist_ok=True)
    src0 = open(SRC).read()
    for name, subs in VARIANTS.items():
        src = src0
        for old, new in subs:
            if old not in src:
                raise SystemExit(f"{name}: substitution not found: {old[:60]!r}")
            src = src.replace(old, new)
        vsrc = os.path.join(OUT, f"small_{name}.hip")
        open(vsrc, "w").write(src)
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC",
                        "-fno-gpu-rdc", "-shared", "-I", B.CSRC, vsrc, "-o",
                        os.path.join(OUT, f"small_{name}.so")], check=True)
        print("built", name)


def run():
    import torch
    P_, L_, I_, F_ = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_float
    nb, hw, cq = 256, 36, 36
    x = torch.randn(nb, hw, 2 * cq, device="cuda")
    y = torch.randn(nb, hw, cq, device="cuda")
    o = torch.empty(nb, hw, cq, device="cuda")
    p = torch.empty(nb, hw, hw, device="cuda")
    do = torch.randn(nb, hw, cq, device="cuda")
    dx, dy = torch.empty_like(x), torch.empty_like(y)
    st = torch.cuda.current_stream().cuda_stream
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(OUT, f"small_{name}.so"))
        fn = lib.tgfr_attn_small_fwd
        fn.argtypes = [P_, L_, L_, P_, L_, L_, I_, I_, I_, I_, I_, I_, F_, P_, L_, L_, P_, P_]
        args = (x.data_ptr(), hw * 2 * cq, 2 * cq, y.data_ptr(), hw * cq, cq, nb, hw, cq, 0, cq,
                cq, 1 / 6.0, o.data_ptr(), hw * cq, cq, p.data_ptr(), st)
        for _ in range(20):
            assert fn(*args) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            fn(*args)
        e1.record()
        e1.synchronize()
        tf = e0.elapsed_time(e1) / 200 * 1000
        bw = lib.tgfr_attn_small_bwd
        bw.argtypes = [P_, L_, L_, P_, L_, L_, I_, I_, I_, I_, I_, I_, F_, P_, P_, L_, L_, P_, L_,
                       L_, P_, L_, L_, P_]
        bargs = (x.data_ptr(), hw * 2 * cq, 2 * cq, y.data_ptr(), hw * cq, cq, nb, hw, cq, 0, cq,
                 cq, 1 / 6.0, p.data_ptr(), do.data_ptr(), hw * cq, cq, dx.data_ptr(),
                 hw * 2 * cq, 2 * cq, dy.data_ptr(), hw * cq, cq, st)
        for _ in range(20):
            assert bw(*bargs) == 0
        e0.record()
        for _ in range(200):
            bw(*bargs)
        e1.record()
        e1.synchronize()
        tb = e0.elapsed_time(e1) / 200 * 1000
        print(f"{name:10s} fwd {tf:6.1f} us  bwd {tb:6.1f} us", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
