"""Lab (not product): variants of tgfr_bn_qkv_bf16 by text substitution on
csrc/tgfr_bn.hip, each built as its own small library (that file alone), and
(on a GPU box) the kernel timed alone per variant with HIP events.

    python tools/lab/qkv_lab.py build        # here
    python tools/lab/qkv_lab.py time         # GPU box
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "text_guided_face_recognition_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "lab", "build", "qkv")

VARIANTS = {
    "base": [],
    "nox": [("    if (ck % n_sl == sl) {", "    if (false) {")],
    "nostore": [("    *(uint4*)(dst + (long long)m * O + 8 * j) = lds_ld16(QKV_OUT + m * QKV_OP + 16 * j);",
                 "    if (m > 100000) *(uint4*)(dst + (long long)m * O + 8 * j) = lds_ld16(QKV_OUT + m * QKV_OP + 16 * j);")],
}


def build():
    os.makedirs(OUT, exist_ok=True)
    src = open(os.path.join(CSRC, "tgfr_bn.hip")).read()
    procs = []
    for name, subs in VARIANTS.items():
        s = src
        for a, b in subs:
            assert a in s, (name, a)
            s = s.replace(a, b)
        path = os.path.join(OUT, f"bn_{name}.hip")
        open(path, "w").write(s)
        so = os.path.join(OUT, f"libqkv_{name}.so")
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3",
                                       "-std=c++17", "-fPIC", "-shared", "-I", CSRC, path,
                                       "-o", so]))
    assert all(p.wait() == 0 for p in procs)


def time_all():
    import torch
    dev = torch.device("cuda")
    n, c, hw, o = 64, 256, 196, 768
    x = torch.randn(n, c, hw, device=dev)
    mean = x.mean((0, 2)).contiguous()
    rstd = (x.var((0, 2)) + 1e-5).rsqrt().contiguous()
    wb = (torch.randn(o, c, device=dev) / 16).to(torch.bfloat16).view(torch.int16)
    bf = torch.randn(o, device=dev)
    px = torch.empty(n * hw, o, dtype=torch.int16, device=dev)
    xh = torch.empty(n, hw, c, dtype=torch.int16, device=dev)
    P = ctypes.c_void_p
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(OUT, f"libqkv_{name}.so"))
        f = lib.tgfr_bn_qkv_bf16
        f.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int, P, P, P]
        args = [P(x.data_ptr()), n, c, hw, P(mean.data_ptr()), P(rstd.data_ptr()),
                P(wb.data_ptr()), P(bf.data_ptr()), o, P(px.data_ptr()), P(xh.data_ptr()),
                P(torch.cuda.current_stream().cuda_stream)]
        for _ in range(5):
            assert f(*args) == 0
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(50):
            f(*args)
        e.record()
        torch.cuda.synchronize()
        print(f"{name}: {s.elapsed_time(e) / 50 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else time_all()
