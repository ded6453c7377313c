"""Lab: phase ablation of the identity heads' ArcMargin kernels
(csrc/tgfr_arc.hip: arc_fwd_kernel<128> via tgfr_arc_fwd_heads, and
arc_bwd_mma_kernel<2> via tgfr_arc_focal_bwd_heads) at the bench shape
(B = 64, D = 256, C = 4500, two heads).

    python tools/lab/arc_lab.py build     # CPU: tools/lab/build/arc_<v>.so
    python tools/lab/arc_lab.py run       # GPU: times each variant

Each variant is the product source with one change by text substitution,
linked with the product's other objects; ablated variants compute garbage
(only their time matters)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "lab", "build")
NAME = os.environ.get("LAB_FILE", "tgfr_arc.hip")

ALL_VARIANTS = {
    "base": [],
    "head": "HEAD",       # the committed source, for A/B against the work tree
    "fwd_nomma": [("    for (int k = k_lo; k < k_hi; k += 4) {", "    for (int k = k_lo; k < k_lo; k += 4) {")],
    "fwd_nosq": [("      for (int k = g; k < kc / 4; k += 16) {", "      for (int k = g; k < 0; k += 16) {")],
    "fwd_noepi": [("      if (r < nb && c0 + cc < C) {\n        const float cv = v * nx[r] * nw[cc];",
                   "      if (r < 0) {\n        const float cv = v * nx[r] * nw[cc];")],
    "fwd_fk256": [("  constexpr int fk = 128;\n  const int lds = ((CBF + FRB)",
                   "  constexpr int fk = 256;\n  const int lds = ((CBF + FRB)")],
    "bwd_nomma": [("    for (int k = 0; k < nb; k += 2) {", "    for (int k = 0; k < 0; k += 2) {")],
    "bwd_nodcs": [("          if (dcs) dcs[", "          if (false) dcs[")],
    "bwd_nodot": [("    for (int t = 0; t < NTW; ++t) sdot = fmaf(wr[32 * t], acc[t][q], sdot);\n",
                   "    for (int t = 0; t < 0; ++t) sdot = fmaf(wr[32 * t], acc[t][q], sdot);\n")],
    "sg_nolse": [("    for (int k = sub; k < n; k += 4) {\n      const int b = col ? k : j, i = col ? j : k;",
                  "    for (int k = sub; k < 0; k += 4) {\n      const int b = col ? k : j, i = col ? j : k;")],
    "sg_nocosv": [("  for (int e = tid; e < n * n; e += SG_T) cosv[e] = cs[(e / n) * (SG_N + 1) + e % n];",
                   "")],
    "sg_nocosasm": [("    cs[r * (SG_N + 1) + c] = v / fmaxf(sqrtf(nx) * sqrtf(ny), eps);",
                     "    cs[r * (SG_N + 1) + c] = v;")],
    "bwd_noepi": [("    for (int t = 0; t < NTW; ++t) o[32 * t] = (acc[t][q] - wr[32 * t] * inv * dot) * inv;",
                   "    for (int t = 0; t < NTW; ++t) o[32 * t] = acc[t][q];")],
}

VARIANTS = {k: v for k, v in ALL_VARIANTS.items()
            if k in os.environ.get("LAB_ONLY", ",".join(ALL_VARIANTS)).split(",")}

SG_CHILD = r'''
import ctypes, sys, torch
sys.path.insert(0, {root!r})
from text_guided_face_recognition_amd import _hip as H
lib = ctypes.CDLL({lib!r}, mode=ctypes.RTLD_GLOBAL)
for n, a in H.SIGNATURES.items():
    f = getattr(lib, n, None)
    if f is not None:
        f.argtypes = a; f.restype = ctypes.c_int
H._lib = lib
from text_guided_face_recognition_amd import kernels as K
torch.manual_seed(0)
x = torch.randn(64, 256, device="cuda", requires_grad=True)
y = torch.randn(64, 256, device="cuda")
cls = torch.randint(0, 40, (64,), device="cuda")
def step():
    a, b_, c = K.sent_global(x, y, cls, 10.0, 10.0)
    (a + b_ + 2 * c).backward()
for _ in range(3):
    step()
torch.cuda.synchronize()
with H.KernelTimer(replay=("tgfr_sent_global", "tgfr_sent_global_bwd"), reps=100) as kt:
    step()
f, g = kt.replayed["tgfr_sent_global"], kt.replayed["tgfr_sent_global_bwd"]
print(f"{name}: fwd {{f*1000:.1f}} us  bwd {{g*1000:.1f}} us  focal 0.0 us", flush=True)
'''

ATTN_CHILD = r'''
import ctypes, sys, torch
sys.path.insert(0, {root!r})
sys.path.insert(0, {root!r} + "/tests")
from text_guided_face_recognition_amd import _hip as H
lib = ctypes.CDLL({lib!r}, mode=ctypes.RTLD_GLOBAL)
for n, a in H.SIGNATURES.items():
    f = getattr(lib, n, None)
    if f is not None:
        f.argtypes = a; f.restype = ctypes.c_int
H._lib = lib
from test_gpu_attn import _attn
nb, hw = int({b!r}), 196
g = torch.Generator(device="cuda").manual_seed(0)
pxb = torch.randn(nb, hw, 768, generator=g, device="cuda").to(torch.bfloat16)
do = torch.randn(nb, hw, 256, generator=g, device="cuda")
for _ in range(3):
    _attn(pxb, do, 1 / 16)
torch.cuda.synchronize()
with H.KernelTimer(replay=("tgfr_attn_fwd", "tgfr_attn_bwd"), reps=100) as kt:
    _attn(pxb, do, 1 / 16)
f, g = kt.replayed["tgfr_attn_fwd"], kt.replayed["tgfr_attn_bwd"]
print(f"{name}: fwd {{f*1000:.1f}} us  bwd {{g*1000:.1f}} us  focal 0.0 us", flush=True)
'''

CHILD = r'''
import ctypes, sys, torch
sys.path.insert(0, {root!r})
from text_guided_face_recognition_amd import _hip as H
lib = ctypes.CDLL({lib!r}, mode=ctypes.RTLD_GLOBAL)
for n, a in H.SIGNATURES.items():
    f = getattr(lib, n, None)
    if f is not None:
        f.argtypes = a; f.restype = ctypes.c_int
H._lib = lib
from text_guided_face_recognition_amd import kernels as K
from text_guided_face_recognition_amd.models.metrics import ArcMarginProduct
dev = torch.device("cuda")
torch.manual_seed(0)
b, d, c = 64, 256, 4500
ht, hi = ArcMarginProduct(d, c).to(dev), ArcMarginProduct(d, c).to(dev)
xt = torch.randn(b, d, device=dev, requires_grad=True)
xi = torch.randn(b, d, device=dev, requires_grad=True)
lab = torch.randint(0, c, (b,), device=dev)
def step():
    lt, li = K.identity_heads(xt, ht, xi, hi, lab, 2.0)
    (lt + li).backward()
for _ in range(3):
    step()
torch.cuda.synchronize()
with H.KernelTimer(replay=("tgfr_arc_fwd_heads", "tgfr_arc_focal_bwd_heads", "tgfr_focal_ce2"),
                  reps=100) as kt:
    step()
f, g = kt.replayed["tgfr_arc_fwd_heads"], kt.replayed["tgfr_arc_focal_bwd_heads"]
fc = kt.replayed.get("tgfr_focal_ce2", 0.0)
print(f"{name}: fwd {{f*1000:.1f}} us  bwd {{g*1000:.1f}} us  focal {{fc*1000:.1f}} us", flush=True)
'''


def build():
    from text_guided_face_recognition_amd import build as B
    B.build()
    os.makedirs(OUT, exist_ok=True)
    src0 = open(os.path.join(B.CSRC, NAME)).read()
    others = [os.path.join(B.OBJ_DIR, os.path.basename(s).replace(".hip", ".o"))
              for s in B.sources() if not s.endswith(NAME)]
    for name, subs in VARIANTS.items():
        src = src0
        if subs == "HEAD":
            src = subprocess.run(["git", "show", f"HEAD:text_guided_face_recognition_amd/csrc/{NAME}"],
                                 cwd=ROOT, check=True, capture_output=True, text=True).stdout
            subs = []
        for old, new in subs:
            if old not in src:
                raise SystemExit(f"{name}: substitution not found: {old[:60]!r}")
            src = src.replace(old, new)
        vsrc = os.path.join(OUT, f"arc_{name}.hip")
        open(vsrc, "w").write(src)
        obj = vsrc[:-4] + ".o"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC",
                        "-fno-gpu-rdc", "-I", B.CSRC, *B.FILE_FLAGS.get(NAME, []), "-c", vsrc,
                        "-o", obj], check=True)
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-fno-gpu-rdc",
                        "-o", os.path.join(OUT, f"arc_{name}.so"), obj, *others], check=True)
        print("built", name, flush=True)


def run():
    rounds = int(os.environ.get("LAB_ROUNDS", "2"))
    times = {}
    for _ in range(rounds):
        for name in VARIANTS:
            lib = os.path.join(OUT, f"arc_{name}.so")
            if os.environ.get("LAB_CASE") == "sg":
                code = SG_CHILD.format(root=ROOT, lib=lib, name=name)
            elif os.environ.get("LAB_CASE") == "attn":
                code = ATTN_CHILD.format(root=ROOT, lib=lib, name=name,
                                         b=os.environ.get("LAB_B", "64"))
            else:
                code = CHILD.format(root=ROOT, lib=lib, name=name)
            res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                                 timeout=300)
            sys.stdout.write(res.stdout)
            if res.returncode:
                sys.stdout.write(res.stderr[-1500:])
                continue
            m = re.search(r"fwd ([\d.]+) us  bwd ([\d.]+) us  focal ([\d.]+) us", res.stdout)
            times.setdefault(name, []).append(tuple(float(m.group(k)) for k in (1, 2, 3)))
    for name, ts in times.items():
        print(f"SUMMARY {name:10s} fwd min {min(t[0] for t in ts):6.1f}  "
              f"bwd min {min(t[1] for t in ts):6.1f}  focal min {min(t[2] for t in ts):6.1f} us")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
