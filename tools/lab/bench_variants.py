"""Lab (GPU): time the word<->region kernels of each tools/lab/build/lib_*.so
at B=64, T=30 bf16 (and check the backward against the product library on the
same inputs).  Each variant runs in its own process."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

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
import torch.nn.functional as F
dev = torch.device("cuda")
b, nw = {b}, 30
torch.manual_seed(0)
unit = lambda x: x / x.norm(dim=-1, keepdim=True)
r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2).requires_grad_()
w = unit(torch.randn(b, nw, 256, device=dev))
lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
labels = torch.arange(b, device=dev)
def step():
    lg = K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode="bf16", bounded=True)
    (F.cross_entropy(lg, labels) + F.cross_entropy(lg.t(), labels)).backward()
    return lg
for _ in range(3):
    r.grad = None; step()
torch.cuda.synchronize()
r.grad = None
lg = step()
torch.save((lg.detach().cpu(), r.grad.cpu()), {out!r})
with H.KernelTimer(replay=("tgfr_wr_fwd", "tgfr_wr_bwd"), reps=50) as kt:
    for _ in range(3):
        step()
fwd, bwd = kt.replayed["tgfr_wr_fwd"], kt.replayed["tgfr_wr_bwd"]
print(f"{name}: fwd {{fwd*1000:.1f}} us ({{4*196*256*nw*b*b/fwd/1e9:.0f}} TF)  "
      f"bwd {{bwd*1000:.1f}} us ({{6*196*256*nw*b*b/bwd/1e9:.0f}} TF)", flush=True)
'''


def main():
    """Each variant runs LAB_ROUNDS times, round-robin (box clocks drift by a
    few percent over a minute: interleaving keeps that out of the A/B)."""
    import re
    b = int(os.environ.get("LAB_B", "64"))
    rounds = int(os.environ.get("LAB_ROUNDS", "3"))
    libs = sorted(glob.glob(os.path.join(ROOT, "tools", "lab", "build", "lib_*.so")))
    outs, times = {}, {}
    for _ in range(rounds):
        for lib in libs:
            name = os.path.basename(lib)[4:-3]
            out = f"/tmp/lab_{name}.pt"
            code = CHILD.format(root=ROOT, lib=lib, b=b, out=out, name=name)
            res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                                 timeout=300)
            sys.stdout.write(res.stdout)
            sys.stdout.flush()
            if res.returncode != 0:
                sys.stdout.write(res.stderr[-2000:])
                continue
            outs[name] = out
            m = re.search(r"fwd ([\d.]+) us.*bwd ([\d.]+) us", res.stdout)
            if m:
                times.setdefault(name, []).append((float(m.group(1)), float(m.group(2))))
    for name, ts in sorted(times.items()):
        f = sorted(x[0] for x in ts)
        bw = sorted(x[1] for x in ts)
        print(f"SUMMARY {name}: fwd min {f[0]:.1f} med {f[len(f) // 2]:.1f} us | "
              f"bwd min {bw[0]:.1f} med {bw[len(bw) // 2]:.1f} us")
    import torch
    if "base" in outs:
        lg0, g0 = torch.load(outs["base"])
        for name, path in outs.items():
            lg, g = torch.load(path)
            print(f"{name}: logits vs base {(lg - lg0).abs().max():.2e}, "
                  f"grad vs base {((g - g0).abs().max() / g0.abs().max()):.2e}")


if __name__ == "__main__":
    main()
