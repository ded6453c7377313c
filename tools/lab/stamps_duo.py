"""Lab (GPU): per-stage timeline of wr_bwd_duo_kernel from the 'stamps'
variant (tools/lab/variants.py): s_memtime after barrier B1, after the
stage's work, after barrier B2, for stages 8..23 of every wave.  Prints the
median work / wait split of S waves and M waves (live region tiles only)."""
import ctypes
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from text_guided_face_recognition_amd import _hip as H  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", "build", "lib_stamps.so"),
                  mode=ctypes.RTLD_GLOBAL)
for n, a in H.SIGNATURES.items():
    f = getattr(lib, n, None)
    if f is not None:
        f.argtypes = a
        f.restype = ctypes.c_int
H._lib = lib
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
b, nw = 64, 30
torch.manual_seed(0)
unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2).requires_grad_()
w = unit(torch.randn(b, nw, 256, device=dev))
lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
labels = torch.arange(b, device=dev)
for _ in range(5):
    r.grad = None
    lg = K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode="bf16", bounded=True)
    (F.cross_entropy(lg, labels) + F.cross_entropy(lg.t(), labels)).backward()
torch.cuda.synchronize()
n = 512 * 8 * 16 * 4
buf = np.zeros(n, dtype=np.uint64)
rc = lib.tgfr_lab_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes))
assert rc == 0, rc
st = buf.reshape(512, 8, 16, 4).astype(np.int64)
n_chunks = 2
grid = n_chunks * 2 * b
st = st[:grid]
# live tiles: workgroup work index -> tg; tile 7 (tg 1, wave 3 / 7) is padding
live = []
for blk in range(grid):
    q, rr, x = grid // 8, grid % 8, blk % 8
    work = (x * (q + 1) if x < rr else rr * (q + 1) + (x - rr) * q) + blk // 8
    tg = (work % (2 * n_chunks)) // n_chunks
    live.append(tg)
live = np.array(live)
for role, waves in (("S", range(0, 4)), ("M", range(4, 8))):
    rows = []
    for blk in range(grid):
        for wv in waves:
            if live[blk] == 1 and wv % 4 == 3:
                continue
            s = st[blk, wv]
            if (s[:, 0] == 0).any():
                continue
            work = s[:, 1] - s[:, 0]
            b2 = s[:, 2] - s[:, 1]
            b1 = s[1:, 0] - s[:-1, 2]
            per = s[1:, 0] - s[:-1, 0]
            rows.append((np.median(work), np.median(b2), np.median(b1), np.median(per)))
    a = np.array(rows)
    print(f"{role} waves ({len(rows)}): median cycles per stage: work {np.median(a[:, 0]):.0f}  "
          f"B2 wait {np.median(a[:, 1]):.0f}  B1 wait {np.median(a[:, 2]):.0f}  "
          f"stage {np.median(a[:, 3]):.0f}  (p10/p90 stage {np.percentile(a[:, 3], 10):.0f}/"
          f"{np.percentile(a[:, 3], 90):.0f})")
