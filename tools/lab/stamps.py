"""Lab (GPU): phase breakdown of the unit backward from the 'stamps' variant
(tools/lab/variants.py): per wave, cycles in the segment prologues, the
pipelined stages (per stage), the flushes and the final reductions."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from text_guided_face_recognition_amd import _hip as H  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools/lab/build/lib_stamps.so"), mode=ctypes.RTLD_GLOBAL)
for n, a in H.SIGNATURES.items():
    f = getattr(lib, n, None)
    if f is not None:
        f.argtypes = a
        f.restype = ctypes.c_int
H._lib = lib
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

L2E = 1.4426950408889634


def main(b=64, nw=30):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    r = unit(torch.randn(b, 196, 256, device=dev))
    w = unit(torch.randn(b, nw, 256, device=dev))
    lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
    r_hi, _, r_norm = K.prep_rows(r, K.NREG, K.RPAD, want_norms=True)
    w_hi, _, w_norm = K.prep_rows(w, nw, K.TPAD, lens=lens, want_norms=True, scale=L2E)
    logits = torch.empty(b, b, device=dev)
    stats = torch.empty(b, b, K.TPAD, 4, device=dev)
    c_hi = torch.empty(b, b, 32, K.TPAD, 8, dtype=torch.int16, device=dev)
    s = H.stream()
    K.call("tgfr_wr_fwd", K.ptr(r_hi), None, K.ptr(w_hi), None, K.ptr(w_norm), K.ptr(r_norm),
           K.ptr(lens), b, b, 0, 4.0, 5.0, 10.0, 1e-8, K.ptr(logits), b, K.ptr(stats),
           K.ptr(c_hi), None, None, 0, 1, K.TPAD, 0, s)
    dl = torch.randn(b, b, device=dev) * 0.01
    tok = torch.empty(b, b, K.TPAD, 8, device=dev)
    K.call("tgfr_wr_bwd_tok", K.ptr(stats), K.ptr(w_norm), K.ptr(r_norm), K.ptr(lens), b, b,
           4.0, 5.0, 10.0, 1e-8, K.ptr(dl), b, 1, K.TPAD, K.ptr(tok), s)
    nws = K.wr_bwd_ws_floats(b, b, 1, K.TPAD, 0)
    ws = torch.zeros(nws, device=dev)
    dR = torch.empty(b, 196, 256, device=dev)
    for _ in range(3):
        K.call("tgfr_wr_bwd", K.ptr(r_hi), None, K.ptr(w_hi), None, b, b, 4.0, K.ptr(tok),
               K.ptr(c_hi), None, K.ptr(dR), 196 * 256, 256, 1, K.ptr(ws), 1,
               K.TPAD, 0, s)
    torch.cuda.synchronize()
    st = ws[-1024 * 16 * 2:].view(torch.int64).view(1024, 16).cpu().numpy().astype(np.float64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0]
    print(f"waves {len(st)}; kernel span {(st[:, 15].max() - t0.min()):.0f} cycles")
    print(f"start->segment loop {np.median(st[:, 1] - t0):.0f}")
    for sg in range(2):
        a, bst, c, kk, nxt = (st[:, 2 + 4 * sg - 1 if sg else 1], st[:, 2 + 4 * sg],
                             st[:, 3 + 4 * sg], st[:, 5 + 4 * sg], st[:, 4 + 4 * sg])
        ok = kk > 0
        if not ok.any():
            continue
        pro = (bst - (st[:, 1] if sg == 0 else st[:, 4]))[ok]
        stg = (c - bst)[ok]
        fl = (nxt - c)[ok]
        print(f"segment {sg}: waves {ok.sum()} K med {np.median(kk[ok]):.0f}  prologue "
              f"{np.median(pro):.0f}  stages {np.median(stg):.0f} "
              f"({np.median(stg / (kk[ok] + 1)):.0f}/stage)  flush {np.median(fl):.0f}")
    print(f"loop end -> kernel end {np.median(st[:, 15] - st[:, 14]):.0f} "
          f"(max {np.max(st[:, 15] - st[:, 14]):.0f})")
    tick = st[:, 13] - st[:, 14]
    red = st[:, 15] - st[:, 13]
    nred = st[:, 12]
    for k in range(int(nred.max()) + 1):
        sel = nred == k
        if sel.any():
            print(f"  n_red={k}: waves {sel.sum()}  ticket {np.median(tick[sel]):.0f} "
                  f"(max {tick[sel].max():.0f})  reduce {np.median(red[sel]):.0f} "
                  f"(max {red[sel].max():.0f})")
    order = np.argsort(-(st[:, 15] - st[:, 0]))[:6]
    for o in order:
        print("  slowest wave", o, "total", st[o, 15] - st[o, 0], "phases",
              np.diff(st[o, [0, 1, 2, 3, 4]]), "K0", st[o, 5], "n_red", st[o, 12])


if __name__ == "__main__":
    main()
