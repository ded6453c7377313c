"""Lab (GPU): per-stage s_memtime stamps of the two-role word<->region
backward (the "stamp" variant of tools/lab/variants.py) at config 2
(B = 64, T = 30, bf16): median cycles per stage of each role's segments.

    TGFR_LAB=1 TGFR_LIB=tools/lab/build/lib_stamp.so python tools/lab/stamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from text_guided_face_recognition_amd import _hip, kernels as K  # noqa: E402


def xcd_remap(L, total):
    q, r, x, s = total // 8, total % 8, L % 8, L // 8
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + s


def main(b=64, nw=30):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2).requires_grad_()
    w = unit(torch.randn(b, nw, 256, device=dev))
    lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
    for _ in range(4):
        r.grad = None
        logits = K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode="bf16", bounded=True)
        logits.sum().backward()
    torch.cuda.synchronize()
    buf = np.zeros(256 * 8 * 64 * 4, dtype=np.uint64)
    rc = _hip.lib().tgfr_lab_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    st = buf.reshape(256, 8, 64, 4).astype(np.int64)
    n_chunks, K_ = 2, 32
    T2 = (K_ + 2) & ~1
    rows = {"S_loop": [], "S_wait": [], "S_tail": [], "S_stage": [], "M_g3": [], "M_idle": [],
            "M_stage": []}
    for L in range(256):
        work = xcd_remap(L, n_chunks * 2 * b)
        tg = (work % (2 * n_chunks)) // n_chunks
        if tg != 0:
            continue
        for wv in range(4):
            s = st[L, wv]
            for t in range(1, T2 - 1):
                rows["S_loop"].append(s[t, 1] - s[t, 0])
                rows["S_wait"].append(s[t, 2] - s[t, 1])
                rows["S_tail"].append(s[t + 1, 0] - s[t, 2])
                rows["S_stage"].append(s[t + 1, 0] - s[t, 0])
            m = st[L, wv + 4]
            for t in range(1, T2 - 1):
                rows["M_g3"].append(m[t, 1] - m[t, 0])
                rows["M_idle"].append(m[t + 1, 0] - m[t, 1])
                rows["M_stage"].append(m[t + 1, 0] - m[t, 0])
    out = {k: {"median": float(np.median(v)), "p10": float(np.percentile(v, 10)),
               "p90": float(np.percentile(v, 90))} for k, v in rows.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
