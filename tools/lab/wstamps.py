"""Lab (GPU): per-stage s_memtime stamps of the 64-token bounded backward
(wr_bwd_wide2_kernel; the "wstamp" variant of tools/lab/variants.py) at the
configs[4] caption length (B = 128, T = 62, fp16): median cycles per caption
stage of G1, the softmax, G3 and the barrier wait.

    TGFR_LAB=1 TGFR_LIB=tools/lab/build/lib_wstamp.so python tools/lab/wstamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from text_guided_face_recognition_amd import _hip, kernels as K  # noqa: E402


def main(b=128, nw=62, mode="fp16"):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2).requires_grad_()
    w = unit(torch.randn(b, nw, 256, device=dev))
    lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
    for _ in range(4):
        r.grad = None
        logits = K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode=mode, bounded=True)
        logits.sum().backward()
    torch.cuda.synchronize()
    buf = np.zeros(256 * 4 * 64 * 4, dtype=np.uint64)
    rc = _hip.lib().tgfr_lab_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    st = buf.reshape(256, 4, 64, 4).astype(np.int64)
    rows = {"G1": [], "softmax": [], "G3": [], "wait": [], "stage": []}
    for L in range(256):
        for wv in range(4):
            s = st[L, wv]
            for t in range(2, 62):
                rows["G1"].append(s[t, 1] - s[t, 0])
                rows["softmax"].append(s[t, 2] - s[t, 1])
                rows["G3"].append(s[t, 3] - s[t, 2])
                rows["wait"].append(s[t + 1, 0] - s[t, 3])
                rows["stage"].append(s[t + 1, 0] - s[t, 0])
    out = {k: {"median": float(np.median(v)), "p10": float(np.percentile(v, 10)),
               "p90": float(np.percentile(v, 90))} for k, v in rows.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
