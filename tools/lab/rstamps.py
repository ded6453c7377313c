"""Lab (GPU): per-pair-step s_memtime stamps of the 64-token forward
(wr_fwd_res2_kernel, bounded; the "rstamp" variant of tools/lab/variants.py)
at B = 128 images x 512 captions, T = 62, fp16 (n_chunks = 2): median cycles
of GEMM1, the softmax sums (two barriers), the tile loop (E + GEMM2), the
epilogue (+ barrier) and the stores up to the next step.

    TGFR_LAB=1 TGFR_LIB=tools/lab/build/lib_rstamp.so python tools/lab/rstamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from text_guided_face_recognition_amd import _hip, kernels as K  # noqa: E402


def main(b=128, n_cap=512, nw=62, mode="fp16"):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2)
    w = unit(torch.randn(n_cap, nw, 256, device=dev))
    lens = torch.full((n_cap,), nw, dtype=torch.int32, device=dev)
    with torch.no_grad():
        for _ in range(3):
            K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode=mode, bounded=True)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 4 * 64 * 8, dtype=np.uint64)
    rc = _hip.lib().tgfr_lab_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    st = buf.reshape(256, 4, 64, 8).astype(np.int64)
    rows = {"gemm1": [], "softmax": [], "tiles": [], "epilogue": [], "stores": [], "step": []}
    for L in range(256):
        for wv in range(4):
            s = st[L, wv]
            for t in range(2, 62):
                rows["gemm1"].append(s[t, 1] - s[t, 0])
                rows["softmax"].append(s[t, 2] - s[t, 1])
                rows["tiles"].append(s[t, 3] - s[t, 2])
                rows["epilogue"].append(s[t, 4] - s[t, 3])
                rows["stores"].append(s[t + 1, 0] - s[t, 4])
                rows["step"].append(s[t + 1, 0] - s[t, 0])
    out = {k: {"median": float(np.median(v)), "p10": float(np.percentile(v, 10)),
               "p90": float(np.percentile(v, 90))} for k, v in rows.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
