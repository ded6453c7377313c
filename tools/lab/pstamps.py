"""Lab (GPU): per-caption s_memtime stamps of the pipelined T <= 32 forward
(wr_fwd_pipe_kernel; the "pstamp" variant of tools/lab/variants.py) at
config 2 (B = 64, T = 30, bf16): median cycles of the 238-slot loop, the
epilogue, the stores and the whole caption.

    TGFR_LAB=1 TGFR_LIB=tools/lab/build/lib_pstamp.so python tools/lab/pstamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from text_guided_face_recognition_amd import _hip, kernels as K  # noqa: E402


def main(b=64, nw=30):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2)
    w = unit(torch.randn(b, nw, 256, device=dev))
    lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
    with torch.no_grad():
        for _ in range(3):
            K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode="bf16", bounded=True)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 4 * 16 * 4, dtype=np.uint64)
    rc = _hip.lib().tgfr_lab_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    st = buf.reshape(256, 4, 16, 4).astype(np.int64)
    rows = {"slots": [], "epilogue": [], "stores": [], "caption": []}
    for L in range(256):
        for wv in range(4):
            s = st[L, wv]
            for t in range(0, 3):
                if s[t + 1, 0] == 0:
                    continue
                rows["slots"].append(s[t, 1] - s[t, 0])
                rows["epilogue"].append(s[t, 2] - s[t, 1])
                rows["stores"].append(s[t, 3] - s[t, 2])
                rows["caption"].append(s[t + 1, 0] - s[t, 0])
    out = {k: {"median": float(np.median(v)), "p10": float(np.percentile(v, 10)),
               "p90": float(np.percentile(v, 90)), "n": len(v)} for k, v in rows.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
