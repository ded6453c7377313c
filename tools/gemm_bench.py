"""Time tgfr_bgemm on the step's GEMM shapes under each tile config
(TGFR_GEMM_CFG is read once per process, so each config runs in a child).

    python tools/gemm_bench.py            # all configs
"""
import json
import os
import subprocess
import sys

SHAPES = {
    # name: (batch, M, N, K, a_layout, b_layout)   row = k-contiguous A / n-contiguous B
    "qkv_fwd": (1, 12544, 768, 256, "row", "kmaj"),
    "qkv_dx": (1, 12544, 256, 768, "row", "row"),
    "qkv_dw": (1, 768, 256, 12544, "col", "row"),
    "conv1_fwd": (1, 12544, 128, 256, "row", "kmaj"),
    "attn_s": (64, 196, 196, 256, "row", "kmaj"),
    "attn_pv": (64, 196, 256, 196, "row", "row"),
    "attn_dv": (64, 196, 256, 196, "col", "row"),
}


def child(cfg):
    import torch
    sys.path.insert(0, ".")
    from text_guided_face_recognition_amd import kernels as K
    dev = torch.device("cuda")
    out = {}
    for name, (nb, m, n, k, la, lb) in SHAPES.items():
        a = torch.randn(nb, m, k, device=dev) if la == "row" else \
            torch.randn(nb, k, m, device=dev).transpose(1, 2)
        b = torch.randn(nb, k, n, device=dev) if lb == "row" else \
            torch.randn(nb, n, k, device=dev).transpose(1, 2)
        ks = K._ksplit(k, nb * -(-m // 64) * -(-n // 64)) if nb == 1 else 1
        for _ in range(3):
            K.bgemm(a, b, mode="bf16", ksplit=ks)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            K.bgemm(a, b, mode="bf16", ksplit=ks)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1000
        byts = 4 * nb * (m * k + k * n + m * n)
        out[name] = (round(us, 1), round(byts / us / 1e3, 2))
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    for cfg in ("auto", "0", "1", "2", "3"):
        env = dict(os.environ)
        if cfg != "auto":
            env["TGFR_GEMM_CFG"] = cfg
        r = subprocess.run([sys.executable, __file__, "--child", cfg], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        print(cfg, line[0] if line else r.stderr[-2000:], flush=True)
