"""CPU checks of the C-ABI boundary: the library loads without a GPU and
exports every entry point include/tgfr.h declares, with the argument counts
the ctypes binding uses.  No kernel is launched."""
import os
import re
import subprocess

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tgfr.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\bint\s+(tgfr_\w+)\s*\(([^)]*)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


def test_header_declares_entry_points():
    decl = _declared()
    assert {"tgfr_wr_fwd", "tgfr_wr_bwd", "tgfr_cos_logits", "tgfr_ce_loss",
            "tgfr_bgemm", "tgfr_attn_softmax"} <= set(decl)


def test_library_exports_every_declared_symbol():
    from text_guided_face_recognition_amd import _hip
    from text_guided_face_recognition_amd.build import LIB, build
    build()
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (tgfr_\w+)", nm))
    decl = _declared()
    assert set(decl) <= exported, set(decl) - exported
    assert set(decl) == set(_hip.SIGNATURES), set(decl) ^ set(_hip.SIGNATURES)
    for name, n in decl.items():
        assert len(_hip.SIGNATURES[name]) == n, (name, n, len(_hip.SIGNATURES[name]))
    lib = _hip.lib()
    assert lib.tgfr_version() == 620
    assert lib.tgfr_wr_lds_bytes(0) < 160 * 1024 and lib.tgfr_wr_lds_bytes(1) < 160 * 1024


def test_device_only_contract():
    """The product path refuses CPU tensors instead of falling back."""
    import pytest
    import torch
    from text_guided_face_recognition_amd import kernels as K
    with pytest.raises(RuntimeError):
        K.cos_logits(torch.randn(4, 256), torch.randn(4, 256), 10.0)


def test_round6_argument_contracts():
    """The round-6 entry points' host-side contracts, checked without a GPU
    (each call returns before any launch): the sentence / global dist
    kernels take up to 128 rows per rank in 64-row tiles, one column-partial
    set per tile (tgfr_sent_global_dist_ws), and reject more; the deferred
    LayerNorm reduce (tgfr_imim_dw_ln) and the fused identity-head backward
    reject missing operands with 1001."""
    import ctypes
    from text_guided_face_recognition_amd import _hip
    lib = _hip.lib()
    out = (ctypes.c_longlong * 3)()
    a = [ctypes.addressof(out) + 8 * k for k in range(3)]
    for n_r, n_c, tiles in ((64, 512, 1), (65, 512, 2), (128, 1024, 2)):
        assert lib.tgfr_sent_global_dist_ws(n_r, n_c, *a) == 0
        assert out[1] == 4 * n_c * tiles, (n_r, out[1])
        assert out[0] == 2 * -(-n_c // 64) * n_r * 2
    assert lib.tgfr_sent_global_dist_ws(129, 1024, *a) == 1001
    nul = [None] * 25
    nul[6], nul[15], nul[16], nul[20] = 12544, 768, 256, 196       # rows, Nq, Kq, hw
    assert lib.tgfr_imim_dw_ln(*nul) == 1001
    assert lib.tgfr_arc_focal_bwd_heads(None, 2, 128, 256, 4500, 0.5, 0, 1e-12, 2.0, None) == 1001
