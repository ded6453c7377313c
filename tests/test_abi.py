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
    assert lib.tgfr_version() == 610
    assert lib.tgfr_wr_lds_bytes(0) < 160 * 1024 and lib.tgfr_wr_lds_bytes(1) < 160 * 1024


def test_device_only_contract():
    """The product path refuses CPU tensors instead of falling back."""
    import pytest
    import torch
    from text_guided_face_recognition_amd import kernels as K
    with pytest.raises(RuntimeError):
        K.cos_logits(torch.randn(4, 256), torch.randn(4, 256), 10.0)
