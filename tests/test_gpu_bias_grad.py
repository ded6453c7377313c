"""tgfr_bias_grad (column sums of dy, optional ReLU mask) against torch fp32 /
fp64 sums: the float4 path (aligned, cols % 4 == 0) and the scalar path,
single and multi-block column groups, ragged row counts."""
import pytest
import torch

from text_guided_face_recognition_amd import _hip
from text_guided_face_recognition_amd._hip import call, ptr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols,relu,pad", [
    (12544, 256, False, 0), (12544, 768, False, 0), (12544, 256, True, 0),
    (12544, 128, True, 0), (1000, 300, True, 0), (77, 12, False, 0),
    (513, 65, True, 0), (300, 256, False, 3)])
def test_bias_grad(gpu, rows, cols, relu, pad):
    g = torch.Generator(device="cpu").manual_seed(rows + cols)
    dy_full = torch.randn(rows, cols + pad, generator=g).to(gpu)
    dy = dy_full[:, :cols]
    y = torch.randn(rows, cols, generator=g).to(gpu) if relu else None
    dym = torch.empty(rows, cols, device=gpu) if relu else None
    db = torch.empty(cols, device=gpu)
    ws = torch.empty(-(-rows // 128) * cols, device=gpu)
    call("tgfr_bias_grad", ptr(dy), dy.stride(0), rows, cols, ptr(y),
         y.stride(0) if relu else 0, ptr(dym), dym.stride(0) if relu else 0, ptr(db), ptr(ws),
         ptr(_hip.counters(gpu)), _hip.stream())
    ref_m = torch.where(y > 0, dy, torch.zeros_like(dy)) if relu else dy
    ref = ref_m.double().sum(0).float()
    assert torch.allclose(db, ref, rtol=1e-5, atol=1e-3), (db - ref).abs().max()
    if relu:
        assert torch.equal(dym, ref_m)
    # counters left zeroed: a second call gives the same bits
    db2 = torch.empty_like(db)
    call("tgfr_bias_grad", ptr(dy), dy.stride(0), rows, cols, ptr(y),
         y.stride(0) if relu else 0, ptr(dym), dym.stride(0) if relu else 0, ptr(db2), ptr(ws),
         ptr(_hip.counters(gpu)), _hip.stream())
    assert torch.equal(db, db2)
