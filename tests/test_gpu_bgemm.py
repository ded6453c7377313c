"""bgemm (csrc/tgfr_attn.hip) against torch fp32 matmul for every operand
layout the kernel stages (k-contiguous, m/n-contiguous, strided gathers),
ragged tile edges, split-K, bias/ReLU/accumulate epilogues and both modes.
Tolerance: fp32 (split-bf16) 2e-5 x sqrt(K) relative to max |C|; bf16 1e-2."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _operand(rows, cols, lay, dev, gen):
    """[rows, cols] fp32 view with the requested unit-stride axis."""
    if lay == "row":                     # unit stride on cols
        return torch.randn(rows, cols, generator=gen).to(dev)
    if lay == "col":                     # unit stride on rows
        return torch.randn(cols, rows, generator=gen).to(dev).t()
    # neither axis unit-stride
    return torch.randn(rows, 2 * cols, generator=gen).to(dev)[:, ::2]


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
@pytest.mark.parametrize("la", ["row", "col", "any"])
@pytest.mark.parametrize("lb", ["row", "col", "any"])
def test_layouts(gpu, mode, la, lb):
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(11)
    m, n, k = 77, 130, 203                      # ragged in every dimension
    a = _operand(m, k, la, gpu, gen)
    b = _operand(k, n, lb, gpu, gen)
    c = K.bgemm(a.unsqueeze(0), b.unsqueeze(0), mode=mode)[0]
    ref = a.double() @ b.double()
    err = (c.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < (2e-5 if mode == "fp32" else 1e-2), err


@pytest.mark.parametrize("lay", ["row", "col"])
def test_split_k_and_batch(gpu, lay):
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(12)
    a = torch.stack([_operand(40, 3000, lay, gpu, gen) for _ in range(3)])
    b = torch.stack([_operand(3000, 96, lay, gpu, gen) for _ in range(3)])
    for ks in (1, 7, 13):
        c = K.bgemm(a, b, mode="fp32", ksplit=ks)
        ref = a.double() @ b.double()
        err = (c.double() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-5, (ks, err)


def test_epilogues(gpu):
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(13)
    a = _operand(65, 64, "col", gpu, gen).unsqueeze(0)
    b = _operand(64, 33, "row", gpu, gen).unsqueeze(0)
    bias = torch.randn(33, generator=gen).to(gpu)
    ref = torch.relu(0.5 * (a[0].double() @ b[0].double()) + bias.double())
    c = K.bgemm(a, b, alpha=0.5, bias=bias, relu=True)[0]
    torch.testing.assert_close(c.double(), ref, rtol=1e-4, atol=2e-4)
    acc = torch.randn(1, 65, 33, generator=gen).to(gpu)
    ref2 = acc[0].double() + a[0].double() @ b[0].double()
    K.bgemm(a, b, out=acc, accumulate=True)
    torch.testing.assert_close(acc[0].double(), ref2, rtol=1e-4, atol=2e-4)
    # transposed (column-major) output
    out = torch.empty(33, 65, device=gpu).t().unsqueeze(0)
    K.bgemm(a, b, out=out)
    torch.testing.assert_close(out[0].double(), a[0].double() @ b[0].double(),
                               rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
@pytest.mark.parametrize("shape", [
    (76, 132, 204, 1),        # ragged tiles, 64x64 DMA path
    (4100, 1028, 96, 1),      # 128x128 tiles
    (12548, 256, 68, 1),      # 128x64 tiles
    (196, 196, 256, 8),       # batched attention-like products
])
@pytest.mark.parametrize("la,lb", [("row", "col"), ("col", "row"), ("row", "row"),
                                   ("col", "col")])
def test_dma_path_configs(gpu, mode, shape, la, lb):
    """Shapes whose operands the DMA path fetches (16-B quads along the unit
    axis), across the tile configurations the launcher picks."""
    from text_guided_face_recognition_amd import kernels as K
    m, n, k, nb = shape
    gen = torch.Generator().manual_seed(14)
    a = torch.stack([_operand(m, k, la, gpu, gen) for _ in range(nb)])
    b = torch.stack([_operand(k, n, lb, gpu, gen) for _ in range(nb)])
    if la == "col":
        a = a.transpose(1, 2).contiguous().transpose(1, 2)
    if lb == "col":
        b = b.transpose(1, 2).contiguous().transpose(1, 2)
    c = K.bgemm(a, b, mode=mode)
    ref = a.double() @ b.double()
    err = (c.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < (2e-5 if mode == "fp32" else 1e-2), err


@pytest.mark.parametrize("m,n,k", [(12544, 768, 256), (12544, 128, 256), (12544, 256, 128),
                                   (4100, 200, 256), (2050, 64, 128), (3000, 130, 256)])
@pytest.mark.parametrize("lb", ["row", "col"])
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "accumulate"])
def test_weight_resident_path(gpu, m, n, k, lb, epi):
    """bf16 products with a tall k-contiguous A and K = 128 / 256 take the
    weight-resident row-stream kernel: ragged M and N, both B layouts (W[n][k]
    forward / W[k][n] dX), the epilogues, a row stride > K on A."""
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(m + n + k)
    a = torch.randn(m, k + 4, generator=gen).to(gpu)[:, :k]          # sAm = k + 4
    b = _operand(k, n, lb, gpu, gen)
    bias = torch.randn(n, generator=gen).to(gpu) if epi == "bias_relu" else None
    ref = 0.75 * (a.double() @ b.double())
    if epi == "bias_relu":
        ref = torch.relu(ref + bias.double())
    out = None
    if epi == "accumulate":
        out = torch.randn(1, m, n, generator=gen).to(gpu)
        ref = ref + out[0].double()
    c = K.bgemm(a.unsqueeze(0), b.unsqueeze(0), out=out, alpha=0.75, mode="bf16", bias=bias,
                relu=epi == "bias_relu", accumulate=epi == "accumulate")[0]
    err = (c.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
