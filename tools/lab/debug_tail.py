"""Intermediate errors of the fused IMIM tail against torch fp32."""
import torch
import torch.nn.functional as F
from text_guided_face_recognition_amd import kernels as K, _hip
from text_guided_face_recognition_amd._hip import call, ptr

def rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30))

def bf(t):  # int16 bf16 bits -> float
    return (t.to(torch.int32) << 16).view(torch.float32)

torch.manual_seed(0)
rows = 256
z = torch.randn(rows, 256, device="cuda")
w1, b1 = torch.randn(128, 256, device="cuda") * .0625, torch.randn(128, device="cuda") * .1
w2, b2 = torch.randn(256, 128, device="cuda") * .088, torch.randn(256, device="cuda") * .1
wp, bp = torch.randn(256, 256, device="cuda") * .0625, torch.randn(256, device="cuda") * .1
dr = torch.randn(rows, 256, device="cuda")
zz = z.clone().requires_grad_()
h1 = F.relu(zz @ w1.t() + b1); h1.retain_grad()
h2 = F.relu(h1 @ w2.t() + b2); h2.retain_grad()
p = h2 @ wp.t() + bp; p.retain_grad()
r = F.normalize(p, dim=-1)
r.backward(dr)
pk = torch.empty(_hip.lib().tgfr_tail_pack_elems(), dtype=torch.int16, device="cuda")
call("tgfr_tail_pack", ptr(w1), ptr(w2), ptr(wp), ptr(pk), _hip.stream())
R = torch.empty(rows, 256, device="cuda"); zb = torch.empty(rows, 256, dtype=torch.int16, device="cuda")
H1 = torch.empty(rows, 128, dtype=torch.int16, device="cuda"); H2 = torch.empty(rows, 256, dtype=torch.int16, device="cuda")
inv = torch.empty(rows, device="cuda")
call("tgfr_tail_fwd", ptr(z), 256, rows, ptr(pk), ptr(b1), ptr(b2), ptr(bp), 1e-12, ptr(R), 256, ptr(zb), ptr(H1), ptr(H2), ptr(inv), None, None, 0, 0, 0, _hip.stream())
print("zb", rel(bf(zb), z), "H1", rel(bf(H1), h1), "H2", rel(bf(H2), h2), "R", rel(R, r), "inv", rel(inv, 1/p.norm(dim=-1)))
dz = torch.empty(rows, 256, device="cuda"); dP = torch.empty(rows, 256, dtype=torch.int16, device="cuda")
dH2 = torch.empty(rows, 256, dtype=torch.int16, device="cuda"); dH1 = torch.empty(rows, 128, dtype=torch.int16, device="cuda")
call("tgfr_tail_bwd", ptr(dr), 256, ptr(R), 256, ptr(inv), rows, 1e-12, ptr(pk), ptr(H1), ptr(H2), ptr(dz), 256, ptr(dP), ptr(dH2), ptr(dH1), _hip.stream())
dh2m = h2.grad * 1  # grad wrt h2 (already masked? no: grad of h2 output)
print("dP", rel(bf(dP), p.grad))
dpre2 = h2.grad * (h2 > 0)
print("dH2m", rel(bf(dH2), dpre2), "unmasked-ref", rel(bf(dH2), h2.grad))
dpre1 = h1.grad * (h1 > 0)
print("dH1m", rel(bf(dH1), dpre1))
print("dz", rel(dz, zz.grad))
# direct recompute from kernel's own dH1
print("dz from dH1", rel(dz, bf(dH1) @ w1))
print("dH1 from dH2", rel(bf(dH1), ((bf(dH2) @ w2) * (h1 > 0))))
print("dH2 from dP", rel(bf(dH2), (bf(dP) @ wp) * (h2 > 0)))
k = bf(dH2); ref = bf(dP) @ wp; m = h2 > 0
print("nz xor mask frac", float(((k != 0) ^ m).float().mean()), "mask frac", float(m.float().mean()))
print("err on mask", rel(k[m], ref[m]), "kernel nonzero where mask false", float((k[~m] != 0).float().mean()))
bad = ((k - ref * m).abs() > 0.05 * ref.abs().max())
idx = bad.nonzero()[:10]
print("bad count", int(bad.sum()), "first bad (row,col)", idx.tolist())
print("bad cols hist", torch.bincount(bad.nonzero()[:, 1] % 64, minlength=64).tolist())
print("bad rows hist", torch.bincount(bad.nonzero()[:, 0] % 64, minlength=64).tolist())
