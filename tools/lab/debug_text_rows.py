"""Lab (GPU): where TextHeading's attached fp16 operand rows differ from prep_rows."""
import sys
import torch
sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K
from text_guided_face_recognition_amd.config import make_args
from text_guided_face_recognition_amd.models.models import TextHeading

for L, prec in ((24, "fp16"), (32, "bf16"), (24, "bf16")):
    torch.manual_seed(L)
    net = TextHeading(make_args(bert_words_num=L, precision=prec)).cuda()
    with torch.no_grad():
        words, _ = net(torch.randn(9, L - 1, 768, device="cuda"))
    T = L - 2
    f16 = prec == "fp16"
    view = K.words_view(words, T)
    rows, nrm = K.attached_rows(view, f16, scale=K.LOG2E)
    hi, _, n2 = K.prep_rows(view.float(), T, 32, want_norms=True, scale=K.LOG2E, f16=f16)
    d = (rows != hi)
    print(prec, L, "differ", int(d.sum()), "of", d.numel())
    if d.any():
        idx = d.nonzero()[:5]
        for b, t, c in idx.tolist():
            x = view[b, t, c].item() if t < T else 0.0
            print("  at", (b, t, c), "word", x, "rows", rows[b, t, c].item(), "prep", hi[b, t, c].item())
        print("  rows[0,0,:8]", rows[0, 0, :8].tolist(), "prep", hi[0, 0, :8].tolist())
