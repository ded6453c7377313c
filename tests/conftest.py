import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def load_golden(name):
    path = os.path.join(GOLDEN, name + ".npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def t(a, **kw):
    return torch.from_numpy(np.ascontiguousarray(a)).to(**kw) if kw else \
        torch.from_numpy(np.ascontiguousarray(a))


@pytest.fixture(scope="session")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def text_heading_golden(name):
    """A TextHeading fixture with its conv weights regenerated from the stored
    seed (tests/golden/make_golden.py:text_heading_inputs)."""
    from tests.golden.make_golden import text_heading_inputs
    g = load_golden(name)
    b, L = g["words_emb"].shape[0], int(g["bert_words_num"])
    words, ws, bs = text_heading_inputs(int(g["seed"]), b, L)
    assert np.array_equal(words, g["words_emb"])
    g["conv_w"], g["conv_b"] = ws, bs
    return g


def words_seeded_golden(name):
    """A full-shape words_loss fixture with its inputs regenerated from the
    stored seed (tests/golden/make_golden.py:words_seeded_inputs), checked
    against the stored input checksums: (fixture, R [B,256,14,14], W [B,256,T])."""
    from tests.golden.make_golden import words_seeded_inputs
    g = load_golden(name)
    b, L = int(g["batch"]), int(g["bert_words_num"])
    r, w = words_seeded_inputs(int(g["seed"]), b, L - 2)
    assert abs(r.double().sum().item() - float(g["r_sum"])) < 1e-9
    assert abs(w.double().sum().item() - float(g["w_sum"])) < 1e-9
    return g, r, w
