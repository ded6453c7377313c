"""GPU, 2 ranks (one process per rank, torch.distributed.run, gloo transport
so both ranks can share the one GPU of a test box): the DP contrastive losses
through the HIP kernels equal the single-process global-batch losses, and
each rank's image gradients equal its rows of the global gradient."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dp_world2_matches_global(gpu, tmp_path):
    import json
    out = str(tmp_path / "dp")
    env = dict(os.environ, TGFR_DIST_BACKEND="gloo", OMP_NUM_THREADS="4", TGFR_DP_OUT=out)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "tests", "dp_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env,
                         cwd=ROOT)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    for rank in range(2):
        r = json.load(open(f"{out}.{rank}"))
        assert r["err_loss"] < 1e-4 and r["err_r"] < 1e-4 and r["err_i"] < 1e-4, r
