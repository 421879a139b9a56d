"""bench.py's N > 1 path end to end on ONE GPU: two ranks under torch.distributed.run (the
launcher only), the torch-free FileStore bootstrap, the host-staged exchange (`--comm host`,
two ranks cannot share a GPU through RCCL) and the max-over-ranks timing; the JSON line
must carry the whole-job numbers of a 2-GPU run.  The launcher imports
torch, which on a fresh box can take minutes the first time (the image pages in): hence the
long time limits."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(420)
def test_bench_two_ranks_host_comm(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--comm", "host", "--config", "tiny", "--steps", "5", "--warmup", "2"]
    try:
        r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=360)
    except subprocess.TimeoutExpired as e:   # show where the ranks were
        out = (e.stdout or b"")[-3000:] if isinstance(e.stdout, bytes) else (e.stdout or "")[-3000:]
        err = (e.stderr or b"")[-3000:] if isinstance(e.stderr, bytes) else (e.stderr or "")[-3000:]
        raise AssertionError("2-rank bench timed out\nstdout: %s\nstderr: %s" % (out, err))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]            # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["warmup"] == 2
    assert d["config"]["db_rows_total"] == 2 * d["config"]["db_rows_per_gpu"]
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["scaling"] == "weak"
    assert d["good_matches"] > 0 and d["valid_bins"] > 0
    assert not any(n.startswith("sod_store_") for n in os.listdir(tmp_path))   # store removed
