"""bench.py's N > 1 path end to end on ONE GPU: two ranks under torch.distributed.run (the
launcher only), the torch-free FileStore bootstrap, the host-staged exchange (`--comm host`,
two ranks cannot share a GPU through RCCL) and the max-over-ranks timing; the JSON line
must carry the whole-job numbers of a 2-GPU run.  The launcher imports
torch, which on a fresh box can take minutes the first time (the image pages in): hence the
long time limits."""
import json
import os
import signal
import socket
import subprocess
import sys
import threading

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
    env.pop("SOD_DEBUG_SYNC", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--comm", "host", "--config", "tiny", "--steps", "5", "--warmup", "2",
           "--no-cpu-baseline", "--no-extras"]
    # the ranks' output is passed through line by line as it comes (a run that prints
    # nothing for minutes reads as hung), and kept for the checks below
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True, start_new_session=True)
    timer = threading.Timer(360, lambda: os.killpg(p.pid, signal.SIGKILL))
    timer.start()
    out = []
    try:
        for line in p.stdout:
            out.append(line)
            print("[2 ranks]", line, end="", flush=True)
        rc = p.wait()
    finally:
        timer.cancel()
    text = "".join(out)
    assert rc == 0, text[-3000:]
    lines = [l for l in text.splitlines() if l.startswith("{")]
    assert len(lines) == 1, text[-2000:]            # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["warmup"] == 2
    assert d["config"]["db_rows_total"] == 2 * d["config"]["db_rows_per_gpu"]
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["scaling"] == "weak"
    assert d["good_matches"] > 0 and d["valid_bins"] > 0
    # self-verifying record: every rank's communicator and the winners each shard gave
    assert d["config"]["rccl_nranks"] is None          # --comm host: no RCCL communicator
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    assert [r["comm"] for r in d["ranks"]] == [{"kind": "host", "nranks": 2, "rank": k}
                                               for k in range(2)]
    assert all(r["shard_winners"] == d["shard_winners"] for r in d["ranks"])
    assert all(r["shard_good_winners"] == d["shard_good_winners"] for r in d["ranks"])
    assert sum(d["shard_winners"]) == d["config"]["queries"] and min(d["shard_winners"]) > 0
    assert sum(d["shard_good_winners"]) == d["good_matches"]
    assert [r["own_shard_winners"] for r in d["ranks"]] == d["shard_winners"]
    assert not any(n.startswith("sod_store_") for n in os.listdir(tmp_path))   # store removed
