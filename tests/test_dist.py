"""The N > 1 path of bench.py on CPU: two ranks under torch.distributed.run with the gloo backend exercise
the same plumbing the GPU node uses with RCCL (one process per device, barrier, max-over-ranks job time,
sum of CRC-ok TBs, per-rank shard seeds, whole-job rate).  Subframes are independent, so there is no
data-path collective to test."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo(tmp_path):
    out = tmp_path / "dist.json"
    env = {**os.environ, "MASTER_ADDR": "127.0.0.1", "OMP_NUM_THREADS": "1"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.load(open(out))
    assert res["world"] == 2
    assert res["dt_max"] >= res["dt"] and res["dt_max"] >= 0.1  # rank 1 slept 0.1 s
    assert res["ok"] == 10 + 11
    assert res["seeds"] == 4242 + 4243  # distinct shards
    assert abs(res["rate"] - 2 * 2048 * 5 / res["dt_max"]) < 1e-6
