"""bench.py's secondary workloads run end to end on the GPU at small sizes (the round-end driver runs only the default
one): --workload tdec (configs[1] regime, with the MAP kernel's bandwidth-only clone) and --workload siso_qpsk
(configs[2]), each a subprocess printing one JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_bench_tdec_workload_small():
    res = _bench(["--workload", "tdec", "--ncb", "2048", "--steps", "1", "--warmup", "1", "--no-cpu"])
    assert res["value"] > 0 and res["n_gpus"] == 1
    roof = res["roofline"]
    assert roof["avg_launch_ms"] > 0 and 0 < roof.get("schedule_frac", 1.0) < 2.0


@pytest.mark.gpu
def test_bench_siso_workload_small():
    res = _bench(["--workload", "siso_qpsk", "--subframes", "256", "--steps", "1", "--warmup", "1", "--no-cpu",
                  "--no-roofline"])
    assert res["crc_ok_tbs"] == "256/256" and res["value"] > 0
