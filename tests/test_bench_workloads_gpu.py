"""bench.py's workloads run end to end on the GPU at small sizes, each a subprocess printing one JSON line.

The round-end driver runs `python3 bench.py --gpus 1 --steps 20 --warmup 5`: the default (pdsch) workload WITH the
MAP-kernel probe (roofline, bandwidth-only clone), the CPU baseline, the configs[0] generic leg, the drop-in latency
leg and the waterfall.  test_bench_default_workload_small runs exactly that code path at a smaller batch; ue_dl and
siso_qpsk run with their probes too (map_probe is shared by all three), tdec with its own clone."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=110):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _check_map_roofline(res):
    roof = res["roofline"]
    assert roof is not None and roof["avg_launch_ms"] > 0
    assert 0 < roof["schedule_frac"] < 2.0
    assert 0 < roof["frac"] < 1.0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_default_workload_small():
    """The driver's command path (default workload, roofline + cpu_baseline on) at 256 subframes per step."""
    res = _bench(["--gpus", "1", "--steps", "2", "--warmup", "1", "--subframes", "256", "--cpu-seconds", "3"],
                 timeout=280)
    assert res["n_gpus"] == 1 and res["value"] > 0 and res["ms_per_step"] > 0
    assert res["crc_ok_tbs"] == "512/512"
    _check_map_roofline(res)
    cpu = res["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] in ("reference", "port")
    assert res["decoder_bound_fixed8"]["ms"] > 0
    assert res["config1_generic"]
    assert "dropin_tti_latency" in res


@pytest.mark.gpu
def test_bench_ue_dl_workload_small():
    res = _bench(["--workload", "ue_dl", "--subframes", "256", "--steps", "1", "--warmup", "1", "--no-cpu"])
    assert res["crc_ok_tbs"] == "512/512" and res["value"] > 0
    _check_map_roofline(res)


@pytest.mark.gpu
def test_bench_tdec_workload_small():
    res = _bench(["--workload", "tdec", "--ncb", "2048", "--steps", "1", "--warmup", "1", "--no-cpu"])
    assert res["value"] > 0 and res["n_gpus"] == 1
    roof = res["roofline"]
    assert roof["avg_launch_ms"] > 0 and 0 < roof.get("schedule_frac", 1.0) < 2.0


@pytest.mark.gpu
def test_bench_siso_workload_small():
    res = _bench(["--workload", "siso_qpsk", "--subframes", "256", "--steps", "1", "--warmup", "1", "--no-cpu"])
    assert res["crc_ok_tbs"] == "256/256" and res["value"] > 0
    assert res["roofline"] is not None and res["roofline"]["avg_launch_ms"] > 0
