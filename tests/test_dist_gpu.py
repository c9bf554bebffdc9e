"""The multi-rank bench path on GPU hardware, rehearsed on the one-GPU box: `bench.py --gpus 2` starts two rank
processes under torch.distributed.run that both decode on device 0 (BENCH_SHARE_GPU) with gloo collectives (RCCL
refuses two ranks on one device) -- the same sharding, barriers, max-over-ranks job time and CRC-bitmap gather as the
8-GPU node, with the real HIP decode behind them.  configs[4]'s contiguous shards (--total-subframes) with resident
sets and a ragged last batch, and the weak-scaling default."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=280):
    env = {**os.environ, "BENCH_DIST_BACKEND": "gloo", "BENCH_SHARE_GPU": "1", "OMP_NUM_THREADS": "1"}
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_ranks_weak_scaling_on_one_gpu():
    res = _run(["--gpus", "2", "--subframes", "256", "--steps", "2", "--warmup", "1", "--workers", "1", "--no-cpu",
                "--no-roofline", "--no-waterfall"])
    assert res["n_gpus"] == 2 and res["scaling"] == "weak"
    assert res["crc_ok_tbs"] == "1024/1024"
    assert res["crc_bitmap"]["length_bits"] == 1024 and res["crc_bitmap"]["ok_tbs"] == 1024
    assert res["payload_checked_tbs"] == "1024/1024"
    assert res["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_ranks_total_subframes_sharded_on_one_gpu():
    """configs[4] plumbing with the real decode: 600 subframes over 2 ranks (300 each: batches of 256 + 44, taken in
    turn by 2 PHY workers per rank), every payload checked, per-rank host CPU reported."""
    res = _run(["--gpus", "2", "--total-subframes", "600", "--subframes", "256", "--warmup", "1", "--workers", "2",
                "--no-cpu", "--no-roofline", "--no-waterfall"])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong"
    assert res["crc_ok_tbs"] == "1200/1200"
    assert res["crc_bitmap"]["subframes"] == 600 and res["crc_bitmap"]["ok_tbs"] == 1200
    assert res["payload_checked_tbs"] == "1200/1200"
    assert [p["subframes"] for p in res["per_rank"]] == [300, 300]
    assert all(p["host_cpu_s"] > 0 and p["workers"] == 2 for p in res["per_rank"])
