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


def _expected_bits(lo, hi):
    import numpy as np
    i = np.arange(lo, hi)
    return np.stack([(i * 7 + t) % 13 != 0 for t in range(2)], axis=1).reshape(-1).astype(int).tolist()


def _run_bench(args, timeout=240):
    env = {**os.environ, "BENCH_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "1"}
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


def test_bench_self_launches_ranks_and_gathers_bitmap():
    """`bench.py --gpus 2` without torchrun starts 2 ranks itself; the gathered CRC bitmap covers both shards in
    rank order (2 bits per subframe)."""
    res = _run_bench(["--gpus", "2", "--workload", "plumbing", "--subframes", "300"])
    assert res["n_gpus"] == 2
    bm = res["crc_bitmap"]
    assert bm["subframes"] == 600 and bm["length_bits"] == 1200 and bm["bits_per_subframe"] == 2
    assert res["bitmap_bits"] == _expected_bits(0, 600)
    assert bm["ok_tbs"] == sum(_expected_bits(0, 600))
    assert res["ms_per_step"] >= 40  # the slowest rank (rank 1 sleeps 40 ms) sets the job time


def test_bench_total_subframes_uneven_shards():
    """configs[4] plumbing: T not divisible by N -- contiguous shards of different length, bitmap trimmed per rank."""
    res = _run_bench(["--gpus", "3", "--workload", "plumbing", "--total-subframes", "1001"])
    assert res["n_gpus"] == 3 and res["scaling"] == "strong"
    assert res["crc_bitmap"]["length_bits"] == 2002
    assert res["bitmap_bits"] == _expected_bits(0, 1001)


def test_bench_rejects_world_mismatch():
    env = {**os.environ, "BENCH_DIST_BACKEND": "gloo", "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2",
                        "--workload", "plumbing"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_shard_range_covers_total():
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    for T, N in ((1 << 20, 8), (1001, 3), (7, 8)):
        rs = [bench.shard_range(T, N, r) for r in range(N)]
        assert rs[0][0] == 0 and rs[-1][1] == T
        assert all(rs[r][1] == rs[r + 1][0] for r in range(N - 1))
        assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_bench_fanout_scatter_equals_local_synthesis():
    """--fanout (north star: RCCL broadcast/gather over xGMI only for batch fan-out): rank 0 holds every rank's
    index-keyed input and scatters the shards; each rank's received shard must equal its own local synthesis of the
    same subframe indices bit for bit, the gathered shard SHA-1s must equal rank 0's, and the CRC bitmap is the
    default mode's."""
    res = _run_bench(["--gpus", "2", "--workload", "plumbing", "--subframes", "300", "--fanout"])
    fan = res["fanout"]
    assert fan["ranks_equal_local_synthesis"] == 2
    assert fan["shard_sha1_match"] is True
    assert fan["bytes_scattered_per_step"] == 300 * 64
    assert res["bitmap_bits"] == _expected_bits(0, 600)


def test_fanout_scatter_world1_is_a_copy():
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import bench
    full = torch.arange(12, dtype=torch.uint8).reshape(1, 12)
    recv = torch.zeros(12, dtype=torch.uint8)
    bench.fanout_scatter(None, full, recv)
    assert torch.equal(recv, full[0])
