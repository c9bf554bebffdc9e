"""Worker of tests/test_dist.py: runs bench.py's distributed plumbing on CPU (gloo) under torch.distributed.run."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["BENCH_DIST_BACKEND"] = "gloo"
import bench  # noqa: E402


def main():
    out = sys.argv[1]
    world, rank, local, pg = bench.dist_setup()
    bench.barrier(pg, local)
    t0 = time.perf_counter()
    time.sleep(0.05 * (rank + 1))  # ranks finish at different times: the job time is the slowest rank's
    dt = time.perf_counter() - t0
    bench.barrier(pg, local)
    dt_max = bench.max_over_ranks(pg, local, dt)
    ok = bench.sum_over_ranks(pg, local, 10 + rank)
    seeds = bench.sum_over_ranks(pg, local, bench.shard_seed(rank))
    rate = bench.whole_job_rate(world, 2048, 5, dt_max)
    if rank == 0:
        json.dump({"world": world, "dt": dt, "dt_max": dt_max, "ok": ok, "seeds": seeds, "rate": rate}, open(out, "w"))
    pg.destroy_process_group()


if __name__ == "__main__":
    main()
