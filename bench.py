#!/usr/bin/env python3
"""bench.py -- batched turbo decoding on MI355X (BASELINE.json configs[1]).

Workload (one "step"): decode 65,536 code blocks of K = 6144 with 8 half-iterations (srslte "8 its"),
bit-exact with the srsLTE AVX2 AUTO decoder, inputs already resident in HBM in the softbuffer layout
that srslte_rm_turbo_rx_lut produces (16-window sub-block layout, 18,540 int16 per CB).  Synthetic data:
random info bits -> LTE turbo encoder -> BPSK/AWGN at Eb/N0 (test units) -> int16(100*llr), a pool of
distinct code blocks tiled over the batch.

    python bench.py [--gpus N --steps K --warmup W]            # N > 1: launched by torch.distributed.run

Multi-GPU: weak scaling -- every rank decodes its own 65,536 code blocks (independent subframes shard
with no data-path collective); ranks only meet at the timing barriers and the max-over-ranks reduction.

Prints ONE JSON line on rank 0 (schema: DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # lane-ops/s: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ncb", type=int, default=65536, help="code blocks per GPU per step")
    ap.add_argument("--K", type=int, default=6144)
    ap.add_argument("--nhalf", type=int, default=8)
    ap.add_argument("--ebno", type=float, default=2.0)
    ap.add_argument("--pool", type=int, default=256, help="distinct synthetic code blocks tiled over the batch")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
        pg = dist
    return world, rank, local, pg


def barrier(pg, local):
    if pg is not None:
        import torch
        pg.barrier(device_ids=[local])
        torch.cuda.synchronize(local)


def max_over_ranks(pg, local, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64, device=f"cuda:{local}")
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def make_pool(K, n, ebno, seed):
    import oracle  # synthetic-data generator only (encoder + AWGN); the product path never imports it
    rng = np.random.default_rng(seed)
    stride = 3 * (K + 32) + 12
    pool = np.zeros((n, stride), np.int16)
    for i in range(n):
        pool[i] = oracle.make_cb(rng, K, ebno)[2]
    return pool


def cpu_baseline(pool, K, nhalf, budget_s):
    """Reference AVX2 decoder (oracle/_ref, compiled from the srsLTE sources) on the host cores,
    or our C port if that .so is not present.  Bounded sample: repeat the pool until budget_s."""
    import oracle
    nthreads = min(os.cpu_count() or 1, 16)
    kind = "reference" if oracle.ref_available() else "port"
    fn = oracle.ref().ref_tdec_run_batch if kind == "reference" else oracle.lib().orc_tdec_run_batch
    reps = 0
    out = np.zeros((pool.shape[0], K // 8), np.uint8)
    t0 = time.perf_counter()
    while True:
        fn(pool, pool.shape[1], pool.shape[0], K, nhalf, out, nthreads)
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    ncb = reps * pool.shape[0]
    return {
        "value": round(ncb * K / dt / 1e6, 2), "unit": "Mbps", "cb_per_s": round(ncb / dt, 1),
        "cores": nthreads, "kind": kind,
        "sample": f"{ncb} x K={K} CBs ({reps} passes over a pool of {pool.shape[0]}), {nhalf} half-its, "
                  f"{nthreads} threads, {dt:.2f} s wall",
    }, out


def load_pmc_traffic():
    p = os.path.join(ROOT, "profiles", "tdec_pmc_traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except Exception:
            return None
    return None


def main():
    args = parse()
    world, rank, local, pg = dist_setup(args)
    import srsran_amd
    from srsran_amd import DeviceBuffer, TdecBatch

    K, nh, ncb = args.K, args.nhalf, args.ncb
    stride = 3 * (K + 32) + 12
    pool = make_pool(K, args.pool, args.ebno, seed=1234 + rank)
    host = np.ascontiguousarray(np.tile(pool, (ncb // args.pool + 1, 1))[:ncb])
    d_in = DeviceBuffer(host.nbytes, local).upload(host)
    del host
    d_out = DeviceBuffer(ncb * (K // 8), local)
    dec = TdecBatch(local)

    def step():
        dec.run_dev(d_in.ptr, stride, ncb, K, nh, d_out.ptr)

    for _ in range(args.warmup):
        step()
    srsran_amd.lib().mi355_device_sync()

    # correctness spot check of this rank's batch against the pool decoded by the oracle
    got = np.zeros((ncb, K // 8), np.uint8)
    d_out.download(got)

    barrier(pg, local)
    srsran_amd.lib().mi355_device_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    srsran_amd.lib().mi355_device_sync()
    barrier(pg, local)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(pg, local, dt)

    # kernel-level timing of the dominant kernel (MAP half-iteration) with HIP events on its stream
    dec.set_profiling(True)
    for _ in range(max(1, min(args.steps, 3))):
        step()
    kms, klaunch = dec.kernel_stats()
    dec.set_profiling(False)

    ms_per_step = dt / args.steps * 1e3
    cb_s = world * ncb * args.steps / dt
    mbps = cb_s * K / 1e6

    # roofline of the MAP half-iteration kernel (DESIGN.md "Measurement")
    #   algorithmic bytes per CB-half-iteration: DEC1 reads S, a1, P0 and writes e; DEC2 reads e, P1 and
    #   writes a1 (int16 x K each) -> (4 + 3) / 2 * 2K bytes on average per launch-CB.
    bytes_per_cb_halfit = 3.5 * 2 * K
    avg_launch_ms = kms / max(klaunch, 1)
    achieved = bytes_per_cb_halfit * ncb / (avg_launch_ms / 1e3) / 1e9
    pmc = load_pmc_traffic()
    # VALU: wave-instructions of the MAP kernel per launch from SQ_INSTS_VALU (profiles/), one wave-
    # instruction = 64 lanes x 2 packed int16 ops; peak = 1024 SIMDs x 1 wave-instruction / 2 clk.
    valu_insts = (pmc or {}).get("valu_insts_per_launch")

    res = {
        "metric": "PDSCH decoded Mbps + code-blocks/sec, 20 MHz TM4 QAM256, 1/2/4/8 GPU",
        "value": round(mbps, 1),
        "unit": "Mbps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic",
        "config": {"workload": f"batched turbo decode: {ncb} x K={K} code blocks per GPU, {nh} half-iterations "
                               f"(srslte '8 its'), AUTO 16-window bit-exact, Eb/N0 {args.ebno} (test units)",
                   "code_blocks_per_gpu": ncb, "K": K, "half_iterations": nh, "parallelism": f"dp{world}"},
        "code_blocks_per_s": round(cb_s, 1),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": (pmc or {}).get("bytes_per_launch"),
                     "kernel": "tdec_win_halfit<16,8>", "avg_launch_ms": round(avg_launch_ms, 4),
                     "algorithmic_bytes_per_launch": int(bytes_per_cb_halfit * ncb)},
    }
    if valu_insts and (pmc or {}).get("launch_ncb") == ncb:
        rate = valu_insts * 64 / (avg_launch_ms / 1e3) / 1e12
        res["roofline_valu"] = {"achieved": round(rate, 2), "peak": round(VALU_PEAK_TOPS, 1),
                                "unit": "T lane-instr/s", "frac": round(rate / VALU_PEAK_TOPS, 4),
                                "source": "SQ_INSTS_VALU from profiles/tdec_pmc_traffic.json"}

    if rank == 0 and world == 1 and not args.no_cpu:
        cb, cpu_out = cpu_baseline(pool[: min(args.pool, 256)], K, nh, args.cpu_seconds)
        res["cpu_baseline"] = cb
        # the GPU result for the pool must equal the CPU (reference) result bit for bit
        res["parity_vs_cpu"] = bool(np.array_equal(got[: cpu_out.shape[0]], cpu_out))
    if rank == 0:
        print(json.dumps(res), flush=True)
    dec.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
