#!/usr/bin/env python3
"""bench.py -- PDSCH receive on MI355X: decoded Mbps + code blocks/s on 20 MHz TM4 2x2 QAM256 subframes
(BASELINE.json metric; configs[3] at N = 1, configs[4] as the sharded multi-GPU run).

Workload (one "step", per GPU): B subframes (default 2048 = 65,536 code blocks) of 100 PRB, 2 ports x 2 rx
antennas, CFI 1, TM4 closed-loop spatial multiplexing with 2 codewords (codebook 0), MCS 27 QAM256 with
TBS 97,896 per codeword (C = 16 x K = 6144), MMSE equaliser with CSI weighting (srsUE defaults), max 10
turbo half-iterations with CRC early stopping.  The step runs the whole srslte_ue_dl chain from
time-domain I/Q already resident in HBM:
    softbuffer reset (new TBs) -> OFDM demodulation (2 x 14 x 1536-pt DFT) -> CRS channel estimation
    (AVERAGE, Gauss, REFS noise) -> RE extraction + MMSE + demap + descramble + CSI -> rate dematching ->
    turbo decoding with per-CB CRC early stop -> TB CRC.
Synthetic data (generated before the timed region, keyed by the subframe's GLOBAL index i, so any shard of a run
regenerates its own subframes): payloads = mi355_enb_synth_payloads(i) -> the product's GPU eNodeB generator
(DL-SCH encode, QAM256, TM4 precoding, CRS) -> phy_dl_test's crossed 2x2 channel [[1,1],[1,-1]] + AWGN keyed by i
(40 dB) -> IFFT + CP; sf_idx = i % 10.

    python bench.py [--gpus N --steps K --warmup W]     # N > 1: re-launches itself under torch.distributed.run
    python bench.py --gpus 8 --total-subframes 1048576  # configs[4]: 1M subframes sharded contiguously by rank
    python bench.py --workload tdec                     # configs[1]: batched turbo decode only
    python bench.py --workload ue_dl                    # + PCFICH / PDCCH blind search -> DCI -> grant
    python bench.py --workload siso_qpsk                # configs[2]: phy_dl_test -p 100 -t 1 -m 9 (SISO QPSK)
    python bench.py --workload plumbing --gpus 2        # CPU dry run of the launcher / sharding / bitmap gather

Multi-GPU: one process per GPU.  Default: weak scaling, rank r decodes subframes [r B, (r+1) B) every step.
--total-subframes T: rank r owns the contiguous shard [r T / N, (r+1) T / N), generated on its own GPU by index
and decoded once in batches of B (the shard is held in HBM in resident sets of at most --resident-gb of I/Q).
No data-path collective: ranks meet at the timing barriers, the max-over-ranks job time and one all-gather of
the per-subframe CRC bitmaps (2 bits per subframe, RCCL over xGMI) to rank 0.

Prints ONE JSON line on rank 0 (schema: DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import ctypes as C
import gc
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# "~78.6 T packed-int16 ops/s (256 CU x 128 ops/clk x 2.4 GHz)"; ~4.3 M int16 ops per CB
# per 8-half-iteration decode and 37,848 compulsory HBM bytes per CB per decode
VALU_PEAK_I16_TOPS = 256 * 128 * 2.4e9 / 1e12
SURVEY_OPS_PER_CB_HALFIT = 4.3e6 / 8
SURVEY_BYTES_PER_CB_DECODE = 37848
METRIC = "PDSCH decoded Mbps + code-blocks/sec, 20 MHz TM4 QAM256, 1/2/4/8 GPU"
TBS = 97896
NB = TBS // 8
MAP_SOURCES = ("srsran_amd/csrc/tdec_kernels.hip", "srsran_amd/csrc/tdec_internal.h", "srsran_amd/csrc/lte_qpp_table.h")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["pdsch", "ue_dl", "siso_qpsk", "tdec", "enb", "plumbing"], default="pdsch",
                    help="pdsch: known grants (decode_batch); ue_dl: phy_dl_test's work_ue with the PCFICH / PDCCH "
                         "blind search deriving every grant (find_and_decode); siso_qpsk: configs[2], phy_dl_test -p "
                         "100 -t 1 -m 9 through find_and_decode; tdec: configs[1]; enb: the GPU "
                         "eNodeB generator (encode side, SURVEY 8f row 2); plumbing: CPU dry run of the multi-rank "
                         "launcher, sharding and CRC-bitmap gather (no GPU, no decoding)")
    ap.add_argument("--subframes", type=int, default=None,
                    help="subframes per GPU per step (batch); default 2048, 8192 for --workload siso_qpsk (its 3 code "
                         "blocks per subframe give a 2048-subframe chunk's MAP launch only 384 waves)")
    ap.add_argument("--total-subframes", type=int, default=0,
                    help="configs[4]: T subframes sharded contiguously over the ranks, each decoded once")
    ap.add_argument("--resident-gb", type=float, default=96.0, help="HBM budget for one rank's resident I/Q")
    ap.add_argument("--seed", type=int, default=4242)
    ap.add_argument("--snr", type=float, default=40.0)
    ap.add_argument("--siso-snr", type=float, default=None, help="siso_qpsk AWGN SNR (default none, as phy_dl_test)")
    ap.add_argument("--waterfall-snr", type=float, default=28.0,
                    help="SNR of the decoder-bound e2e field (EPA 5 Hz fading)")
    ap.add_argument("--no-waterfall", action="store_true")
    ap.add_argument("--parity-subframes", type=int, default=64,
                    help="waterfall subframes re-decoded by the reference AVX2 chain (crc_parity_vs_avx2)")
    ap.add_argument("--ncb", type=int, default=65536, help="tdec workload: code blocks per GPU per step")
    ap.add_argument("--K", type=int, default=6144)
    ap.add_argument("--nhalf", type=int, default=8)
    ap.add_argument("--ebno", type=float, default=6.0, help="tdec workload Eb/N0 (SURVEY 8(d) config 2: 6.0 and 4.0)")
    ap.add_argument("--pool", type=int, default=256, help="tdec workload: distinct code blocks tiled")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="wall budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip the per-stage and MAP-kernel probes (profiling runs)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="ue_dl / siso_qpsk: find_and_decode chunks per call (default: 1 with several workers, else "
                         "the library's choice)")
    ap.add_argument("--workers", type=int, default=None,
                    help="pdsch / ue_dl: PHY worker threads, each with its own receive context (ue_dl, stream, "
                         "softbuffers) decoding every W-th batch (srsUE's sf_worker pool, 3 by default); 1 = one "
                         "synchronous loop.  Default 3 (measured best with one find_and_decode chunk per call, "
                         "profiles/r05/workers_ab.txt, uedl_chunks_ab.txt)")
    ap.add_argument("--fanout", action="store_true",
                    help="batch fan-out: rank 0 holds every rank's I/Q and scatters the shards over RCCL each step "
                         "(pdsch / ue_dl / plumbing workloads); payload SHA-1s and CRC bitmaps gathered back")
    args = ap.parse_args(argv)
    if args.subframes is None:
        args.subframes = 8192 if args.workload == "siso_qpsk" else 2048
    if args.workers is None:
        args.workers = 3
    return args


# ====================================================================================== launcher / distributed

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(args) -> None:
    """`--gpus N` (N > 1) without a torch.distributed environment: start N rank processes under
    torch.distributed.run and exit with its return code.  Nothing here touches the GPU (the ranks do)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def dist_backend() -> str:
    """RCCL ("nccl") on the GPU node; BENCH_DIST_BACKEND=gloo runs the same plumbing on CPU (tests/test_dist.py)."""
    return os.environ.get("BENCH_DIST_BACKEND", "nccl")


def dist_setup(expect_world: int | None = None):
    """One process per GPU (torch.distributed.run): the ranks share nothing but the timing barriers, the
    max-over-ranks reduction and the CRC-bitmap gather -- subframes are independent."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BENCH_SHARE_GPU"):
        # rehearsal of the multi-rank path on a one-GPU box (tests/test_dist_gpu.py): every rank decodes on device 0,
        # the collectives go over gloo (RCCL refuses two ranks on one device)
        if dist_backend() == "nccl":
            raise SystemExit("bench.py: BENCH_SHARE_GPU needs BENCH_DIST_BACKEND=gloo")
        local = 0
    if expect_world is not None and world != expect_world:
        raise SystemExit(f"bench.py: --gpus {expect_world} but the launcher started WORLD_SIZE={world} ranks")
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if dist_backend() == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(dist_backend(), rank=rank, world_size=world)
        pg = dist
    return world, rank, local, pg


def barrier(pg, local):
    if pg is not None:
        if dist_backend() == "nccl":
            import torch
            pg.barrier(device_ids=[local])
            torch.cuda.synchronize(local)
        else:
            pg.barrier()


def _dev(local):
    return f"cuda:{local}" if dist_backend() == "nccl" else "cpu"


def max_over_ranks(pg, local, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64, device=_dev(local))
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(pg, local, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64, device=_dev(local))
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def gather_bitmap(pg, local, bits: np.ndarray):
    """Per-subframe CRC bits of every rank (rank order) on rank 0: each rank packs its 0/1 bits (2 per subframe),
    one all-gather of the packed bytes over RCCL (padded to the longest shard) and rank 0 trims each rank's part.
    Returns the concatenated bits on rank 0, None elsewhere (the local bits without a process group)."""
    bits = np.ascontiguousarray(bits, np.uint8)
    if pg is None:
        return bits
    import torch
    world, rank = pg.get_world_size(), pg.get_rank()
    n = torch.tensor([bits.size], dtype=torch.int64, device=_dev(local))
    ns = [torch.zeros_like(n) for _ in range(world)]
    pg.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    nbytes = (max(ns) + 7) // 8
    packed = np.zeros(nbytes, np.uint8)
    p = np.packbits(bits)
    packed[: p.size] = p
    t = torch.from_numpy(packed).to(_dev(local))
    outs = [torch.zeros_like(t) for _ in range(world)]
    pg.all_gather(outs, t)
    if rank != 0:
        return None
    return np.concatenate([np.unpackbits(o.cpu().numpy())[: ns[r]] for r, o in enumerate(outs)])


def gather_bytes(pg, local, b: bytes, n: int) -> list[bytes] | None:
    """n bytes of every rank on rank 0 (all-gather of one uint8 tensor), None elsewhere; [b] without a group."""
    if pg is None:
        return [b]
    import torch
    t = torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to(_dev(local))
    assert t.numel() == n
    outs = [torch.zeros_like(t) for _ in range(pg.get_world_size())]
    pg.all_gather(outs, t)
    return [o.cpu().numpy().tobytes() for o in outs] if pg.get_rank() == 0 else None


def fanout_scatter(pg, full, recv) -> None:
    """Batch fan-out (north star: "RCCL broadcast/gather over xGMI only for batch fan-out"): rank 0 holds
    the I/Q of every rank's shard as one (world, shard bytes) tensor, and ONE scatter puts row r into rank r's
    receive buffer -- srsUE's I/Q enters one host (srsue/src/phy/sync.cc:884-892), the decode fans out.  RCCL (or
    gloo on CPU) moves (world - 1) shards over xGMI; without a process group it is a local copy."""
    if pg is None:
        recv.copy_(full[0])
        return
    pg.scatter(recv, list(full.unbind(0)) if pg.get_rank() == 0 else None, src=0)


class TorchBuf:
    """A torch device tensor as a raw buffer of the C ABI (.ptr): the fan-out's RCCL scatter writes where the decoder
    reads, without a copy."""

    def __init__(self, nbytes: int, local: int):
        import torch
        self.t = torch.empty(int(nbytes), dtype=torch.uint8, device=f"cuda:{local}")
        self.ptr, self.nbytes = self.t.data_ptr(), int(nbytes)


def plumbing_iq(first: int, n: int, nbytes: int) -> np.ndarray:
    """The plumbing workload's fabricated "I/Q" of subframes [first, first + n): nbytes per subframe keyed by the
    global index (the CPU stand-in for the GPU generator's index-keyed synthesis)."""
    i = np.arange(first, first + n, dtype=np.uint64)[:, None]
    j = np.arange(nbytes, dtype=np.uint64)[None, :]
    return (((i * np.uint64(2654435761)) ^ (j * np.uint64(40503))) >> np.uint64(7)).astype(np.uint8)


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard of rank r: [r T / N, (r + 1) T / N)."""
    return total * rank // world, total * (rank + 1) // world


def shard_seed(rank: int) -> int:
    """Per-rank seed of the turbo-only workload's code-block pool (weak scaling: distinct work per rank)."""
    return 4242 + rank


def whole_job_rate(world: int, units_per_rank: int, steps: int, dt_max: float) -> float:
    """Units of all ranks over the slowest rank's time (value = whole-job aggregate)."""
    return world * units_per_rank * steps / dt_max


def bitmap_summary(bits: np.ndarray, nsf: int) -> dict:
    return {"subframes": nsf, "bits_per_subframe": 2, "length_bits": int(bits.size), "ok_tbs": int(bits.sum()),
            "sha1": hashlib.sha1(np.packbits(bits).tobytes()).hexdigest()}


# ====================================================================================== host facts

def host_cores() -> tuple[int, dict]:
    """CPU threads this process may use: the affinity mask, capped by the cgroup CPU quota (cpu.max / cfs)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except Exception:
            pass
    n = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return n, {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(), "model": model}


# ====================================================================================== roofline

def map_kernel_hash() -> str:
    h = hashlib.sha1()
    for p in MAP_SOURCES:
        h.update(open(os.path.join(ROOT, p), "rb").read())
    return h.hexdigest()


def pmc_file(mode: str) -> str:
    """The MAP kernel's PMC summary for a probe mode (tools/map_pmc_summary.py): e2e (pdsch / ue_dl probes), siso,
    tdec."""
    return os.path.join(ROOT, "profiles", f"map_pmc_{mode}.json")


def load_pmc(ncb: int, mode: str = "e2e"):
    """PMC summary of the MAP kernel for this probe mode, accepted only if it was recorded on the current kernel
    sources and the same launch size; otherwise (None, reason)."""
    path = pmc_file(mode)
    if not os.path.exists(path):
        return None, f"no PMC summary for {mode} ({os.path.relpath(path, ROOT)})"
    try:
        pmc = json.load(open(path))
    except Exception as e:  # noqa: BLE001
        return None, f"unreadable PMC summary: {e}"
    if pmc.get("kernel_src_sha1") != map_kernel_hash():
        return None, "PMC summary recorded on different MAP kernel sources (stale): traffic not reported"
    if pmc.get("launch_ncb") != ncb:
        return None, f"PMC summary recorded at {pmc.get('launch_ncb')} CBs per launch, not {ncb}"
    return pmc, None


def tdec_roofline(ms, launches, ncb, K, mode="e2e"):
    """Roofline of the MAP half-iteration kernel (tdec_win_halfit) from HIP-event timing on its stream.
    Primary (schema) entry: HBM against SURVEY 8(d)'s compulsory bytes, 37,848 B per CB per 8-half-iteration
    decode (= 4,731 B per CB half-iteration); roofline_valu: SURVEY's ~537.5 k int16 ops per CB half-iteration
    against 78.6 T ops/s.  What actually binds is HBM on the kernel's REAL traffic (both passes read the inputs, beta
    checkpoints are written and read back: DESIGN.md 4.1, profiles/r02f_mapexp): traffic_frac = PMC bytes per launch
    / launch time / peak, reported when the PMC summary matches the kernel sources."""
    avg = ms / max(launches, 1)
    bytes_launch = SURVEY_BYTES_PER_CB_DECODE / 8 * ncb * K / 6144
    achieved = bytes_launch / (avg / 1e3) / 1e9
    pmc, why = load_pmc(ncb, mode)
    traffic = None
    if pmc:
        traffic = pmc["hbm_bytes_per_launch"]
    design_bytes = 3.5 * 2 * K * ncb  # the design's own per-launch reads + writes
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "tdec_win_halfit<16,8>",
            "avg_launch_ms": round(avg, 4), "algorithmic_bytes_per_launch": int(bytes_launch),
            "algorithmic_bytes_source": "SURVEY 8(d): 37,848 B per CB per decode / 8 half-iterations",
            "design_bytes_per_launch": int(design_bytes),
            "design_frac": round(design_bytes / (avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "cbs_per_launch": ncb, "binding_roof": "hbm on the real traffic (traffic_frac)"}
    if why:
        roof["traffic_note"] = why
    else:
        roof["traffic_source"] = (f"{os.path.relpath(pmc_file(mode), ROOT)} ({pmc.get('tag')}): 2 x FETCH_SIZE + "
                                  "WRITE_SIZE, the same 8-half-iteration probe (tools/map_pmc.py)")
        roof["traffic_bytes_per_cb_halfit"] = round(traffic / ncb)
        roof["traffic_gbs"] = round(traffic / (avg / 1e3) / 1e9, 1)
        roof["traffic_frac"] = round(traffic / (avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    ops = SURVEY_OPS_PER_CB_HALFIT * ncb * K / 6144
    rate = ops / (avg / 1e3) / 1e12
    valu = {"bound": "valu", "achieved": round(rate, 2), "peak": round(VALU_PEAK_I16_TOPS, 1),
            "unit": "T int16 ops/s", "frac": round(rate / VALU_PEAK_I16_TOPS, 4),
            "ops_per_launch": int(ops), "ops_source": "SURVEY 8(d): ~4.3 M int16 ops per CB per 8 half-iterations"}
    if pmc and pmc.get("valu_insts_per_launch"):
        lane = pmc["valu_insts_per_launch"] * 64
        valu["measured_valu_lane_instr_per_cb_halfit"] = round(lane / ncb)
        valu["measured_lane_instr_rate_T"] = round(lane / (avg / 1e3) / 1e12, 2)
    return roof, valu


# ====================================================================================== TM4 data + decoder

def tm4_setup(nof_prb=100, cell_id=1):
    from srsran_amd import pdsch as P
    return P.make_cell(nof_prb, 2, cell_id)


def tm4_cfg(P, cell, sf_idx, rnti=0x1234, softbuffers=(0, 1)):
    prb = np.ones((2, cell.nof_prb), np.uint8)
    g = P.make_grant(cell, prb, 1, sf_idx, P.TXSCHEME_SPATIALMUX, 2,
                     [dict(mod=P.MOD_256QAM, tbs=TBS, rv=0, cw_idx=0),
                      dict(mod=P.MOD_256QAM, tbs=TBS, rv=0, cw_idx=1)], pmi=0)
    cfg = P.PdschCfg()
    cfg.grant = g
    cfg.rnti = rnti
    cfg.decoder_type = P.MIMO_DECODER_MMSE
    cfg.csi_enable = 1
    # p_a = 0 dB: the transmitter scales the PDSCH by rho_a = sqrt(2) (2 ports) whatever power_scale says
    # (pdsch.c:1174-1188), the UE undoes it with power_scale; p_b = 1: rho_b = 1 (phy_dl_test.c:173-175, 213-215)
    cfg.power_scale, cfg.p_a, cfg.p_b = 1, 0.0, 1
    cfg.softbuffer[0], cfg.softbuffer[1] = softbuffers
    return cfg


def tm4_dci_msg(cell, sf_idx, rnti=0x1234):
    """The TM4 grant of tm4_cfg as a DCI format 2 (type-0 allocation of every RBG, MCS 27 on both TBs with the
    256QAM table, precoding information 0) at the UE's first aggregation-level-4 candidate (CFI 1)."""
    from srsran_amd import pdcch as D
    d = D.DciDl()
    d.rnti, d.format, d.alloc_type = rnti, D.FORMAT2, D.ALLOC_TYPE0
    d.type0_alloc.rbg_bitmask = (1 << 25) - 1  # 100 PRB: 25 RBGs of 4
    for t in range(2):
        d.tb[t].mcs_idx, d.tb[t].rv, d.tb[t].ndi = 27, 0, 1
    d.tb[1].cw_idx = 1
    m = D.pack(cell, d, sf_idx)
    locs = D.ue_locations(D.nof_cce(cell, 1), sf_idx, rnti)
    L, n = next(lv for lv in locs if lv[0] == 2)
    m.location, m.rnti = D.DciLocation(L, n), rnti
    return m


def tm4_plans(cell, ctrl):
    """One SfPlan per subframe index 0..9: the TM4 grant of tm4_cfg (+ its DCI format 2 on the PDCCH)."""
    from srsran_amd import pdsch as P
    from srsran_amd.synth import SfPlan
    return {sf: SfPlan(sf, 1, tm4_cfg(P, cell, sf), tm4_dci_msg(cell, sf) if ctrl else None, tm=3, tbs_alt=True)
            for sf in range(10)}


def Tm4Source(cell, n_max, device, ctrl=False, chunk=256, iq_buffer=None):
    """Up to n_max TM4 subframes resident in HBM (I/Q per rx antenna + the transmitted payloads), synthesised on the
    GPU by global subframe index with the product's eNodeB generator (srsran_amd.synth.DlSource): payloads keyed by
    index -> put_pdsch -> put_refs [-> control region] -> crossed 2x2 channel + AWGN keyed by index -> IFFT."""
    from srsran_amd.synth import DlSource

    class _Tm4(DlSource):
        def generate(self, first, n, snr_db, seed, fading=None):
            super().generate(first, [self.plan_sf[(first + k) % 10] for k in range(n)], snr_db, seed, fading,
                             ctrl=self.ctrl)

    src = _Tm4(cell, 2, n_max, NB, device, H=[[1, 1], [1, -1]], chunk=chunk, iq_buffer=iq_buffer)
    src.ctrl, src.plan_sf = ctrl, tm4_plans(cell, ctrl)
    return src


def Tm4Rx(cell, B, device, ctrl=False):
    """The UE side of one TM4 batch of B subframes (srsran_amd.synth.DlReceiver); the AVERAGE estimate is written to
    row 0 only (mi355_ue_dl_set_ce_rows(1): the fused chain reads nothing else)."""
    from srsran_amd.synth import DlReceiver
    return DlReceiver(cell, 2, B, NB, device, ctrl=ctrl, max_cb=16, ce_rows=1)


CALLER_SO = os.path.join(ROOT, "tests", "dropin", "libdropin_caller.so")


class CallerCfg(C.Structure):  # caller_cfg_t of tests/dropin/caller.c
    _fields_ = [(n, C.c_uint32) for n in ("nof_prb", "nof_ports", "nof_rx", "cell_id", "rnti", "tm",
                                          "use_tbs_index_alt", "decoder_type", "csi_enable", "max_nof_iterations",
                                          "cfo_estimate_enable", "estimator_alg", "noise_alg", "sync_error_enable",
                                          "power_scale")]


def dropin_tti_latency(args, cell, local, ntti=1000, nwarm=20):
    """Per-TTI latency of the srslte_* drop-in as srsUE's DL worker drives it (cc_worker.cc:214-300, :423-470):
    decode_fft_estimate -> find_dl_dci -> dci_to_pdsch_grant -> softbuffer reset -> decode_pdsch on ONE TM4 100-PRB
    subframe at a time, from host I/Q buffers (staged over PCIe by the drop-in), in the calling thread
    (tests/dropin/caller.c caller_tti_latency, compiled against the reference headers).  10 subframes (sf_idx 0..9,
    DCI format 2 on the PDCCH, the bench's TM4 grant) from the GPU generator, cycled over `ntti` timed TTIs."""
    if not os.path.exists(CALLER_SO):
        return {"error": f"{os.path.relpath(CALLER_SO, ROOT)} not built (make -C tests/dropin where the reference "
                         "headers exist)"}
    L = C.CDLL(CALLER_SO)
    L.caller_tti_latency.argtypes = [C.POINTER(CallerCfg), C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_void_p, C.c_void_p]
    L.caller_tti_latency.restype = C.c_int
    from srsran_amd import pdsch as P
    cell = P.make_cell(cell.nof_prb, 2, cell.id, phich_resources=2)  # the caller's cell: SRSLTE_PHICH_R_1
    src = Tm4Source(cell, 10, local, ctrl=True)
    try:
        src.generate(0, 10, args.snr, args.seed)
        iq = np.ascontiguousarray(src.iq_host(0, 10))
    finally:
        src.close()
    c = CallerCfg(nof_prb=cell.nof_prb, nof_ports=2, nof_rx=2, cell_id=cell.id, rnti=0x1234, tm=3,
                  use_tbs_index_alt=1, decoder_type=1, csi_enable=1, max_nof_iterations=10, cfo_estimate_enable=1,
                  estimator_alg=0, noise_alg=0, sync_error_enable=0, power_scale=1)
    us = np.zeros((ntti, 3), np.float32)
    ok = np.zeros(ntti, np.int32)
    r = L.caller_tti_latency(C.byref(c), iq.ctypes.data, 10, nwarm, ntti, us.ctypes.data, ok.ctypes.data)
    if r != 0:
        return {"error": f"caller_tti_latency returned {r}"}
    tot = us.sum(axis=1) / 1e3
    pct = lambda v, q: round(float(np.percentile(v, q)), 3)  # noqa: E731
    return {"flow": "srslte_ue_dl_decode_fft_estimate + find_dl_dci + dci_to_pdsch_grant + decode_pdsch, one TM4 "
                    "100-PRB 2x2 QAM256 subframe per call from host I/Q (PCIe-inclusive), caller's thread",
            "ttis": ntti, "p50_ms": pct(tot, 50), "p99_ms": pct(tot, 99), "max_ms": round(float(tot.max()), 3),
            "stage_p50_ms": {"fft_estimate": pct(us[:, 0] / 1e3, 50), "pdcch_grant": pct(us[:, 1] / 1e3, 50),
                             "pdsch": pct(us[:, 2] / 1e3, 50)},
            "tbs_ok": f"{int(ok.sum())}/{2 * ntti}",
            "budget_note": "srsUE: a TTI's DL decode + UL encode must finish before its n+4 uplink (36.213 10.1); "
                           "with srsUE's default 3 PHY workers each worker has ~3 ms per TTI"}


def cpu_baseline_pdsch(src, gpu_bufs, avg_its, budget_s, ocfg_of=None, K=6144, C=16, ntb=2, tbs=TBS, max_cb=16,
                       S_max=16, label="TM4"):
    """CPU reference-path timing on the host cores (rank 0, N = 1), bounded sample of the same workload:
    S subframes' I/Q (downloaded from HBM) through oracle/orc_front.c's C chain (OFDM by a float Stockham FFT,
    estimation, RE extraction and CSI weighting restated in C; MMSE equalisation, demapping, descrambling and rate
    dematching through the reference's own AVX2 code when oracle/_ref is built, else the scalar restatement; one
    subframe per thread task) and their ntb C S code blocks through the reference's own AVX2 turbo
    decoder (oracle/_ref, compiled from the srsLTE sources) for ceil(avg half-iterations) half-iterations;
    1 thread and every usable core.  gpu_bufs: (ncb, stride) softbuffer contents the GPU produced for the same S
    subframes -- the CPU front end must reproduce them (parity_vs_gpu).  ocfg_of(d): the oracle Cfg of resident
    subframe d (default: the TM4 bench grant)."""
    import oracle
    from oracle import pdsch_chain as pc
    nthreads, host = host_cores()
    S = min(src.n, S_max)
    iq = np.ascontiguousarray(src.iq_host(0, S))
    if ocfg_of is None:
        def ocfg_of(d):
            return pc.Cfg(nof_prb=100, nof_ports=2, nof_rx=2, cell_id=1, cfi=1, sf_idx=(src.first + d) % 10, scheme=2,
                          nof_layers=2, qm=[8, 8], tbs=[TBS, TBS], csi_enable=True, power_scale=True, p_a=0.0, p_b=1)
    cfgs = (oracle.FrontCfg * S)()
    for d in range(S):
        cfgs[d] = oracle.front_cfg(ocfg_of(d))
    stride = 18600
    sb = np.zeros(S * 2 * max_cb * stride, np.int16)
    L = oracle.lib()

    def front(nt):
        reps, t0 = 0, time.perf_counter()
        while True:
            assert L.orc_ue_dl_rx_batch(cfgs, S, iq.view(np.float32).reshape(-1), 2 * src.nof_rx * src.sf_len, sb,
                                        stride, max_cb, nt) == 0
            reps += 1
            if time.perf_counter() - t0 >= budget_s / 4:
                return (time.perf_counter() - t0) / (reps * S), reps

    kind_t = "reference" if oracle.ref_available() else "port"
    fn = oracle.ref().ref_tdec_run_batch if kind_t == "reference" else L.orc_tdec_run_batch
    nh = max(1, int(math.ceil(avg_its)))
    ncb = ntb * S * C
    out = np.zeros((ncb, K // 8), np.uint8)
    cpb = ntb * C  # code blocks per subframe

    def turbo(nt, n_cb, nhalf=nh):
        reps, t0 = 0, time.perf_counter()
        while True:
            fn(bufs[:n_cb], stride, n_cb, K, nhalf, out[:n_cb], nt)
            reps += 1
            if time.perf_counter() - t0 >= budget_s / 4:
                return (time.perf_counter() - t0) / reps / n_cb, reps

    # the equaliser, demapper, descrambler and rate dematcher run as the reference's own AVX2 code when oracle/_ref
    # is built (oracle/ref/ref_front.c); OFDM, estimation, RE extraction and CSI weighting stay the C restatement's
    front_ref = oracle.front_use_reference(True)
    try:
        if front_ref:  # the rate-matching tables once, single-threaded (srslte_rm_turbo_gentables is not thread-safe)
            oracle.ref().ref_rm_turbo_rx(np.zeros(64, np.int16), 64, np.zeros(stride, np.int16), 40, 0)
        f1, r_f1 = front(1)
        fN, r_fN = front(nthreads)
    finally:
        oracle.front_use_reference(False)
    front_desc = ("float Stockham FFT, oracle chest / RE extraction / CSI weighting; the reference's AVX2 MMSE "
                  "equaliser, demapper, descrambler and rate dematcher (oracle/_ref)" if front_ref else
                  "float Stockham FFT, oracle chest / MMSE+CSI / demap / descramble / rate dematching")
    bufs = np.ascontiguousarray(sb.reshape(S, 2, max_cb, stride)[:, :ntb, :C].reshape(ncb, stride))
    # the CPU chain's decoder buffers vs the GPU's for the same subframes (systematic, parity 1, parity 2, tails):
    # equal up to the LSB-level LLR differences of the float32 FFT / estimator (tests: within +-2)
    cols = np.r_[0:K, K + 32:2 * K + 32, 2 * K + 64:3 * K + 64, 3 * K + 96:3 * K + 108]
    diff = np.abs(bufs[:, cols].astype(np.int32) - gpu_bufs[:ncb, cols].astype(np.int32))
    parity = {"max_abs_diff": int(diff.max()), "frac_entries_differing": round(float(np.mean(diff > 0)), 6)}
    t1, r_t1 = turbo(1, min(ncb, 64))
    tN, r_tN = turbo(nthreads, ncb)
    # the decoder-bound regime (fixed 8 half-iterations), one thread: per-CB fixed costs
    # (input copy, extract_input, decision) amortised as in SURVEY 6's turbodecoder_test figure
    t1_8, _ = turbo(1, min(ncb, 64), 8)
    per_sf_1 = f1 + cpb * t1
    per_sf_N = fN + cpb * tN
    bits = ntb * tbs
    return {
        "value": round(bits / per_sf_N / 1e6, 2), "unit": "Mbps", "cb_per_s": round(cpb / per_sf_N, 1),
        "cores": nthreads, "kind": "reference" if kind_t == "reference" else "port",
        "host": host,
        "one_thread": {"value": round(bits / per_sf_1 / 1e6, 2), "cb_per_s": round(cpb / per_sf_1, 1),
                       "front_ms_per_subframe": round(f1 * 1e3, 3),
                       "turbo_us_per_cb_halfit": round(t1 / nh * 1e6, 2),
                       "turbo_us_per_cb_halfit_at_8": round(t1_8 / 8 * 1e6, 2)},
        "all_cores": {"front_ms_per_subframe": round(fN * 1e3, 3),
                      "turbo_us_per_cb_halfit_per_thread": round(tN / nh * nthreads * 1e6, 2)},
        "parity_front_vs_gpu_softbuffers": parity,
        "front_kind": "reference stages" if front_ref else "port",
        "sample": (f"{S} distinct {label} subframes of this batch: C front end (oracle/orc_front.c: {front_desc}) "
                   f"{r_f1}+{r_fN} passes at 1 "
                   f"and {nthreads} threads; their {ncb} CBs (K={K}) through the reference AVX2 turbo decoder "
                   f"({kind_t}, oracle/_ref) x {nh} half-iterations (= ceil of the GPU run's mean), "
                   f"{r_t1}+{r_tN} passes"),
        "turbo_kind": kind_t,
    }


def softbuffer_contents(rx, ncb):
    """Device address and stride of the pool's decoder buffers, materialised (the fused rate dematcher leaves a fresh
    buffer's empty parity rows unwritten; the turbo-only API and the CPU baseline read every row)."""
    from srsran_amd import lib
    rx.pool.materialize()
    buf, stride, mcb = C.POINTER(C.c_int16)(), C.c_uint32(), C.c_uint32()
    lib().mi355_softbuffer_pool_buffer.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_int16)),
                                                   C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    lib().mi355_softbuffer_pool_buffer(rx.pool.h, C.byref(buf), C.byref(stride), C.byref(mcb))
    return C.cast(buf, C.c_void_p).value, stride.value


def map_probe(rx, ncb, local, K=6144, mode="e2e"):
    """Dominant kernel: the MAP half-iteration over this batch's ncb code blocks (the first ncb softbuffer slots hold
    the rate-dematched LLRs of the last step), a fixed 8 half-iterations without early stop (configs[1]'s regime
    on the e2e code blocks), HIP events on the decoder's stream.  Returns (roofline, roofline_valu, fixed8 dict)."""
    from srsran_amd import lib
    from srsran_amd.tdec import DeviceBuffer, TdecBatch
    ptr, stride = softbuffer_contents(rx, ncb)
    d_out = DeviceBuffer(ncb * (K // 8), local)
    dec = TdecBatch(local)
    dec.run_dev(ptr, stride, ncb, K, 8, d_out.ptr)
    lib().mi355_device_sync()
    t0 = time.perf_counter()
    dec.run_dev(ptr, stride, ncb, K, 8, d_out.ptr)
    lib().mi355_device_sync()
    wall = time.perf_counter() - t0
    dec.set_profiling(True)
    for _ in range(2):
        dec.run_dev(ptr, stride, ncb, K, 8, d_out.ptr)
    kms, kl = dec.kernel_stats()
    # the kernel's bandwidth-only clone (mi355_tdec_set_diag(20): same grid, loads, checkpoint stores, extrinsic
    # scatter, one xor per trellis step): the time this schedule's memory traffic alone takes on this box
    old = lib().mi355_tdec_set_diag(20)
    d_junk = DeviceBuffer(ncb * (K // 8), local)  # the clone's decisions are meaningless: kept out of d_out
    for _ in range(2):
        dec.run_dev(ptr, stride, ncb, K, 8, d_junk.ptr)
    cms, cl = dec.kernel_stats()
    lib().mi355_tdec_set_diag(old)
    d_junk.free()
    dec.set_profiling(False)
    roof, valu = tdec_roofline(kms, kl, ncb, K, mode)
    if cl:
        clone = cms / cl
        roof["schedule_clone_ms"] = round(clone, 4)
        roof["schedule_frac"] = round(clone / roof["avg_launch_ms"], 4)
        roof["schedule_note"] = ("bandwidth-only clone of tdec_win_halfit (MI355_TDEC_DIAG 20) over the same "
                                 f"{ncb:,}-CB launches: schedule_frac = clone time / real time (1.0 = the trellis math "
                                 "is fully hidden under this schedule's memory traffic)")
    fixed8 = {"code_blocks": ncb, "half_iterations": 8, "ms": round(wall * 1e3, 3),
              "code_blocks_per_s": round(ncb / wall, 1), "mbps": round(ncb * (K - 24) / wall / 1e6, 1),
              "note": f"the batch's {ncb:,} rate-dematched CBs decoded with a fixed 8 half-iterations (no early stop), "
                      f"K-24 = {K - 24:,} information bits per CB"}
    dec.close()
    return roof, valu, fixed8, (ptr, stride, d_out)


def config1_generic(local, budget_s=2.0, with_cpu=True):
    """configs[0] (turbodecoder_test -l 6144 -i 8 -d 1, turbodecoder_test.c:106-310): the GENERIC max-log-MAP on
    ONE K=6144 code block in the linear [s p0 p1] + tails layout, 8 half-iterations, on the reference's own
    input (tests/golden/tdec_generic.npz, recorded from the reference harness).  GPU: the srslte_tdec_* drop-in
    (init_manual GENERIC + force_not_sb + run_all from a host buffer, as the test calls it) -- one code block is a
    latency figure; the batched generic kernel on 16,384 copies gives its throughput.  CPU: the reference's
    generic decoder (oracle/_ref) on one host core.  Parity: every output equals the golden trace."""
    from srsran_amd import lib
    from srsran_amd.srslte import SRSLTE_TDEC_GENERIC, SrslteTdec
    from srsran_amd.tdec import DeviceBuffer, TdecBatch
    z = np.load(os.path.join(ROOT, "tests", "golden", "tdec_generic.npz"), allow_pickle=False)
    c = next(i for i in range(int(z["ncases"])) if int(z[f"c{i}_K"]) == 6144)
    K, lin, want = 6144, z[f"c{c}_lin"], z[f"c{c}_trace"][-1]
    buf = np.zeros(3 * (K + 32) + 12, np.int16)
    buf[: lin.size] = lin
    dec = SrslteTdec(6144, SRSLTE_TDEC_GENERIC)
    dec.force_not_sb()
    ok = np.array_equal(dec.run_all(buf.copy(), 8, K), want)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s / 4:
        dec.run_all(buf.copy(), 8, K)
        reps += 1
    gpu_one = (time.perf_counter() - t0) / reps
    dec.free()
    n = 16384
    stride = (3 * K + 12 + 7) // 8 * 8
    host = np.zeros((n, stride), np.int16)
    host[:, : lin.size] = lin
    d_in = DeviceBuffer(host.nbytes, local).upload(host)
    d_out = DeviceBuffer(n * (K // 8), local)
    tb = TdecBatch(local)
    lib().mi355_tdec_batch_set_impl(tb.h, 1)  # MI355_TDEC_GENERIC
    tb.run_dev(d_in.ptr, stride, n, K, 8, d_out.ptr)
    lib().mi355_device_sync()
    t0 = time.perf_counter()
    tb.run_dev(d_in.ptr, stride, n, K, 8, d_out.ptr)
    lib().mi355_device_sync()
    gpu_batch = time.perf_counter() - t0
    outs = d_out.download(np.zeros((n, K // 8), np.uint8))
    ok_batch = bool((outs == want[None, :]).all())
    tb.close()
    res = {"workload": "configs[0]: turbodecoder_test -l 6144 -i 8 -d 1 (generic MAP, linear layout, 8 half-its)",
           "gpu_one_cb_us": round(gpu_one * 1e6, 1), "gpu_one_cb_path": "srslte_tdec_run_all drop-in, host buffers",
           "gpu_batch_cbs": n, "gpu_batch_cb_per_s": round(n / gpu_batch, 1),
           "gpu_batch_mbps": round(n * K / gpu_batch / 1e6, 1), "bit_exact_vs_golden": bool(ok and ok_batch)}
    if with_cpu:
        import oracle
        if oracle.ref_available():
            ref = oracle.RefTdec(generic=True)
            okc = np.array_equal(ref.run(buf, K, 8), want)
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < budget_s / 2:
                ref.run(buf, K, 8)
                reps += 1
            cpu_one = (time.perf_counter() - t0) / reps
            res["cpu_baseline"] = {"value_us_per_cb": round(cpu_one * 1e6, 1), "cb_per_s": round(1 / cpu_one, 1),
                                   "mbps": round(K / cpu_one / 1e6, 2), "cores": 1, "kind": "reference",
                                   "bit_exact_vs_golden": bool(okc),
                                   "sample": f"{reps} decodes of the golden K=6144 block, reference generic "
                                             "decoder (turbodecoder_gen.c) on one host thread"}
    return res


class PhyWorkers:
    """srsUE's sf_worker pool (srsue/src/phy/phy.cc:135-189): one persistent host thread per receive context for the
    whole run (W = 1: the calling thread), so the warm-up steps and the timed steps run on the same threads -- a
    thread's first HIP calls carry one-off runtime setup (tens of ms, seen as the timed region's first calls when each
    run started fresh threads).  run(work, reps): reps steps, rxs[w] decoding work[w] (its list of bound batches) on
    steps w, w + W, ...; every call is synchronous, so a worker's host work between calls overlaps the others' GPU
    work.  Returns each call's wall time (s).  The cyclic garbage collector is paused for the calls (as timeit does;
    the caller collects before the warm-up): a full collection over torch's heap takes ~75 ms, 20 steps.  BENCH_CALL_TRACE=<file>: the last run's calls as (worker, start ms, end ms) JSON."""

    def __init__(self, rxs):
        import threading
        self.rxs, self.W = rxs, len(rxs)
        self.job, self.errs, self.stop = None, [], False
        # worker w starts its first call of a run w ms after worker 0, as srsUE's workers receive subframes one TTI
        # apart: three threads entering their launch phases at the same instant stall each other inside the HIP
        # runtime for 15-50 ms on some boxes (profiles/r05/stagger_ab.txt), once per run
        self.stagger = float(os.environ.get("BENCH_STAGGER_MS", "1")) * 1e-3
        self.go = threading.Barrier(self.W + 1) if self.W > 1 else None
        self.done = threading.Barrier(self.W + 1) if self.W > 1 else None
        self.th = [threading.Thread(target=self._loop, args=(w,), daemon=True) for w in range(self.W)] \
            if self.W > 1 else []
        for t in self.th:
            t.start()

    def _steps(self, w):
        work, reps, calls, post = self.job
        if w and self.stagger:
            time.sleep(w * self.stagger)
        for _ in range(w, reps, self.W):
            for b in work[w]:
                t = time.perf_counter()
                self.rxs[w].step(b)
                calls[w].append((t, time.perf_counter()))
                if post is not None:
                    post(w, b)

    def _loop(self, w):
        while True:
            self.go.wait()
            if self.stop:
                return
            try:
                self._steps(w)
            except Exception as e:  # noqa: BLE001 -- re-raised on the calling thread
                self.errs.append(e)
            self.done.wait()

    def run(self, work, reps, post=None):
        """post(w, bound), when given, runs on worker w's thread after each of its calls (results read while the
        worker's receive context still holds them)."""
        calls = [[] for _ in range(self.W)]
        self.job, self.errs = (work, reps, calls, post), []
        gc.disable()
        try:
            if self.W == 1:
                self._steps(0)
            else:
                self.go.wait()
                self.done.wait()
                if self.errs:
                    raise self.errs[0]
        finally:
            gc.enable()
        trace = os.environ.get("BENCH_CALL_TRACE")
        if trace:
            t0 = min((c[0][0] for c in calls if c), default=0.0)
            with open(trace, "w") as f:
                json.dump([[w, round((a - t0) * 1e3, 3), round((b - t0) * 1e3, 3)] for w, cw in enumerate(calls)
                           for a, b in cw], f)
        return [b - a for cw in calls for a, b in cw]

    def close(self):
        if self.th:
            self.stop = True
            self.go.wait()
            for t in self.th:
                t.join()
            self.th = []


def chunks_for(args, W):
    """find_and_decode chunks per call: --chunks, else 1 with several PHY workers, else the library's default (0)"""
    if args.chunks is not None:
        return args.chunks
    return 1 if W > 1 else 0


def run_workers(rxs, work, reps):
    """one run of a PhyWorkers pool over rxs (threads started and joined here)"""
    pool = PhyWorkers(rxs)
    try:
        return pool.run(work, reps)
    finally:
        pool.close()


def call_stats(calls):
    """p50 / max of the timed calls' wall times (a step far above p50 is a host-side stall inside the timed region)"""
    if not calls:
        return None
    a = np.sort(np.asarray(calls)) * 1e3
    return {"calls": int(a.size), "p50_ms": round(float(a[a.size // 2]), 3), "max_ms": round(float(a[-1]), 3)}


def run_pdsch(args, world, rank, local, pg):
    if args.total_subframes:
        return run_pdsch_total(args, world, rank, local, pg)
    from srsran_amd import lib
    cell = tm4_setup()
    B = args.subframes
    ctrl = args.workload == "ue_dl"
    lo, hi = rank * B, (rank + 1) * B
    R, nsets = B, 1
    src = Tm4Source(cell, R, local, ctrl)
    rx = Tm4Rx(cell, B, local, ctrl)
    # PHY workers (srsUE runs 3 sf_worker threads, srsue/src/phy/phy.cc:135-189): W receive contexts (own ue_dl, stream,
    # softbuffer pool, grids), each host thread decoding every W-th batch, so one worker's host work between its
    # synchronous calls (result read-back, next call's planning) overlaps the GPU work of the others
    W = max(1, args.workers)
    rxs = [rx] + [Tm4Rx(cell, B, local, ctrl) for _ in range(W - 1)]
    if ctrl and chunks_for(args, W):
        # find_and_decode's two-chunk pipelining overlaps one call's host replay with its own GPU work; with several
        # workers the other workers' batches fill those gaps, and one chunk saves the second chunk's launches
        # (profiles/r05/uedl_chunks_ab.txt)
        for r in rxs:
            r.ue.set_chunks(chunks_for(args, W))
    pool = PhyWorkers(rxs)
    dt_total, ok_sample, sample_tbs, bits_all, its_all, batches = 0.0, 0, 0, [], [], 0
    for s in range(nsets):
        a = lo + s * R
        n = max(0, min(R, hi - a))
        if n:
            src.generate(a, n, args.snr, args.seed)
        bound = [rx.bind(src, k0, min(B, n - k0)) for k0 in range(0, n, B)]
        wbound = [bound] + [[r.bind(src, k0, min(B, n - k0)) for k0 in range(0, n, B)] for r in rxs[1:]]
        if s == 0 and bound:
            gc.collect()  # before the warm-up: the timed steps follow it without an idle gap (a collection over
            # torch's heap is ~75 ms, long enough for the GPU to drop its clocks)
            pool.run([wb[:1] for wb in wbound], args.warmup * W)  # every worker warms up on its own thread
            lib().mi355_device_sync()
        reps = args.steps
        barrier(pg, local)
        lib().mi355_device_sync()
        t0 = time.perf_counter()
        calls = pool.run(wbound, reps)
        lib().mi355_device_sync()
        barrier(pg, local)
        dt_total += time.perf_counter() - t0
        batches += reps * len(bound)
        if bound:  # payload check of the batch every worker decoded last
            wk = rxs[: min(W, reps)]
            for r, wb in zip(wk, wbound):
                ok_sample += r.payload_ok(src, wb[-1])
                sample_tbs += 2 * wb[-1][3]
            its_all.append(rx.avg_its(bound[-1][3]))
            b = rx.crc_bits(bound[-1][3])
            for r, wb in zip(wk[1:], wbound[1:]):
                b = b & r.crc_bits(wb[-1][3])  # a TB counts only if every worker decoded it
            bits_all.append(b)
    pool.close()
    dt = max_over_ranks(pg, local, dt_total)
    bits = np.concatenate(bits_all) if bits_all else np.zeros(0, np.uint8)
    gathered = gather_bitmap(pg, local, bits)
    ok_sample_all = int(sum_over_ranks(pg, local, ok_sample))
    sample_all = int(sum_over_ranks(pg, local, sample_tbs))
    its = float(np.mean(its_all)) if its_all else 0.0

    res = {"metric": METRIC, "n_gpus": world}
    ok_tbs = int(gathered.sum()) if rank == 0 else 0
    mbps = whole_job_rate(world, B * 2 * TBS, args.steps, dt) / 1e6 * (ok_tbs / (2 * B * world))
    res.update({"value": round(mbps, 1), "unit": "Mbps", "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(dt / args.steps * 1e3, 3),
                "code_blocks_per_s": round(world * 32 * B * args.steps / dt, 1),
                "subframes_per_s": round(world * B * args.steps / dt, 1), "worker_calls": call_stats(calls)})
    nsf = world * B
    res.update({
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32+int16", "data": "synthetic",
        "config": {"workload": pdsch_workload(args, B, ctrl, W), "subframes_per_gpu_batch": B,
                   "code_blocks_per_gpu_batch": 32 * B, "total_subframes": None, "workers_per_gpu": W,
                   "parallelism": f"dp{world}"},
        "crc_ok_tbs": f"{ok_tbs}/{2 * nsf}",
        "crc_bitmap": bitmap_summary(gathered, nsf) if rank == 0 else None,
        "payload_checked_tbs": f"{ok_sample_all}/{sample_all}",
        "avg_half_iterations": round(its, 3),
    })
    if args.no_roofline:
        res["roofline"] = None
    else:
        stages = {}
        if not ctrl:
            last = rx.bind(src, 0, min(B, src.n))
            rx.step(last, stages)
            res["stage_ms"] = {k: round(v, 3) for k, v in stages.items()}
        roof, valu, fixed8, (ptr, stride, _d_out) = map_probe(rx, 32 * B, local)
        res["roofline"] = roof
        res["roofline_valu"] = valu
        res["decoder_bound_fixed8"] = fixed8
        if rank == 0 and world == 1 and not args.no_cpu:
            ncb = 2 * min(src.n, 16) * 16
            gb = np.zeros((ncb, stride), np.int16)
            lib().mi355_memcpy_d2h(gb.ctypes.data, ptr, gb.nbytes)
            res["cpu_baseline"] = cpu_baseline_pdsch(src, gb, its, args.cpu_seconds)
            # the fixed-8 decisions of a CB sample against the reference decoder (cpu_baseline leg)
            res["decoder_bound_fixed8"]["parity_vs_reference"] = fixed8_parity(gb[:64], _d_out)
        if rank == 0 and world == 1:
            res["config1_generic"] = config1_generic(local, with_cpu=not args.no_cpu)
            if not ctrl:
                res["dropin_tti_latency"] = dropin_tti_latency(args, cell, local)
    if not ctrl and not args.no_waterfall:
        res["e2e_waterfall"] = waterfall(args, cell, B, src, rx, pg, local, world)
    for r in rxs:
        r.close()
    src.close()
    return res


def pdsch_workload(args, B, ctrl, W):
    workload = (f"srslte_ue_dl chain from time-domain I/Q: {B} subframes/GPU/batch, 20 MHz (100 PRB), TM4 2x2 "
                "spatial multiplexing, 2 codewords QAM256 TBS 97896 (C=16, K=6144), MMSE+CSI, max 10 half-its with "
                f"CRC early stop, {args.snr:g} dB crossed 2x2 channel, every subframe distinct (GPU eNodeB generator, "
                "keyed by global subframe index)")
    if ctrl:
        workload += ("; grants from the PCFICH/PDCCH blind search (DCI format 2 per subframe, find_and_decode = "
                     "phy_dl_test work_ue)")
    if W > 1:
        workload += (f"; {W} PHY worker threads (own ue_dl / stream / softbuffers each) decode alternate batches, "
                     "every batch a synchronous call")
    return workload


def host_cpu_seconds() -> float:
    """user + system CPU seconds of this process, every thread"""
    import resource
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def gather_floats(pg, local, vals) -> list | None:
    """a fixed-length float64 vector of every rank on rank 0 (rank order), None elsewhere"""
    b = np.asarray(vals, np.float64).tobytes()
    g = gather_bytes(pg, local, b, len(b))
    return None if g is None else [np.frombuffer(x, np.float64).tolist() for x in g]


def run_pdsch_total(args, world, rank, local, pg):
    """configs[4]: T subframes sharded contiguously over the ranks ([r T / N, (r + 1) T / N) on rank r), each decoded
    ONCE.  A rank holds its shard in HBM in resident sets of at most --resident-gb of I/Q (whole batches; synthesised
    on its GPU by global subframe index before each set's timed region), and its W PHY workers (srsUE's sf_worker
    pool, each with its own receive context) take the set's batches in turn, batch j on worker j mod W.  After each
    call the worker reads the batch's CRC bits and checks every decoded payload on the GPU against the index-keyed
    transmitted payload (mi355_enb_payload_check: ~12 KB compared per TB, a few tens of us per batch, inside the
    timed region).  Timed: the decode of every set (barrier + device sync on both sides), summed over sets, max over
    ranks.  The per-subframe CRC bitmap of the whole job (2 bits per subframe) is all-gathered to rank 0."""
    from srsran_amd import lib
    from srsran_amd.tdec import DeviceBuffer
    cell = tm4_setup()
    B = args.subframes
    ctrl = args.workload == "ue_dl"
    sf_bytes = 2 * 15 * 1536 * 8
    T = args.total_subframes
    lo, hi = shard_range(T, world, rank)
    max_shard = -(-T // world)
    R = max(B, int(args.resident_gb * 1e9 / sf_bytes) // B * B)  # resident set, whole batches
    R = min(R, -(-max_shard // B) * B)
    nsets = -(-max_shard // R)
    src = Tm4Source(cell, R, local, ctrl)
    W = max(1, args.workers)
    rxs = [Tm4Rx(cell, B, local, ctrl) for _ in range(W)]
    if ctrl and chunks_for(args, W):
        for r in rxs:
            r.ue.set_chunks(chunks_for(args, W))
    d_ok = DeviceBuffer(max(1, 2 * (hi - lo)), local)  # per TB of the shard: decoded payload == transmitted
    lib().mi355_memset_dev(d_ok.ptr, 0, d_ok.nbytes)
    pool = PhyWorkers(rxs)
    bits = np.zeros(2 * (hi - lo), np.uint8)
    its_sum, its_n, batches, dt_total, cpu_total = 0.0, 0, 0, 0.0, 0.0
    prog = os.environ.get("BENCH_PROGRESS") is not None
    t_job = time.perf_counter()
    for s in range(nsets):
        a = lo + s * R  # first global subframe of the set
        n = max(0, min(R, hi - a))
        if n:
            src.generate(a, n, args.snr, args.seed)
        ks = list(range(0, n, B))
        wbound = [[rxs[w].bind(src, k0, min(B, n - k0)) for j, k0 in enumerate(ks) if j % W == w] for w in range(W)]
        if s == 0:
            gc.collect()
            if ks:
                pool.run([wb[:1] for wb in wbound], args.warmup * W)  # every worker warms up on its own thread
            lib().mi355_device_sync()

        def post(w, b, a=a):
            k0, m = b[4], b[3]
            g0 = a - lo + k0  # first subframe of the batch within the shard
            rx = rxs[w]
            bits[2 * g0: 2 * (g0 + m)] = rx.crc_bits(m)
            src.enb.payload_check(rx.d_pay.ptr, rx.plen, a + k0, m, 2, NB, args.seed, d_ok.ptr + 2 * g0)

        barrier(pg, local)
        lib().mi355_device_sync()
        c0, t0 = host_cpu_seconds(), time.perf_counter()
        pool.run(wbound, W, post)  # every batch of the set once, batch j on worker j mod W
        lib().mi355_device_sync()
        barrier(pg, local)
        dt_total += time.perf_counter() - t0
        cpu_total += host_cpu_seconds() - c0
        batches += len(ks)
        for w in range(W):
            if wbound[w]:
                its_sum += rxs[w].avg_its(wbound[w][-1][3])
                its_n += 1
        if prog:
            print(f"[bench rank {rank}] set {s + 1}/{nsets}: {n} subframes, decode {dt_total:.3f} s so far, "
                  f"{time.perf_counter() - t_job:.1f} s wall", file=sys.stderr, flush=True)
    pool.close()
    ok_pay = np.zeros(2 * (hi - lo), np.uint8)
    if ok_pay.size:
        lib().mi355_memcpy_d2h(ok_pay.ctypes.data, d_ok.ptr, ok_pay.nbytes)
    d_ok.free()
    pay_ok = int(((ok_pay != 0) & (bits != 0)).sum())
    dt = max_over_ranks(pg, local, dt_total)
    gathered = gather_bitmap(pg, local, bits)
    pay_all = int(sum_over_ranks(pg, local, pay_ok))
    host = gather_floats(pg, local, [dt_total, cpu_total, hi - lo, W])
    ok_tbs = int(gathered.sum()) if rank == 0 else 0
    mbps = ok_tbs * TBS / dt / 1e6
    workload = (f"configs[4]: {T} subframes sharded contiguously over {world} GPU(s), each decoded once; "
                + pdsch_workload(args, B, ctrl, W))
    res = {"metric": METRIC, "n_gpus": world, "value": round(mbps, 1), "unit": "Mbps", "steps": batches,
           "warmup": args.warmup, "ms_per_step": round(dt / max(batches, 1) * 1e3, 3),
           "code_blocks_per_s": round(T * 32 / dt, 1), "subframes_per_s": round(T / dt, 1),
           "job_seconds": round(dt, 3), "resident_sets": nsets, "resident_subframes": R,
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32+int16",
           "data": "synthetic",
           "config": {"workload": workload, "subframes_per_gpu_batch": B, "code_blocks_per_gpu_batch": 32 * B,
                      "total_subframes": T, "workers_per_gpu": W, "parallelism": f"dp{world}"},
           "crc_ok_tbs": f"{ok_tbs}/{2 * T}",
           "crc_bitmap": bitmap_summary(gathered, T) if rank == 0 else None,
           "payload_checked_tbs": f"{pay_all}/{2 * T}",
           "payload_check": "every TB: decoded bytes == the index-keyed transmitted payload (GPU compare after each "
                            "call, mi355_enb_payload_check) and its CRC bit set",
           "avg_half_iterations": round(its_sum / max(its_n, 1), 3), "roofline": None}
    if rank == 0:
        res["per_rank"] = [{"rank": r, "subframes": int(h[2]), "decode_s": round(h[0], 3),
                            "host_cpu_s": round(h[1], 3), "host_cores_busy": round(h[1] / max(h[0], 1e-9), 2),
                            "workers": int(h[3])} for r, h in enumerate(host)]
        res["host_cpu_note"] = ("host_cpu_s: user + system CPU seconds of the rank's process (all threads) inside "
                                "its timed regions; host_cores_busy = host_cpu_s / decode_s")
        if os.environ.get("BENCH_SHARE_GPU"):
            res["rehearsal"] = (f"BENCH_SHARE_GPU: all {world} ranks on device 0 of one GPU (gloo collectives); the "
                                "value is that one GPU's, shared")
    for r in rxs:
        r.close()
    src.close()
    return res


class FanShard:
    """What a rank decodes in fan-out mode: its shard's I/Q in the scatter's receive buffer (rx-major per subframe,
    as DlSource lays it out) and the subframes' plans (grants are known per subframe index)."""

    def __init__(self, buf, plans, sf_len, nof_rx=2):
        self.buf, self.plans, self.sf_len, self.nof_rx = buf, plans, sf_len, nof_rx

    def iq_ptr(self, k: int, r: int) -> int:
        return self.buf.ptr + (k * self.nof_rx + r) * self.sf_len * 8


def tb_digest(pay: np.ndarray) -> bytes:
    """SHA-1 over the TB payload bytes of a batch, (n, 2, >= NB) -> 20 bytes."""
    return hashlib.sha1(np.ascontiguousarray(pay[:, :, :NB]).tobytes()).digest()


def run_pdsch_fanout(args, world, rank, local, pg):
    """configs[3]/[4] with the batch fan-out the north star names ("RCCL broadcast/gather over xGMI only for batch
    fan-out"): the I/Q of all world x B subframes of a step is resident on rank 0 (synthesised there by global index),
    and every step starts with ONE RCCL scatter of the shards (B x 368,640 bytes of I/Q per rank, over xGMI) into
    each rank's receive buffer, which the decoder reads in place; the ranks decode their shard (decode_batch, or
    find_and_decode with --workload ue_dl) and the CRC bitmaps plus per-rank payload SHA-1s are gathered back to
    rank 0, which checks them against the transmitted payloads.  The timed step is scatter + decode.  Every rank also
    synthesises its own shard locally once (the default mode's data) and checks the received I/Q equals it bit for
    bit, so the decode results are those of local synthesis."""
    import torch
    from srsran_amd import lib
    cell = tm4_setup()
    B = args.subframes
    ctrl = args.workload == "ue_dl"
    sf_len = 15 * 1536
    sf_bytes = 2 * sf_len * 8
    lo = rank * B
    plan_sf = tm4_plans(cell, ctrl)
    src = full = None
    if rank == 0:
        full_buf = TorchBuf(world * B * sf_bytes, local)
        src = Tm4Source(cell, world * B, local, ctrl, iq_buffer=full_buf)
        src.generate(0, world * B, args.snr, args.seed)
        full = full_buf.t.view(world, B * sf_bytes)
    recv = TorchBuf(B * sf_bytes, local)
    shard = FanShard(recv, [plan_sf[(lo + k) % 10] for k in range(B)], sf_len)
    rx = Tm4Rx(cell, B, local, ctrl)
    bound = rx.bind(shard, 0, B)

    def step():
        fanout_scatter(pg, full, recv.t)
        torch.cuda.synchronize(local)
        rx.step(bound)

    for _ in range(args.warmup):
        step()
    lib().mi355_device_sync()
    barrier(pg, local)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    lib().mi355_device_sync()
    barrier(pg, local)
    dt = max_over_ranks(pg, local, time.perf_counter() - t0)
    # the scatter alone (same buffers), for the xGMI rate
    barrier(pg, local)
    t1 = time.perf_counter()
    for _ in range(3):
        fanout_scatter(pg, full, recv.t)
    torch.cuda.synchronize(local)
    barrier(pg, local)
    dts = max_over_ranks(pg, local, time.perf_counter() - t1) / 3

    bits = rx.crc_bits(B)
    gathered = gather_bitmap(pg, local, bits)
    digs = gather_bytes(pg, local, tb_digest(rx.received(B)), 20)
    # received I/Q == this rank's own index-keyed synthesis of the same subframes (the default mode's input)
    mine = TorchBuf(B * sf_bytes, local)
    loc = Tm4Source(cell, B, local, ctrl, iq_buffer=mine)
    loc.generate(lo, B, args.snr, args.seed)
    same = int(sum_over_ranks(pg, local, float(torch.equal(mine.t, recv.t))))
    loc.close()
    ok_tbs = int(gathered.sum()) if rank == 0 else 0
    mbps = whole_job_rate(world, B * 2 * TBS, args.steps, dt) / 1e6 * (ok_tbs / (2 * B * world))
    res = {"metric": METRIC, "n_gpus": world, "value": round(mbps, 1), "unit": "Mbps", "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
           "code_blocks_per_s": round(world * 32 * B * args.steps / dt, 1),
           "subframes_per_s": round(world * B * args.steps / dt, 1), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32+int16", "data": "synthetic",
           "config": {"workload": f"batch fan-out: rank 0 holds {world} x {B} TM4 subframes of I/Q (20 MHz, 2x2, QAM256, "
                                  f"{args.snr:g} dB), one RCCL scatter per step, then each rank decodes its shard"
                                  + (" with find_and_decode" if ctrl else " with decode_batch"),
                      "subframes_per_gpu_batch": B, "parallelism": f"dp{world}+scatter"},
           "crc_ok_tbs": f"{ok_tbs}/{2 * B * world}", "roofline": None,
           "crc_bitmap": bitmap_summary(gathered, world * B) if rank == 0 else None}
    if rank == 0:
        want = [tb_digest(src.payloads(r * B, B)) for r in range(world)]
        moved = (world - 1) * B * sf_bytes
        res["fanout"] = {"bytes_per_subframe": sf_bytes, "bytes_scattered_per_step": moved,
                         "scatter_ms": round(dts * 1e3, 3),
                         "scatter_gbs": round(moved / dts / 1e9, 1) if world > 1 else None,
                         "scatter_share_of_step": round(dts / (dt / args.steps), 3),
                         "ranks_received_equal_local_synthesis": f"{same}/{world}",
                         "payload_sha1_match": [d == w for d, w in zip(digs, want)]}
        src.close()
    rx.pool.close()
    return res


SISO_TBS, SISO_K, SISO_C = 15840, 5312, 3


def run_siso(args, world, rank, local, pg):
    """configs[2]: phy_dl_test -p 100 -t 1 -m 9 (lib/test/phy/phy_dl_test.c:308-660) at batch scale: B subframes per
    GPU per step of a 20 MHz SISO cell (1 port, 1 rx, CFI 1, DCI format 1 over every RBG, MCS 9 QPSK, TBS 15,840 =
    3 CBs of K = 5312), no noise and the DCI at the test's UE-specific locations, synthesised by the GPU generator;
    the UE side is phy_dl_test's work_ue as one mi355_ue_dl_find_and_decode_batch (OFDM, estimation, PCFICH /
    PDCCH blind search, grant, PDSCH, DL-SCH) from I/Q resident in HBM."""
    from srsran_amd import lib, synth
    cell, nrx = synth.phy_dl_test_cell(100, 0)
    B = args.subframes
    lo = rank * B
    nb = SISO_TBS // 8
    plans = synth.phy_dl_test_plans(cell, 0, 9, False, nof_subframes=B, first=lo)
    src = synth.DlSource(cell, nrx, B, nb, local)
    src.generate(lo, plans, args.siso_snr, args.seed, ctrl=True)
    W = max(1, args.workers)
    rxs = [synth.DlReceiver(cell, nrx, B, nb, local, ctrl=True, max_cb=SISO_C, ce_rows=1) for _ in range(W)]
    if chunks_for(args, W):  # one find_and_decode chunk per call with several workers (as run_pdsch)
        for r in rxs:
            r.ue.set_chunks(chunks_for(args, W))
    rx = rxs[0]
    wbound = [[r.bind(src, 0, B, tb_major=True)] for r in rxs]  # TB0 code blocks contiguous in the pool (MAP probe)
    bound = wbound[0][0]
    pool = PhyWorkers(rxs)
    gc.collect()  # before the warm-up, so the timed steps follow it without an idle gap (as run_pdsch)
    pool.run(wbound, args.warmup * W)  # every worker warms up on its own thread
    lib().mi355_device_sync()
    barrier(pg, local)
    t0 = time.perf_counter()
    calls = pool.run(wbound, args.steps)
    lib().mi355_device_sync()
    barrier(pg, local)
    dt = max_over_ranks(pg, local, time.perf_counter() - t0)
    pool.close()
    bits = rx.crc_bits(B).reshape(B, 2)[:, 0].copy()  # one TB per subframe
    for r in rxs[1: min(W, args.steps)]:
        bits &= r.crc_bits(B).reshape(B, 2)[:, 0]  # a TB counts only if every worker decoded it
    gathered = gather_bitmap(pg, local, bits)
    ok_pay = int(sum_over_ranks(pg, local, min(r.payload_ok(src, wb[0]) for r, wb in zip(rxs[: max(1, min(W, args.steps))], wbound))))
    its = rx.avg_its(B) * 2  # the disabled second TB reads 0
    ok_tbs = int(gathered.sum()) if rank == 0 else 0
    mbps = whole_job_rate(world, B * SISO_TBS, args.steps, dt) / 1e6 * (ok_tbs / (B * world))
    res = {"metric": "PDSCH decoded Mbps + code-blocks/sec, 20 MHz SISO QPSK MCS 9 (configs[2], phy_dl_test -p 100 "
                     "-t 1 -m 9)",
           "value": round(mbps, 1), "unit": "Mbps", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(dt / args.steps * 1e3, 3), "worker_calls": call_stats(calls),
           "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32+int16", "data": "synthetic",
           "config": {"workload": f"phy_dl_test -p 100 -t 1 -m 9 work_ue as mi355_ue_dl_find_and_decode_batch: {B} "
                                  "subframes/GPU/batch from time-domain I/Q, 1 port / 1 rx, CFI 1, DCI format 1 at the "
                                  "test's UE locations, TBS 15840 (3 x K=5312), "
                                  + ("no noise (as phy_dl_test)" if args.siso_snr is None else f"{args.siso_snr:g} dB"),
                      "subframes_per_gpu_batch": B, "code_blocks_per_gpu_batch": SISO_C * B,
                      "workers_per_gpu": W, "parallelism": f"dp{world}"},
           "code_blocks_per_s": round(world * SISO_C * B * args.steps / dt, 1),
           "subframes_per_s": round(world * B * args.steps / dt, 1),
           "crc_ok_tbs": f"{ok_tbs}/{B * world}", "crc_bitmap": bitmap_summary(gathered, B * world) if rank == 0 else None,
           "payload_checked_tbs": f"{ok_pay}/{B * world}", "avg_half_iterations": round(its, 3)}
    if not args.no_roofline:
        roof, valu, fixed8, (ptr, stride, _d_out) = map_probe(rx, SISO_C * B, local, K=SISO_K, mode="siso")
        res["roofline"], res["roofline_valu"], res["decoder_bound_fixed8"] = roof, valu, fixed8
        if rank == 0 and world == 1 and not args.no_cpu:
            from oracle import pdsch_chain as pc
            S = min(B, 48)
            gb = np.zeros((S * SISO_C, stride), np.int16)
            lib().mi355_memcpy_d2h(gb.ctypes.data, ptr, gb.nbytes)

            def ocfg(d):
                return pc.Cfg(nof_prb=100, nof_ports=1, nof_rx=1, cell_id=1, cfi=1, sf_idx=(lo + d) % 10, scheme=0,
                              nof_layers=1, qm=[2], tbs=[SISO_TBS], csi_enable=False, power_scale=True, p_a=0.0,
                              p_b=0)
            res["cpu_baseline"] = cpu_baseline_pdsch(src, gb, its, args.cpu_seconds, ocfg_of=ocfg, K=SISO_K,
                                                     C=SISO_C, ntb=1, tbs=SISO_TBS, max_cb=SISO_C, S_max=S,
                                                     label="SISO QPSK")
    for r in rxs:
        r.close()
    src.close()
    return res


def fixed8_parity(bufs, d_out):
    """GPU decisions after a fixed 8 half-iterations on the first CBs vs the reference's AVX2 decoder
    (oracle/_ref where built, else the oracle restatement)."""
    import oracle
    n = bufs.shape[0]
    got = np.zeros((n, 768), np.uint8)
    from srsran_amd import lib
    lib().mi355_memcpy_d2h(got.ctypes.data, d_out.ptr, got.nbytes)
    want = np.zeros((n, 768), np.uint8)
    b = np.ascontiguousarray(bufs)
    if oracle.ref_available():
        oracle.ref().ref_tdec_run_batch(b, b.shape[1], n, 6144, 8, want, 1)
        kind = "reference"
    else:
        oracle.lib().orc_tdec_run_batch(b, b.shape[1], n, 6144, 8, want, 1)
        kind = "port"
    return {"cbs": n, "bit_exact": bool(np.array_equal(got, want)), "checker": kind}


def waterfall(args, cell, B, src, rx, pg, local, world):
    """Decoder-bound regime: the same batch shape through srslte_channel_fading_t EPA 5 Hz (generator, per-OFDM
    symbol block fading) at a waterfall SNR where the turbo decoder needs most of its 10 half-iterations."""
    from srsran_amd import lib
    src.generate(10_000_000 + pg_rank(pg) * B, src.n_max, args.waterfall_snr, args.seed + 1, fading="epa5")
    bound = [rx.bind(src, 0, min(B, src.n))]
    rx.step(bound[0])
    lib().mi355_device_sync()
    barrier(pg, local)
    t0 = time.perf_counter()
    steps = max(1, min(args.steps, 3))
    for _ in range(steps):
        rx.step(bound[0])
    lib().mi355_device_sync()
    barrier(pg, local)
    dt = max_over_ranks(pg, local, time.perf_counter() - t0)
    ok = int(sum_over_ranks(pg, local, int(rx.crc_bits(bound[0][3]).sum())))
    its = rx.avg_its(bound[0][3])
    out = {"snr_db": args.waterfall_snr, "channel": "EPA 5 Hz 2x2 (srslte_channel_fading_t taps, per-symbol)",
           "avg_half_iterations": round(its, 3), "crc_ok_tbs": f"{ok}/{2 * B * world}",
           "ms_per_step": round(dt / steps * 1e3, 3),
           "mbps": round(ok * TBS * steps / dt / 1e6, 1),
           "code_blocks_per_s": round(world * 32 * B * steps / dt, 1)}
    if pg_rank(pg) == 0 and world == 1 and not args.no_cpu:  # after timing: the reference AVX2 chain as checker
        out["crc_parity_vs_avx2"] = avx2_crc_parity(src, rx, S_max=args.parity_subframes)
    return out


def avx2_crc_parity(src, rx, S_max=64, max_half=10, K=6144, ncb_tb=16):
    """Decoded-CRC parity of the GPU against the reference's AVX2 chain where code blocks fail:
    the first S resident subframes of the waterfall batch the GPU just decoded (EPA 28 dB, ~1/3 of the TBs fail) go
    through the CPU front end with the reference's own AVX2 stages (srslte_predecoding_type MMSE + CSI,
    srslte_demod_soft_demodulate_s, srslte_scrambling_s_offset, srslte_rm_turbo_rx_lut via oracle/_ref; OFDM and
    estimation restated) and every TB through the reference's AVX2 turbo decoder under sch.c's early stop
    (oracle.ref_dlsch_decode_cbs, max 10 half-iterations).  Reported: TB CRC, payload and per-TB iteration agreement,
    per-CB CRC-flag agreement, and the softbuffer entries that differ.  The same reference decoder is also run on the
    GPU's own softbuffers: that leg must agree everywhere (the GPU turbo decoder is bit-exact), so every disagreement
    of the full chain is attributed to the LLR differences of the front end (the AVX2 MMSE's _mm256_rcp_ps,
    simd.h:321-337 / precoding.c:1447-1550, and the restated float FFT / estimator)."""
    import oracle
    from oracle import pdsch_chain as pc
    from srsran_amd import lib
    if not oracle.ref_available():
        return {"error": "oracle/_ref not built"}
    nthreads, _ = host_cores()
    S = min(S_max, src.n, rx.B)
    iq = np.ascontiguousarray(src.iq_host(0, S))
    cfgs = (oracle.FrontCfg * S)()
    for d in range(S):
        cfgs[d] = oracle.front_cfg(pc.Cfg(nof_prb=100, nof_ports=2, nof_rx=2, cell_id=1, cfi=1,
                                          sf_idx=(src.first + d) % 10, scheme=2, nof_layers=2, qm=[8, 8],
                                          tbs=[TBS, TBS], csi_enable=True, power_scale=True, p_a=0.0, p_b=1))
    stride = 18600
    sb = np.zeros(S * 2 * 16 * stride, np.int16)
    if not oracle.front_use_reference(True):
        return {"error": "reference front-end stages unavailable"}
    try:
        oracle.ref().ref_rm_turbo_rx(np.zeros(64, np.int16), 64, np.zeros(stride, np.int16), 40, 0)
        assert oracle.lib().orc_ue_dl_rx_batch(cfgs, S, iq.view(np.float32).reshape(-1), 2 * src.nof_rx * src.sf_len,
                                               sb, stride, 16, nthreads) == 0
    finally:
        oracle.front_use_reference(False)
    cpu_bufs = sb.reshape(S * 2, 16, stride)
    ptr, gstride = softbuffer_contents(rx, 2 * S * 16)
    gpu_bufs = np.zeros((2 * S * 16, gstride), np.int16)
    lib().mi355_memcpy_d2h(gpu_bufs.ctypes.data, ptr, gpu_bufs.nbytes)
    gpu_bufs = gpu_bufs.reshape(S * 2, 16, gstride)[:, :, :stride]
    res = np.ctypeslib.as_array(rx.res)[: 2 * S]
    g_crc = (res["crc"] != 0) & (res["ret"] == 0)
    g_its = res["avg_iterations_block"].astype(np.float64)
    g_pay = rx.received(S).reshape(2 * S, -1)[:, :NB]
    L = lib()
    L.mi355_softbuffer_get_cb_crc.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    g_cb = np.zeros((2 * S, 16), np.uint8)
    for t in range(2 * S):
        row = np.zeros(rx.pool.max_cb, np.uint8)
        L.mi355_softbuffer_get_cb_crc(rx.pool.h, t, row.ctypes.data, None)
        g_cb[t] = row[:16]
    cols = np.r_[0:K, K + 32:2 * K + 32, 2 * K + 64:3 * K + 64, 3 * K + 96:3 * K + 108]
    dec = oracle.RefTdec()
    legs = {}
    t0 = time.perf_counter()
    for leg, bufs in (("avx2_chain", cpu_bufs), ("avx2_decoder_on_gpu_softbuffers", gpu_bufs)):
        tb_agree = pay_agree = its_agree = cb_agree = ok_ref = 0
        dis = []
        for t in range(2 * S):
            tb_ok, data, cb_ok, cb_its = oracle.ref_dlsch_decode_cbs(np.ascontiguousarray(bufs[t]), K, TBS, max_half,
                                                                    dec)
            ok_ref += int(tb_ok)
            same_crc = tb_ok == bool(g_crc[t])
            same_pay = (not tb_ok) or np.array_equal(data[:NB], g_pay[t])
            same_its = abs(float(cb_its.sum()) / ncb_tb - g_its[t]) < 1e-4
            same_cb = np.array_equal(cb_ok, g_cb[t] != 0)
            tb_agree += int(same_crc)
            pay_agree += int(same_crc and same_pay)
            its_agree += int(same_its)
            cb_agree += int((cb_ok == (g_cb[t] != 0)).sum())
            if not (same_crc and same_pay and same_its and same_cb):
                d = np.abs(cpu_bufs[t][:, cols].astype(np.int32) - gpu_bufs[t][:, cols].astype(np.int32))
                dis.append({"tb": t, "ref_crc": tb_ok, "gpu_crc": bool(g_crc[t]),
                            "ref_half_its": round(float(cb_its.sum()) / ncb_tb, 4), "gpu_half_its": round(g_its[t], 4),
                            "cbs_flag_differ": [int(c) for c in np.nonzero(cb_ok != (g_cb[t] != 0))[0]],
                            "softbuffer_entries_differing": int((d > 0).sum()), "max_abs_llr_diff": int(d.max())})
        legs[leg] = {"tbs": 2 * S, "ref_crc_ok": ok_ref, "gpu_crc_ok": int(g_crc.sum()),
                     "tb_crc_agree": tb_agree, "payload_agree": pay_agree, "tb_iterations_agree": its_agree,
                     "cb_crc_flags_agree": f"{cb_agree}/{2 * S * ncb_tb}", "disagreements": dis[:24],
                     "disagreeing_tbs": len(dis)}
    d_all = np.abs(cpu_bufs[:, :, cols].astype(np.int32) - gpu_bufs[:, :, cols].astype(np.int32))
    dis = legs["avx2_chain"]["disagreements"]
    return {"subframes": S, "tbs": 2 * S, "max_half_iterations": max_half,
            "front_kind": "reference AVX2 stages (predecoding MMSE+CSI, demapper, descrambler, rate dematcher), "
                          "restated float OFDM / estimator",
            "softbuffer_entries_differing_frac": round(float((d_all > 0).mean()), 6),
            "softbuffer_max_abs_diff": int(d_all.max()),
            "legs": legs,
            "crc_agreement_vs_avx2": round(legs["avx2_chain"]["tb_crc_agree"] / (2 * S), 4),
            "every_disagreement_has_differing_softbuffers": all(x["softbuffer_entries_differing"] > 0 for x in dis),
            "cpu_seconds": round(time.perf_counter() - t0, 2)}


def pg_rank(pg) -> int:
    return pg.get_rank() if pg is not None else 0


# ====================================================================================== turbo only (configs[1])

def make_cb_pool(K, n, ebno, seed):
    """n code blocks: random bits -> product turbo encoder (mi355_tcod_encode_host) -> BPSK/AWGN at Eb/N0 (test
    units, turbodecoder_test.c:236-247) -> int16(100*llr) in the 16-window sub-block softbuffer layout."""
    from srsran_amd import enb_dl
    L = enb_dl._declare()
    L.mi355_tcod_encode_host.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    rng = np.random.default_rng(seed)
    nsb = 16 if (K > 800 and K % 16 == 0) else (8 if (K > 400 and K % 8 == 0) else 0)
    assert nsb, "tdec workload uses the windowed layout"
    Lw = K // nsb
    stride = tdec_stride(K)
    pool = np.zeros((n, stride), np.int16)
    sigma = 10 ** (-(ebno + 10 * np.log10(1 / 3)) / 20)
    m = np.arange(K)
    pos = (m % Lw) * nsb + m // Lw
    for i in range(n):
        bits = rng.integers(0, 2, K, dtype=np.uint8)
        enc = np.zeros(3 * K + 12, np.uint8)
        assert L.mi355_tcod_encode_host(bits.ctypes.data, K, enc.ctypes.data) == 0
        y = np.where(enc.astype(bool), 1.0, -1.0) + sigma * rng.standard_normal(enc.size)
        llr = np.trunc(100 * y).clip(-32768, 32767).astype(np.int16)
        for s in range(3):
            pool[i, s * (K + 32) + pos] = llr[s: 3 * K: 3]
        pool[i, 3 * (K + 32): 3 * (K + 32) + 12] = llr[3 * K:]
    return pool


def tdec_stride(K):
    """int16 per code-block buffer of the tdec workload: the windowed layout (3 (K+32) + 12) rounded up to 8, so
    every buffer is 16-byte aligned as the softbuffer pool's are (the MAP kernel's 16-byte loads need it)."""
    return (3 * (K + 32) + 12 + 7) // 8 * 8


def run_tdec(args, world, rank, local, pg):
    from srsran_amd import lib
    from srsran_amd.tdec import DeviceBuffer, TdecBatch
    K, nh, ncb = args.K, args.nhalf, args.ncb
    stride = tdec_stride(K)
    pool = make_cb_pool(K, args.pool, args.ebno, seed=shard_seed(rank))
    host = np.ascontiguousarray(np.tile(pool, (ncb // args.pool + 1, 1))[:ncb])
    d_in = DeviceBuffer(host.nbytes, local).upload(host)
    del host
    d_out = DeviceBuffer(ncb * (K // 8), local)
    dec = TdecBatch(local)

    def step():
        dec.run_dev(d_in.ptr, stride, ncb, K, nh, d_out.ptr)

    for _ in range(args.warmup):
        step()
    lib().mi355_device_sync()
    got = np.zeros((ncb, K // 8), np.uint8)
    d_out.download(got)
    barrier(pg, local)
    lib().mi355_device_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    lib().mi355_device_sync()
    barrier(pg, local)
    dt = max_over_ranks(pg, local, time.perf_counter() - t0)
    dec.set_profiling(True)
    for _ in range(2):
        step()
    kms, kl = dec.kernel_stats()
    # the kernel's bandwidth-only clone (mi355_tdec_set_diag(20): same grid, loads, checkpoint stores, extrinsic
    # scatter, one xor per trellis step): the time this schedule's memory traffic alone takes on this box
    old = lib().mi355_tdec_set_diag(20)
    d_junk = DeviceBuffer(ncb * (K // 8), local)  # the clone's decisions are meaningless: kept out of d_out
    for _ in range(2):
        dec.run_dev(d_in.ptr, stride, ncb, K, nh, d_junk.ptr)
    cms, cl = dec.kernel_stats()
    lib().mi355_tdec_set_diag(old)
    d_junk.free()
    dec.set_profiling(False)
    roof, valu = tdec_roofline(kms, kl, ncb, K, "tdec")
    if cl:
        clone = cms / cl
        roof["schedule_clone_ms"] = round(clone, 4)
        roof["schedule_frac"] = round(clone / roof["avg_launch_ms"], 4)
        roof["schedule_note"] = ("bandwidth-only clone of tdec_win_halfit (MI355_TDEC_DIAG 20) over the same "
                                 f"{ncb:,}-CB launches: schedule_frac = clone time / real time (1.0 = the trellis math "
                                 "is fully hidden under this schedule's memory traffic)")
    cb_s = world * ncb * args.steps / dt
    res = {
        "metric": METRIC, "value": round(cb_s * K / 1e6, 1), "unit": "Mbps", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16", "data": "synthetic",
        "config": {"workload": f"batched turbo decode (configs[1]): {ncb} x K={K} code blocks per GPU, {nh} "
                               f"half-iterations, AUTO 16-window bit-exact, Eb/N0 {args.ebno}",
                   "code_blocks_per_gpu": ncb, "K": K, "half_iterations": nh, "parallelism": f"dp{world}"},
        "code_blocks_per_s": round(cb_s, 1), "roofline": roof, "roofline_valu": valu,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle
        nthreads, hostinfo = host_cores()
        kind = "reference" if oracle.ref_available() else "port"
        fn = oracle.ref().ref_tdec_run_batch if kind == "reference" else oracle.lib().orc_tdec_run_batch
        sub = pool[: min(args.pool, 256)]
        out = np.zeros((sub.shape[0], K // 8), np.uint8)
        legs = {}
        for nt, n_cb in ((1, 16), (nthreads, sub.shape[0])):
            reps, t1 = 0, time.perf_counter()
            while True:
                fn(sub[:n_cb], stride, n_cb, K, nh, out[:n_cb], nt)
                reps += 1
                if time.perf_counter() - t1 >= min(args.cpu_seconds, 4.0):
                    break
            legs[nt] = (reps * n_cb, time.perf_counter() - t1)
        n, dtc = legs[nthreads]
        n1, dt1 = legs[1]
        res["cpu_baseline"] = {"value": round(n * K / dtc / 1e6, 2), "unit": "Mbps", "cb_per_s": round(n / dtc, 1),
                               "cores": nthreads, "kind": kind, "host": hostinfo,
                               "one_thread": {"cb_per_s": round(n1 / dt1, 1),
                                              "us_per_cb_halfit": round(dt1 / n1 / nh * 1e6, 2)},
                               "sample": f"{n} x K={K} CBs, {nh} half-its, {nthreads} threads, {dtc:.2f} s; "
                                         f"{n1} CBs on 1 thread, {dt1:.2f} s"}
        res["parity_vs_cpu"] = bool(np.array_equal(got[: out.shape[0]], out))
    return res


# ====================================================================================== eNodeB generator (8f row 2)

def run_enb(args, world, rank, local, pg):
    """The GPU eNodeB generator on the TM4 batch: payloads resident in HBM -> put_pdsch (DL-SCH encode, QAM256,
    precoding, RE map) -> put_refs -> crossed 2x2 channel + AWGN -> gen_signal (IFFT + CP), B subframes per step.
    Parity: the last step's I/Q decodes through the product's UE chain with every payload (checked after timing)."""
    from srsran_amd import enb_dl, lib
    from srsran_amd import pdsch as P
    from srsran_amd.tdec import DeviceBuffer
    from srsran_amd.ue_dl import symbol_sz
    cell = tm4_setup()
    B = args.subframes
    G, N = 14 * 12 * cell.nof_prb, symbol_sz(cell.nof_prb)
    sf_len = 15 * N
    rng = np.random.default_rng(shard_seed(rank))
    payloads = rng.integers(0, 256, (B, 2, NB), dtype=np.uint8)
    d_pl = DeviceBuffer(payloads.nbytes, local).upload(payloads)
    d_tx = DeviceBuffer(B * 2 * G * 8, local)
    d_rx = DeviceBuffer(B * 2 * G * 8, local)
    d_iq = DeviceBuffer(B * 2 * sf_len * 8, local)
    lib().mi355_memset_dev(d_tx.ptr, 0, B * 2 * G * 8)
    enb = enb_dl.EnbDl(cell, local)
    cfg_sf = {sf: tm4_cfg(P, cell, sf) for sf in range(10)}
    tx = [d_tx.ptr + (i * 2 + p) * G * 8 for i in range(B) for p in range(2)]
    rx = [d_rx.ptr + (i * 2 + r) * G * 8 for i in range(B) for r in range(2)]
    iq = [d_iq.ptr + (i * 2 + r) * sf_len * 8 for i in range(B) for r in range(2)]
    jobs = []
    for i in range(B):
        j = enb_dl.EnbPdschJob()
        j.sf.tti, j.sf.cfi = i % 10, 1
        j.cfg = cfg_sf[i % 10]
        for t in range(2):
            j.data[t] = d_pl.ptr + (i * 2 + t) * NB
        for p in range(2):
            j.sf_symbols[p] = tx[2 * i + p]
        jobs.append(j)
    ttis = (C.c_uint32 * B)(*[i % 10 for i in range(B)])
    jobs = (enb_dl.EnbPdschJob * B)(*jobs)
    tx, rx, iq = [(C.c_void_p * len(v))(*v) for v in (tx, rx, iq)]
    H = np.array([[1, 1], [1, -1]], np.complex64)
    sigma = math.sqrt(10 ** (-args.snr / 10) / 2)

    def step(k):
        enb.put_pdsch(jobs)
        enb.put_refs(ttis, tx)
        enb.channel(tx, rx, 2, H, sigma, 1000003 * shard_seed(rank) + k)
        enb.gen_signal(rx, iq)

    for k in range(args.warmup):
        step(k)
    lib().mi355_device_sync()
    barrier(pg, local)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    lib().mi355_device_sync()
    barrier(pg, local)
    dt = max_over_ranks(pg, local, time.perf_counter() - t0)
    ok = decode_check(cell, B, d_iq, payloads, local)
    ok_all = int(sum_over_ranks(pg, local, ok))
    mbps = whole_job_rate(world, B * 2 * TBS, args.steps, dt) / 1e6
    # algorithmic HBM bytes per subframe of the chain: payload in, codeword bits out + in, PDSCH and
    # CRS REs out, channel grids in + out, IFFT grids in + I/Q out
    nre_pdsch = 2 * 14400
    per_sf = 2 * NB + 2 * 2 * 115200 + 2 * nre_pdsch * 8 + 2 * 800 * 8 + 2 * 2 * G * 8 + 2 * G * 8 + 2 * sf_len * 8
    ach = B * per_sf * args.steps / dt / 1e9
    return {
        "metric": "PDSCH encoded Mbps (GPU eNodeB generator), 20 MHz TM4 QAM256", "value": round(mbps, 1),
        "unit": "Mbps", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8+fp32", "data": "synthetic",
        "config": {"workload": f"srslte_enb_dl put_pdsch + put_refs + crossed 2x2 channel + gen_signal for {B} TM4 "
                               "QAM256 subframes/GPU/step (2 x TBS 97896, 32 CBs of K=6144 each), payloads in HBM",
                   "subframes_per_gpu": B, "parallelism": f"dp{world}"},
        "subframes_per_s": round(world * B * args.steps / dt, 1),
        "decoded_back_ok_tbs": f"{ok_all}/{2 * B * world}",
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(ach / 8000.0, 4), "traffic": None, "kernel": "whole generator chain",
                     "algorithmic_bytes_per_subframe": per_sf},
    }


def decode_check(cell, B, d_iq, payloads, device):
    """CRC-ok TBs with the right payload when the I/Q in d_iq (B x 2 x sf_len) goes through mi355_ue_dl_decode_batch."""
    from srsran_amd import pdsch as P
    from srsran_amd.dlsch import SoftbufferPool
    from srsran_amd.tdec import DeviceBuffer
    from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg, symbol_sz
    G, sf_len, plen = 14 * 12 * cell.nof_prb, 15 * symbol_sz(cell.nof_prb), NB + 16
    ue = UeDl(cell, 2, device)
    d_grid = DeviceBuffer(B * 2 * G * 8, device)
    d_ce = DeviceBuffer(B * 4 * G * 8, device)
    d_pay = DeviceBuffer(B * 2 * plen, device)
    pool = SoftbufferPool(2 * B, max_cb=16, device=device)
    jobs, sfs, cfgs = (DlSfJob * B)(), (P.DlSfCfg * B)(), (P.PdschCfg * B)()
    pays = (C.c_void_p * (2 * B))()
    for i in range(B):
        j = jobs[i]
        j.tti = i % 10
        for r in range(2):
            j.in_buffer[r] = d_iq.ptr + (i * 2 + r) * sf_len * 8
            j.sf_symbols[r] = d_grid.ptr + (i * 2 + r) * G * 8
            for p in range(2):
                j.ce[p][r] = d_ce.ptr + (i * 4 + p * 2 + r) * G * 8
        sfs[i] = P.DlSfCfg(i % 10, 1)
        cfgs[i] = tm4_cfg(P, cell, i % 10, softbuffers=(2 * i, 2 * i + 1))
        pays[2 * i], pays[2 * i + 1] = d_pay.ptr + 2 * i * plen, d_pay.ptr + (2 * i + 1) * plen
    _chest, res = ue.decode(pool, list(jobs), list(sfs), list(cfgs), default_chest_cfg(), list(pays))
    host = d_pay.download(np.zeros(B * 2 * plen, np.uint8)).reshape(B, 2, plen)
    ok = 0
    for i in range(B):
        for t in range(2):
            if res[2 * i + t].crc and np.array_equal(host[i, t, :NB], payloads[i, t]):
                ok += 1
    return ok


# ====================================================================================== plumbing dry run (CPU)

def run_plumbing(args, world, rank, local, pg):
    """CPU dry run of the multi-GPU plumbing (launcher, contiguous sharding, barriers, max-over-ranks, CRC-bitmap
    gather) with gloo: NO decoding happens -- each rank fabricates the CRC bits of its shard from the subframe index
    (TB t of subframe i "fails" iff (i * 7 + t) % 13 == 0) so the gathered bitmap's order can be checked."""
    T = args.total_subframes or world * args.subframes
    lo, hi = shard_range(T, world, rank) if args.total_subframes else (rank * args.subframes, (rank + 1) * args.subframes)
    fan = None
    if args.fanout:  # rank 0 fabricates every shard's "I/Q" by global index and scatters it
        import torch
        assert not args.total_subframes, "--fanout uses equal shards of --subframes"
        B, SFB = args.subframes, 64
        full = torch.from_numpy(plumbing_iq(0, world * B, SFB).reshape(world, B * SFB)) if rank == 0 else None
        recv = torch.empty(B * SFB, dtype=torch.uint8)
    barrier(pg, local)
    t0 = time.perf_counter()
    if args.fanout:
        fanout_scatter(pg, full, recv)
    i = np.arange(lo, hi, dtype=np.int64)
    bits = np.stack([(i * 7 + t) % 13 != 0 for t in range(2)], axis=1).reshape(-1).astype(np.uint8)
    time.sleep(0.02 * (rank + 1))
    barrier(pg, local)
    dt = max_over_ranks(pg, local, time.perf_counter() - t0)
    g = gather_bitmap(pg, local, bits)
    if args.fanout:
        got = recv.numpy().reshape(B, SFB)
        eq = int(sum_over_ranks(pg, local, float(np.array_equal(got, plumbing_iq(lo, B, SFB)))))
        dig = gather_bytes(pg, local, hashlib.sha1(got.tobytes()).digest(), 20)
        if rank == 0:
            want = [hashlib.sha1(plumbing_iq(r * B, B, SFB).tobytes()).digest() for r in range(world)]
            fan = {"ranks_equal_local_synthesis": eq, "shard_sha1_match": dig == want,
                   "bytes_per_subframe": SFB, "bytes_scattered_per_step": (world - 1) * B * SFB}
    return {"fanout": fan,"metric": "plumbing dry run (no decoding)", "value": None, "unit": None, "n_gpus": world,
            "steps": 1, "warmup": 0, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "scaling": "weak" if not args.total_subframes else "strong", "vs_baseline": None, "dtype": None,
            "data": "synthetic", "config": {"workload": "plumbing", "total_subframes": T,
                                            "parallelism": f"dp{world}"},
            "shard": [lo, hi], "crc_bitmap": bitmap_summary(g, T) if rank == 0 else None,
            "bitmap_bits": g.tolist() if (rank == 0 and T <= 4096) else None}


def main():
    args = parse()
    self_launch(args)
    world, rank, local, pg = dist_setup(args.gpus)
    if args.workload == "tdec":
        res = run_tdec(args, world, rank, local, pg)
    elif args.workload == "enb":
        res = run_enb(args, world, rank, local, pg)
    elif args.workload == "plumbing":
        res = run_plumbing(args, world, rank, local, pg)
    elif args.workload == "siso_qpsk":
        res = run_siso(args, world, rank, local, pg)
    elif args.fanout:
        res = run_pdsch_fanout(args, world, rank, local, pg)
    else:
        res = run_pdsch(args, world, rank, local, pg)
    if rank == 0:
        # (numpy scalars in the result -- counts, flags -- as plain JSON numbers)
        print(json.dumps(res, default=lambda o: o.item() if hasattr(o, "item") else str(o)), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
