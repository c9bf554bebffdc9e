#!/usr/bin/env python3
"""bench.py -- PDSCH receive on MI355X: decoded Mbps + code blocks/s on 20 MHz TM4 2x2 QAM256 subframes
(BASELINE.json metric; configs[3] at N = 1, configs[4] as the weak-scaling multi-GPU run).

Workload (one "step", per GPU): B subframes (default 2048 = 65,536 code blocks) of 100 PRB, 2 ports x 2 rx
antennas, CFI 1, TM4 closed-loop spatial multiplexing with 2 codewords (codebook 0), MCS 27 QAM256 with
TBS 97,896 per codeword (C = 16 x K = 6144), MMSE equaliser with CSI weighting (srsUE defaults), max 10
turbo half-iterations with CRC early stopping.  The step runs the whole srslte_ue_dl chain from
time-domain I/Q already resident in HBM:
    softbuffer reset (new TBs) -> OFDM demodulation (2 x 14 x 1536-pt DFT) -> CRS channel estimation
    (AVERAGE, Gauss, REFS noise) -> RE extraction + MMSE + demap + descramble + CSI -> rate dematching ->
    turbo decoding with per-CB CRC early stop -> TB CRC.
Synthetic data (generated before the timed region): random payloads -> the product's GPU eNodeB generator
(include/srsran_amd/enb_dl.h: DL-SCH encode, QAM256, TM4 precoding, CRS) -> phy_dl_test's crossed 2x2 channel
[[1,1],[1,-1]] + AWGN (40 dB) -> IFFT + CP; every subframe of the batch distinct (sf_idx cycling 0..9), seeded
per rank.  --gen host: D distinct subframes from the host encoder tiled over the batch (the earlier data).

    python bench.py [--gpus N --steps K --warmup W]            # N > 1: launched by torch.distributed.run
    python bench.py --workload tdec                            # configs[1]: batched turbo decode only
    python bench.py --workload ue_dl                           # + PCFICH / PDCCH blind search -> DCI -> grant
                                                               #   (phy_dl_test.c:194-247 work_ue per subframe)

Multi-GPU: weak scaling -- every rank decodes its own B subframes (independent subframes shard with no
data-path collective); ranks only meet at the timing barriers and the max-over-ranks reduction.

Prints ONE JSON line on rank 0 (schema: DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # lane-ops/s: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz
# the MAP kernel's instructions are packed int16 (v_pk_add_i16 clamp / v_pk_max_i16), which issue at half that
# rate on gfx950: tools/microbench/valu_rate.hip measured 0.555 wave-instr/ns/SIMD (profiles/r01c_valu_rate.txt)
VALU_PK_I16_TOPS = 0.555 * 64 * 1024 / 1e3
METRIC = "PDSCH decoded Mbps + code-blocks/sec, 20 MHz TM4 QAM256, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["pdsch", "ue_dl", "tdec", "enb"], default="pdsch",
                    help="pdsch: known grants (decode_batch); ue_dl: phy_dl_test's work_ue with the PCFICH / PDCCH "
                         "blind search deriving every grant (find_and_decode); tdec: configs[1]; enb: the GPU "
                         "eNodeB generator (encode side, SURVEY 8f row 2)")
    ap.add_argument("--subframes", type=int, default=2048, help="TM4 subframes per GPU per step")
    ap.add_argument("--gen", choices=["device", "host"], default="device",
                    help="device: every subframe of the batch distinct, synthesised by the product's GPU eNodeB "
                         "generator (mi355_enb_dl_*); host: --distinct subframes from the host encoder, tiled")
    ap.add_argument("--distinct", type=int, default=20, help="--gen host: distinct synthetic subframes tiled")
    ap.add_argument("--snr", type=float, default=40.0)
    ap.add_argument("--ncb", type=int, default=65536, help="tdec workload: code blocks per GPU per step")
    ap.add_argument("--K", type=int, default=6144)
    ap.add_argument("--nhalf", type=int, default=8)
    ap.add_argument("--ebno", type=float, default=2.0)
    ap.add_argument("--pool", type=int, default=256, help="tdec workload: distinct code blocks tiled")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip the per-stage and MAP-kernel probes (profiling runs)")
    return ap.parse_args()


def dist_backend() -> str:
    """RCCL ("nccl") on the GPU node; BENCH_DIST_BACKEND=gloo runs the same plumbing on CPU (tests/test_dist.py)."""
    return os.environ.get("BENCH_DIST_BACKEND", "nccl")


def dist_setup():
    """One process per GPU (torch.distributed.run): the ranks share nothing but the timing barrier and the
    max-over-ranks reduction -- subframes are independent, so there is no data-path collective."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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


def max_over_ranks(pg, local, v: float) -> float:
    if pg is None:
        return v
    import torch
    dev = f"cuda:{local}" if dist_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(pg, local, v: float) -> float:
    if pg is None:
        return v
    import torch
    dev = f"cuda:{local}" if dist_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def shard_seed(rank: int) -> int:
    """Each rank synthesises its own subframes (weak scaling: per-GPU work fixed as N grows)."""
    return 4242 + rank


def whole_job_rate(world: int, units_per_rank: int, steps: int, dt_max: float) -> float:
    """Units of all ranks over the slowest rank's time (value = whole-job aggregate)."""
    return world * units_per_rank * steps / dt_max


def load_pmc():
    p = os.path.join(ROOT, "profiles", "tdec_pmc_traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except Exception:
            return None
    return None


def tdec_roofline(ms, launches, ncb, K):
    """Roofline of the MAP half-iteration kernel: algorithmic bytes per CB-half-iteration = DEC1 reads S, a1,
    P0 and writes e; DEC2 reads e, P1 and writes a1 (int16 x K each) -> (4 + 3) / 2 * 2K on average."""
    bytes_cb = 3.5 * 2 * K
    avg = ms / max(launches, 1)
    achieved = bytes_cb * ncb / (avg / 1e3) / 1e9
    pmc = load_pmc() or {}
    traffic = pmc.get("bytes_per_launch") if pmc.get("launch_ncb") == ncb else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "tdec_win_halfit<16,8>",
            "avg_launch_ms": round(avg, 4), "algorithmic_bytes_per_launch": int(bytes_cb * ncb),
            "cbs_per_launch": ncb}
    valu = None
    if pmc.get("valu_insts_per_launch") and pmc.get("launch_ncb") == ncb:
        rate = pmc["valu_insts_per_launch"] * 64 / (avg / 1e3) / 1e12
        valu = {"achieved": round(rate, 2), "peak": round(VALU_PEAK_TOPS, 1), "unit": "T lane-instr/s",
                "frac": round(rate / VALU_PEAK_TOPS, 4), "peak_packed_i16": round(VALU_PK_I16_TOPS, 1),
                "frac_packed_i16": round(rate / VALU_PK_I16_TOPS, 4),
                "source": "SQ_INSTS_VALU, profiles/tdec_pmc_traffic.json; packed-int16 issue rate measured"}
    return roof, valu


# ====================================================================================== PDSCH (configs[3])

def tm4_setup(nof_prb=100, cell_id=1):
    from srsran_amd import pdsch as P
    cell = P.make_cell(nof_prb, 2, cell_id)
    return cell


def tm4_cfg(P, cell, sf_idx, rnti=0x1234, softbuffers=(0, 1)):
    prb = np.ones((2, cell.nof_prb), np.uint8)
    g = P.make_grant(cell, prb, 1, sf_idx, P.TXSCHEME_SPATIALMUX, 2,
                     [dict(mod=P.MOD_256QAM, tbs=97896, rv=0, cw_idx=0),
                      dict(mod=P.MOD_256QAM, tbs=97896, rv=0, cw_idx=1)], pmi=0)
    cfg = P.PdschCfg()
    cfg.grant = g
    cfg.rnti = rnti
    cfg.decoder_type = P.MIMO_DECODER_MMSE
    cfg.csi_enable = 1
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


def synth_tm4(cell, D, snr_db, seed, ctrl=False):
    """D distinct subframes as time-domain I/Q (D, 2 rx, 15*N) + payloads, via the product encoder (with ctrl: the
    PCFICH (CFI 1) and the subframe's DCI on the PDCCH too)."""
    from srsran_amd import enb_dl
    from srsran_amd import pdsch as P
    from srsran_amd.ue_dl import symbol_sz
    rng = np.random.default_rng(seed)
    nre = 12 * cell.nof_prb
    N = symbol_sz(cell.nof_prb)
    cp0, cp1 = int(math.ceil(160 * N / 2048)), int(math.ceil(144 * N / 2048))
    iq = np.zeros((D, 2, 15 * N), np.complex64)
    payloads = []
    sigma = math.sqrt(10 ** (-snr_db / 10) / 2)
    for d in range(D):
        sf = d % 10
        cfg = tm4_cfg(P, cell, sf)
        pl = [rng.integers(0, 256, 97896 // 8, dtype=np.uint8) for _ in range(2)]
        payloads.append(pl)
        grids = np.zeros((2, 14 * nre), np.complex64)
        enb_dl.pdsch_encode(cell, P.DlSfCfg(sf, 1), cfg, pl, grids)
        enb_dl.put_refs(cell, sf, grids)
        if ctrl:
            from srsran_amd import pdcch as Dc
            Dc.encode_ctrl_host(cell, sf, 1, [tm4_dci_msg(cell, sf)], grids)
        # phy_dl_test crossed channel: rx0 = p0 + p1, rx1 = p0 - p1, plus AWGN per RE
        y = np.stack([grids[0] + grids[1], grids[0] - grids[1]]).reshape(2, 14, nre)
        y = y + sigma * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
        for r in range(2):
            for s in range(14):
                sl, l = divmod(s, 7)
                X = np.zeros(N, np.complex128)
                X[N - nre // 2:] = y[r, s, : nre // 2]
                X[1: nre // 2 + 1] = y[r, s, nre // 2:]
                t = np.fft.ifft(X)
                cp = cp0 if l == 0 else cp1
                start = sl * (15 * N // 2) + (0 if l == 0 else cp0 + N + (l - 1) * (N + cp1))
                iq[d, r, start: start + cp] = t[N - cp:]
                iq[d, r, start + cp: start + cp + N] = t
    return iq, payloads


def synth_tm4_device(cell, B, snr_db, seed, device, ctrl, d_iq, sf_len, chunk=256):
    """B distinct subframes straight into d_iq (B x 2 rx x sf_len complex) with the product's GPU eNodeB generator:
    random payloads -> mi355_enb_dl_put_pdsch_batch (TB/CB CRC, turbo coding, rate matching, scrambling, QAM256,
    TM4 precoding, RE map) + put_refs (CRS) [+ the host-encoded PCFICH/PDCCH row of the subframe index, CFI 1] ->
    phy_dl_test's crossed 2x2 channel + AWGN (mi355_channel_grid_batch) -> gen_signal (IFFT + CP).  Returns the
    payloads (B, 2, tbs/8)."""
    from srsran_amd import enb_dl, lib
    from srsran_amd import pdsch as P
    from srsran_amd.tdec import DeviceBuffer
    rng = np.random.default_rng(seed)
    G, nre, nb = 14 * 12 * cell.nof_prb, 12 * cell.nof_prb, 97896 // 8
    payloads = rng.integers(0, 256, (B, 2, nb), dtype=np.uint8)
    d_pl = DeviceBuffer(payloads.nbytes, device).upload(payloads)
    enb = enb_dl.EnbDl(cell, device)
    chunk = min(chunk, B)
    d_tx = DeviceBuffer(chunk * 2 * G * 8, device)
    d_rx = DeviceBuffer(chunk * 2 * G * 8, device)
    cfg_sf = {sf: tm4_cfg(P, cell, sf) for sf in range(10)}
    rows = None
    if ctrl:  # symbol 0 (CFI 1) of each port: CRS + PCFICH + the subframe's DCI on the PDCCH
        from srsran_amd import pdcch as Dc
        rows = {}
        for sf in range(10):
            g = np.zeros((2, G), np.complex64)
            enb_dl.put_refs(cell, sf, g)
            Dc.encode_ctrl_host(cell, sf, 1, [tm4_dci_msg(cell, sf)], g)
            rows[sf] = np.ascontiguousarray(g[:, :nre])
    H = np.array([[1, 1], [1, -1]], np.complex64)
    sigma = math.sqrt(10 ** (-snr_db / 10) / 2)
    for c0 in range(0, B, chunk):
        n = min(chunk, B - c0)
        lib().mi355_memset_dev(d_tx.ptr, 0, n * 2 * G * 8)
        jobs = []
        tx = [d_tx.ptr + (k * 2 + p) * G * 8 for k in range(n) for p in range(2)]
        rx = [d_rx.ptr + (k * 2 + r) * G * 8 for k in range(n) for r in range(2)]
        for k in range(n):
            i, sf = c0 + k, (c0 + k) % 10
            j = enb_dl.EnbPdschJob()
            j.sf.tti, j.sf.cfi = sf, 1
            j.cfg = cfg_sf[sf]
            for t in range(2):
                j.data[t] = d_pl.ptr + (i * 2 + t) * nb
            for p in range(2):
                j.sf_symbols[p] = tx[2 * k + p]
            jobs.append(j)
        enb.put_pdsch(jobs)
        enb.put_refs([(c0 + k) % 10 for k in range(n)], tx)
        if ctrl:
            for k in range(n):
                for p in range(2):
                    lib().mi355_memcpy_h2d(tx[2 * k + p], rows[(c0 + k) % 10][p].ctypes.data, nre * 8)
        enb.channel(tx, rx, 2, H, sigma, seed * 1000003 + c0)
        enb.gen_signal(rx, [d_iq.ptr + ((c0 + k) * 2 + r) * sf_len * 8 for k in range(n) for r in range(2)])
    enb.close()
    return payloads


class Tm4Batch:
    """B subframes resident in HBM with their grids, channel estimates, softbuffers and payload buffers."""

    def __init__(self, cell, B, D, snr, seed, device, ctrl=False, gen="host"):
        from srsran_amd import lib
        from srsran_amd import pdsch as P
        from srsran_amd.dlsch import SoftbufferPool
        from srsran_amd.tdec import DeviceBuffer
        from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg
        self.P, self.B, self.D = P, B, D
        self.ctrl = ctrl
        from srsran_amd.ue_dl import symbol_sz
        sf_len = 15 * symbol_sz(cell.nof_prb)
        G = 14 * 12 * cell.nof_prb
        self.G = G
        self.plen = 97896 // 8 + 16
        # every subframe gets its own I/Q buffers, so the OFDM stage streams B inputs from HBM
        self.d_iq = DeviceBuffer(B * 2 * sf_len * 8, device)
        if gen == "device":  # all B subframes distinct, synthesised on the GPU
            self.D = D = B
            self.payloads = synth_tm4_device(cell, B, snr, seed, device, ctrl, self.d_iq, sf_len)
            S = min(B, 10)  # the CPU baseline's sample
            self.iq_host = np.zeros((S, 2, sf_len), np.complex64)
            self.d_iq.download(self.iq_host)
        else:  # D distinct host-encoded subframes tiled over the batch
            self.iq_host, self.payloads = synth_tm4(cell, D, snr, seed, ctrl)
            iq = np.ascontiguousarray(self.iq_host, np.complex64)
            for i in range(B):
                lib().mi355_memcpy_h2d(C.c_void_p(self.d_iq.ptr + i * 2 * sf_len * 8), iq[i % D].ctypes.data,
                                       C.c_size_t(2 * sf_len * 8))
        self.d_grid = DeviceBuffer(B * 2 * G * 8, device)
        self.d_ce = DeviceBuffer(B * 4 * G * 8, device)
        self.d_pay = DeviceBuffer(B * 2 * self.plen, device)
        lib().mi355_memset_dev(self.d_pay.ptr, 0, B * 2 * self.plen)
        self.pool = SoftbufferPool(2 * B, max_cb=16, device=device)
        self.ue = UeDl(cell, 2, device)
        self.chest_cfg = default_chest_cfg()
        self.jobs = (DlSfJob * B)()
        self.sfs = (P.DlSfCfg * B)()
        self.cfgs = (P.PdschCfg * B)()
        self.pays = (C.c_void_p * (2 * B))()
        self.res_chest = None
        cfg_sf = {sf: tm4_cfg(P, cell, sf) for sf in range(10)}
        for i in range(B):
            d = i % D
            j = self.jobs[i]
            j.tti = d % 10
            for r in range(2):
                j.in_buffer[r] = self.d_iq.ptr + (i * 2 + r) * sf_len * 8
                j.sf_symbols[r] = self.d_grid.ptr + (i * 2 + r) * G * 8
                for p in range(2):
                    j.ce[p][r] = self.d_ce.ptr + (i * 4 + p * 2 + r) * G * 8
            self.sfs[i] = P.DlSfCfg(d % 10, 1)
            self.cfgs[i] = cfg_sf[d % 10]
            self.cfgs[i].softbuffer[0], self.cfgs[i].softbuffer[1] = 2 * i, 2 * i + 1
            self.pays[2 * i] = self.d_pay.ptr + (2 * i) * self.plen
            self.pays[2 * i + 1] = self.d_pay.ptr + (2 * i + 1) * self.plen
        from srsran_amd.ue_dl import ChestRes, _declare
        self.L = _declare()
        self.L.mi355_softbuffer_reset_range.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        self.chest = (ChestRes * B)()
        self.res = (P.PdschRes * (2 * B))()
        if ctrl:
            from srsran_amd import pdcch as Dc
            self.Lc = Dc._declare()
            u = Dc.UeDlCfg()
            u.tm, u.use_tbs_index_alt = Dc.TM4, 1
            self.ue_cfgs = (Dc.UeDlCfg * B)(*([u] * B))
            self.ctrl_res = (Dc.CtrlRes * B)()
            self.dci = (Dc.DciDl * (B * Dc.MAX_DCI_MSG))()

    def step(self, stages=None):
        """One batch: new-TB softbuffer reset + mi355_ue_dl_decode_batch (OFDM, estimation, PDSCH, DL-SCH).
        With `stages`, the two-call form (decode_fft_estimate, then decode_pdsch) is timed per stage instead."""
        from srsran_amd import check, lib
        t0 = time.perf_counter()
        if self.ctrl:
            # find_and_decode resets each TB's softbuffer itself (ue_dl.c:1522-1529)
            C.memset(self.res, 0, C.sizeof(self.res))
            check(self.Lc.mi355_ue_dl_find_and_decode_batch(self.ue.h, self.pool.h, self.jobs, self.sfs, self.ue_cfgs,
                                                            self.cfgs, C.byref(self.chest_cfg), self.chest, self.pays,
                                                            self.B, self.ctrl_res, self.dci, self.res, None),
                  "ue_dl_find_and_decode_batch")
            return
        check(self.L.mi355_softbuffer_reset_range(self.pool.h, 0, 2 * self.B, None), "softbuffer_reset_range")
        C.memset(self.res, 0, C.sizeof(self.res))
        if stages is None:
            check(self.L.mi355_ue_dl_decode_batch(self.ue.h, self.pool.h, self.jobs, self.sfs, self.cfgs,
                                                  C.byref(self.chest_cfg), self.chest, self.pays, self.B, self.res,
                                                  None), "ue_dl_decode_batch")
            return
        check(self.L.mi355_ue_dl_decode_fft_estimate_batch(self.ue.h, self.jobs, self.B, C.byref(self.chest_cfg),
                                                           self.chest, None), "decode_fft_estimate")
        t1 = time.perf_counter()
        check(self.L.mi355_ue_dl_decode_pdsch_batch(self.ue.h, self.pool.h, self.jobs, self.sfs, self.cfgs,
                                                    self.chest, self.pays, self.B, self.res, None), "decode_pdsch")
        lib().mi355_device_sync()
        t2 = time.perf_counter()
        stages["reset_fft_chest_ms"] = stages.get("reset_fft_chest_ms", 0) + (t1 - t0) * 1e3
        stages["pdsch_decode_ms"] = stages.get("pdsch_decode_ms", 0) + (t2 - t1) * 1e3

    def check_payloads(self):
        """All TBs CRC-ok and every payload equal to what the encoder was given (and, with the control channels,
        exactly one DCI found per subframe)."""
        host = np.zeros(self.B * 2 * self.plen, np.uint8)
        self.d_pay.download(host)
        host = host.reshape(self.B, 2, self.plen)
        ok = 0
        for i in range(self.B):
            for t in range(2):
                r = self.res[2 * i + t]
                dci_ok = not self.ctrl or self.ctrl_res[i].nof_dci == 1
                if dci_ok and r.crc and np.array_equal(host[i, t, : 97896 // 8], self.payloads[i % self.D][t]):
                    ok += 1
        its = float(np.mean([self.res[k].avg_iterations_block for k in range(2 * self.B)]))
        return ok, its


def cpu_baseline_pdsch(batch, nthreads, budget_s, avg_its):
    """CPU reference-path timing on the host cores (rank 0, N = 1), bounded sample:
    front-end (OFDM as a float64 numpy DFT, channel estimation and PDSCH symbol processing by the oracle's C
    restatement of the reference) on S distinct subframes with a thread pool, plus the reference's own AVX2
    turbo decoder (oracle/_ref, compiled from the srsLTE sources) on their 32 x S code blocks -- taken from
    the GPU's softbuffers after rate dematching -- for ceil(avg half-iterations) half-iterations."""
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    from oracle import pdsch_chain as pc
    from oracle import ue_dl_chain as uc
    S = min(batch.D, 10)
    cfgs = [pc.Cfg(nof_prb=100, nof_ports=2, nof_rx=2, cell_id=1, cfi=1, sf_idx=d % 10, scheme=2, nof_layers=2,
                   qm=[8, 8], tbs=[97896, 97896], csi_enable=True) for d in range(S)]

    def front(d):
        grids = np.stack([uc.ofdm_rx_sf(batch.iq_host[d, r], 100) for r in range(2)])
        ce, res = uc.chest_estimate(grids, 100, 2, 1, d % 10)
        return pc.rx_front(cfgs[d], grids, ce, res["noise_estimate"])[2]

    t0 = time.perf_counter()
    reps_f = 0
    with ThreadPoolExecutor(nthreads) as ex:
        while True:
            list(ex.map(front, range(S)))
            reps_f += 1
            if time.perf_counter() - t0 >= budget_s / 2:
                break
    t_front = (time.perf_counter() - t0) / (reps_f * S)  # per subframe, nthreads cores
    # turbo part: the first S subframes' code blocks (softbuffers 0 .. 2S-1) from the device pool
    from srsran_amd import lib
    buf, stride, mcb = C.POINTER(C.c_int16)(), C.c_uint32(), C.c_uint32()
    lib().mi355_softbuffer_pool_buffer.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_int16)),
                                                   C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    lib().mi355_softbuffer_pool_buffer(batch.pool.h, C.byref(buf), C.byref(stride), C.byref(mcb))
    ncb = 2 * S * 16
    host = np.zeros((ncb, stride.value), np.int16)
    lib().mi355_memcpy_d2h(host.ctypes.data, C.cast(buf, C.c_void_p).value, host.nbytes)
    nh = max(1, int(math.ceil(avg_its)))
    kind_t = "reference" if oracle.ref_available() else "port"
    fn = oracle.ref().ref_tdec_run_batch if kind_t == "reference" else oracle.lib().orc_tdec_run_batch
    out = np.zeros((ncb, 6144 // 8), np.uint8)
    t1 = time.perf_counter()
    reps = 0
    while True:
        fn(host, stride.value, ncb, 6144, nh, out, nthreads)
        reps += 1
        if time.perf_counter() - t1 >= budget_s / 2:
            break
    t_tdec = (time.perf_counter() - t1) / (reps * S)  # per subframe
    per_sf = t_front + t_tdec
    bits = 2 * 97896
    return {
        "value": round(bits / per_sf / 1e6, 2), "unit": "Mbps", "cb_per_s": round(32 / per_sf, 1),
        "cores": nthreads, "kind": "port",
        "sample": (f"{S} distinct TM4 subframes: front-end (numpy float64 DFT + oracle C chest/MMSE/demap) "
                   f"{t_front * 1e3:.2f} ms/subframe x {reps_f} passes, reference AVX2 turbo decoder "
                   f"({kind_t}, oracle/_ref) on their {ncb} CBs x {nh} half-iterations {t_tdec * 1e3:.2f} "
                   f"ms/subframe x {reps} passes; {nthreads} threads"),
        "turbo_kind": kind_t,
    }


def run_pdsch(args, world, rank, local, pg):
    from srsran_amd import lib
    from srsran_amd.tdec import DeviceBuffer, TdecBatch
    cell = tm4_setup()
    B = args.subframes
    ctrl = args.workload == "ue_dl"
    b = Tm4Batch(cell, B, min(args.distinct, B), args.snr, seed=shard_seed(rank), device=local, ctrl=ctrl,
                 gen=args.gen)
    for _ in range(args.warmup):
        b.step()
    lib().mi355_device_sync()
    ok, its = b.check_payloads()

    barrier(pg, local)
    lib().mi355_device_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.step()
    lib().mi355_device_sync()
    barrier(pg, local)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(pg, local, dt)
    ok_last, _ = b.check_payloads()

    stages = {}
    roof, valu = None, None
    if args.no_roofline:
        kms = None
    elif not ctrl:
        b.step(stages)
    # dominant kernel: the MAP half-iteration over this batch's 32*B code blocks (the softbuffers hold the
    # rate-dematched LLRs of the last step), 8 half-iterations without early stop, HIP events on its stream
    from srsran_amd.dlsch import _declare as _dd
    L = _dd()
    buf, stride, mcb = C.POINTER(C.c_int16)(), C.c_uint32(), C.c_uint32()
    L.mi355_softbuffer_pool_buffer.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_int16)),
                                               C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.mi355_softbuffer_pool_buffer(b.pool.h, C.byref(buf), C.byref(stride), C.byref(mcb))
    ncb = 2 * B * 16
    if not args.no_roofline:
        d_out = DeviceBuffer(ncb * 768, local)
        dec = TdecBatch(local)
        ptr = C.cast(buf, C.c_void_p).value
        dec.run_dev(ptr, stride.value, ncb, 6144, 8, d_out.ptr)
        dec.set_profiling(True)
        for _ in range(2):
            dec.run_dev(ptr, stride.value, ncb, 6144, 8, d_out.ptr)
        kms, kl = dec.kernel_stats()
        dec.set_profiling(False)
        roof, valu = tdec_roofline(kms, kl, ncb, 6144)

    subframes = world * B * args.steps
    ok_all = int(sum_over_ranks(pg, local, ok_last))  # CRC-ok TBs of the last step, all ranks
    mbps = whole_job_rate(world, B * 2 * 97896, args.steps, dt) / 1e6 * (ok_all / (2 * B * world))
    res = {
        "metric": METRIC, "value": round(mbps, 1), "unit": "Mbps", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32+int16", "data": "synthetic",
        "config": {"workload": f"srslte_ue_dl chain from time-domain I/Q: {B} subframes/GPU/step, 20 MHz (100 PRB), "
                               "TM4 2x2 spatial multiplexing, 2 codewords QAM256 TBS 97896 (C=16, K=6144), "
                               "MMSE+CSI, max 10 half-its with CRC early stop, 40 dB crossed 2x2 channel, " +
                               ("every subframe distinct (GPU eNodeB generator)" if args.gen == "device" else
                                f"{b.D} distinct host-encoded subframes tiled") +
                               ("; grants from the PCFICH/PDCCH blind search (DCI format 2 per subframe, "
                                "find_and_decode = phy_dl_test work_ue)" if ctrl else ""),
                   "subframes_per_gpu": B, "code_blocks_per_gpu": 32 * B, "distinct_subframes": b.D,
                   "parallelism": f"dp{world}"},
        "code_blocks_per_s": round(world * 32 * B * args.steps / dt, 1),
        "subframes_per_s": round(subframes / dt, 1),
        "crc_ok_tbs": f"{ok_all}/{2 * B * world}", "avg_half_iterations": round(its, 3),
        "stage_ms": {k: round(v, 3) for k, v in stages.items()},
        "roofline": roof,
    }
    if valu:
        res["roofline_valu"] = valu
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_pdsch(b, min(os.cpu_count() or 1, 16), args.cpu_seconds, its)
    return res


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
    stride = 3 * (K + 32) + 12
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


def run_tdec(args, world, rank, local, pg):
    from srsran_amd import lib
    from srsran_amd.tdec import DeviceBuffer, TdecBatch
    K, nh, ncb = args.K, args.nhalf, args.ncb
    stride = 3 * (K + 32) + 12
    pool = make_cb_pool(K, args.pool, args.ebno, seed=1234 + rank)
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
    dec.set_profiling(False)
    roof, valu = tdec_roofline(kms, kl, ncb, K)
    cb_s = world * ncb * args.steps / dt
    res = {
        "metric": METRIC, "value": round(cb_s * K / 1e6, 1), "unit": "Mbps", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16", "data": "synthetic",
        "config": {"workload": f"batched turbo decode (configs[1]): {ncb} x K={K} code blocks per GPU, {nh} "
                               f"half-iterations, AUTO 16-window bit-exact, Eb/N0 {args.ebno}",
                   "code_blocks_per_gpu": ncb, "K": K, "half_iterations": nh, "parallelism": f"dp{world}"},
        "code_blocks_per_s": round(cb_s, 1), "roofline": roof,
    }
    if valu:
        res["roofline_valu"] = valu
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle
        nthreads = min(os.cpu_count() or 1, 16)
        kind = "reference" if oracle.ref_available() else "port"
        fn = oracle.ref().ref_tdec_run_batch if kind == "reference" else oracle.lib().orc_tdec_run_batch
        sub = pool[: min(args.pool, 256)]
        out = np.zeros((sub.shape[0], K // 8), np.uint8)
        reps, t1 = 0, time.perf_counter()
        while True:
            fn(sub, stride, sub.shape[0], K, nh, out, nthreads)
            reps += 1
            if time.perf_counter() - t1 >= min(args.cpu_seconds, 3.0):
                break
        dtc = time.perf_counter() - t1
        n = reps * sub.shape[0]
        res["cpu_baseline"] = {"value": round(n * K / dtc / 1e6, 2), "unit": "Mbps", "cb_per_s": round(n / dtc, 1),
                               "cores": nthreads, "kind": kind,
                               "sample": f"{n} x K={K} CBs, {nh} half-its, {nthreads} threads, {dtc:.2f} s"}
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
    G, N, nb = 14 * 12 * cell.nof_prb, symbol_sz(cell.nof_prb), 97896 // 8
    sf_len = 15 * N
    rng = np.random.default_rng(shard_seed(rank))
    payloads = rng.integers(0, 256, (B, 2, nb), dtype=np.uint8)
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
            j.data[t] = d_pl.ptr + (i * 2 + t) * nb
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
    # parity: decode the last step's I/Q with the product's UE chain
    ok = decode_check(cell, B, d_iq, payloads, local)
    ok_all = int(sum_over_ranks(pg, local, ok))
    mbps = whole_job_rate(world, B * 2 * 97896, args.steps, dt) / 1e6
    # algorithmic HBM bytes per subframe of the chain: payload in, codeword bits out + in, PDSCH and
    # CRS REs out, channel grids in + out, IFFT grids in + I/Q out
    nre_pdsch = 2 * 14400
    per_sf = 2 * nb + 2 * 2 * 115200 + 2 * nre_pdsch * 8 + 2 * 800 * 8 + 2 * 2 * G * 8 + 2 * G * 8 + 2 * sf_len * 8
    ach = B * per_sf * args.steps / dt / 1e9
    res = {
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
    return res


def decode_check(cell, B, d_iq, payloads, device):
    """CRC-ok TBs with the right payload when the I/Q in d_iq (B x 2 x sf_len) goes through mi355_ue_dl_decode_batch."""
    from srsran_amd import pdsch as P
    from srsran_amd.dlsch import SoftbufferPool
    from srsran_amd.tdec import DeviceBuffer
    from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg, symbol_sz
    G, sf_len, plen = 14 * 12 * cell.nof_prb, 15 * symbol_sz(cell.nof_prb), 97896 // 8 + 16
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
    chest, res = ue.decode(pool, list(jobs), list(sfs), list(cfgs), default_chest_cfg(), list(pays))
    host = d_pay.download(np.zeros(B * 2 * plen, np.uint8)).reshape(B, 2, plen)
    ok = 0
    for i in range(B):
        for t in range(2):
            if res[2 * i + t].crc and np.array_equal(host[i, t, : 97896 // 8], payloads[i, t]):
                ok += 1
    return ok


def main():
    args = parse()
    world, rank, local, pg = dist_setup()
    if args.workload == "tdec":
        res = run_tdec(args, world, rank, local, pg)
    elif args.workload == "enb":
        res = run_enb(args, world, rank, local, pg)
    else:
        res = run_pdsch(args, world, rank, local, pg)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
