"""Batched downlink workloads resident in HBM: the product's GPU eNodeB generator (mi355_enb_dl_*)
synthesising subframes by global index, and the UE side that decodes them through the batched C ABI.  Used by
bench.py (configs[2..4]) and by the GPU tests that run the BASELINE configs and phy_dl_test's matrix at size.

A subframe is described by an `SfPlan` (what srslte_enb_dl would be told: tti, CFI, the PDSCH configuration with
its grant, and optionally the DCI message put on the PDCCH); `DlSource.generate` turns a list of plans into
time-domain I/Q (payloads keyed by the global subframe index -> put_pdsch -> put_refs -> host-encoded control
region -> test channel -> IFFT), `DlReceiver` binds resident subframes to job tables and decodes them with
mi355_ue_dl_decode_batch (known grants) or mi355_ue_dl_find_and_decode_batch (grants from the PDCCH)."""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from . import check, lib
from . import pdsch as P


@dataclass
class SfPlan:
    tti: int                    # subframe index within the frame (tti % 10 is what the chains read)
    cfi: int
    cfg: P.PdschCfg             # grant + rnti + p_a (the transmitter) and the UE's decoder fields
    msg: object = None          # pdcch.DciMsg on the PDCCH (None: no control region beyond the CRS)
    tm: int = 3                 # UE transmission mode index (find_and_decode) ...
    tbs_alt: bool = False       # ... and its 256QAM table flag


def tb_bytes(cfg: P.PdschCfg) -> list[int]:
    return [cfg.grant.tb[t].tbs // 8 if cfg.grant.tb[t].enabled else 0 for t in range(2)]


class DlSource:
    """Up to n_max subframes of one cell resident in HBM (I/Q per rx antenna + the transmitted payloads, `nbytes`
    per TB slot), synthesised on the GPU by global subframe index.  H: (nof_rx, nof_ports) test channel mixing
    the port grids (phy_dl_test's crossed 2x2 [[1,1],[1,-1]], identity for SISO)."""

    def __init__(self, cell: P.Cell, nof_rx: int, n_max: int, nbytes: int, device: int = 0, H=None, chunk=256,
                 iq_buffer=None):
        from . import enb_dl
        from .tdec import DeviceBuffer
        from .ue_dl import symbol_sz
        self.cell, self.nof_rx, self.n_max, self.nbytes, self.device = cell, nof_rx, n_max, nbytes, device
        self.np = cell.nof_ports
        self.sf_len = 15 * symbol_sz(cell.nof_prb)
        self.G, self.nre = 14 * 12 * cell.nof_prb, 12 * cell.nof_prb
        self.H = np.asarray(H if H is not None else np.eye(nof_rx, self.np), np.complex64)
        assert self.H.shape == (nof_rx, self.np)
        # iq_buffer: a caller-owned device buffer (.ptr, .nbytes) to synthesise into (bench.py --fanout: a torch
        # tensor that RCCL scatters from)
        if iq_buffer is not None:
            assert iq_buffer.nbytes >= n_max * nof_rx * self.sf_len * 8
        self.d_iq = iq_buffer if iq_buffer is not None else DeviceBuffer(n_max * nof_rx * self.sf_len * 8, device)
        self.d_pl = DeviceBuffer(n_max * 2 * nbytes, device)
        self.enb = enb_dl.EnbDl(cell, device)
        self.chunk = min(chunk, n_max)
        self.d_tx = DeviceBuffer(self.chunk * self.np * self.G * 8, device)
        self.d_rx = DeviceBuffer(self.chunk * nof_rx * self.G * 8, device)
        self._rows: dict = {}
        self.first, self.n, self.plans = 0, 0, []

    def iq_ptr(self, k: int, r: int) -> int:
        return self.d_iq.ptr + (k * self.nof_rx + r) * self.sf_len * 8

    def pay_ptr(self, k: int, t: int) -> int:
        return self.d_pl.ptr + (k * 2 + t) * self.nbytes

    def _ctrl_rows(self, p: SfPlan) -> np.ndarray:
        """The control region of every port -- cfi OFDM symbols, one more below 10 PRB (SRSLTE_NOF_CTRL_SYMBOLS):
        CRS + PCFICH + the plan's DCI on the PDCCH -- host-encoded once per distinct (tti, cfi, message): the PDSCH
        never occupies it."""
        from . import enb_dl
        from . import pdcch as D
        key = (p.tti % 10, p.cfi, bytes(p.msg) if p.msg is not None else b"")
        row = self._rows.get(key)
        if row is None:
            g = np.zeros((self.np, self.G), np.complex64)
            enb_dl.put_refs(self.cell, p.tti % 10, g)
            D.encode_ctrl_host(self.cell, p.tti % 10, p.cfi, [p.msg] if p.msg is not None else [], g)
            nsym = p.cfi + (1 if self.cell.nof_prb < 10 else 0)
            row = np.ascontiguousarray(g[:, : nsym * self.nre])
            if len(self._rows) < 4096:
                self._rows[key] = row
        return row

    def generate(self, first: int, plans: list[SfPlan], snr_db: float | None, seed: int, fading=None,
                 ctrl: bool = False):
        """Subframes [first, first + len(plans)): payloads keyed by index -> put_pdsch -> put_refs [-> control
        region] -> test channel (H, or `fading`: a srslte_channel_fading_t model string) + AWGN keyed by index
        (snr_db None: no noise, as phy_dl_test) -> IFFT."""
        n = len(plans)
        assert n <= self.n_max
        self.first, self.n, self.plans = first, n, list(plans)
        enb, G = self.enb, self.G
        enb.synth_payloads(self.d_pl.ptr, first, n, 2, self.nbytes, seed)
        sigma = 0.0 if snr_db is None else math.sqrt(10 ** (-snr_db / 10) / 2)
        from . import enb_dl
        for c0 in range(0, n, self.chunk):
            m = min(self.chunk, n - c0)
            lib().mi355_memset_dev(self.d_tx.ptr, 0, m * self.np * G * 8)
            tx = [self.d_tx.ptr + (k * self.np + p) * G * 8 for k in range(m) for p in range(self.np)]
            rx = [self.d_rx.ptr + (k * self.nof_rx + r) * G * 8 for k in range(m) for r in range(self.nof_rx)]
            jobs = (enb_dl.EnbPdschJob * m)()
            for k in range(m):
                pl = plans[c0 + k]
                j = jobs[k]
                j.sf.tti, j.sf.cfi = pl.tti % 10, pl.cfi
                j.cfg = pl.cfg
                for t in range(2):
                    j.data[t] = self.pay_ptr(c0 + k, t)
                for p in range(self.np):
                    j.sf_symbols[p] = tx[self.np * k + p]
            enb.put_pdsch(jobs)
            enb.put_refs([plans[c0 + k].tti % 10 for k in range(m)], tx)
            if ctrl:
                for k in range(m):
                    row = self._ctrl_rows(plans[c0 + k])
                    for p in range(self.np):
                        lib().mi355_memcpy_h2d(tx[self.np * k + p], row[p].ctypes.data, row[p].nbytes)
            if fading is None:
                enb.channel(tx, rx, self.nof_rx, self.H, sigma, seed, first_index=first + c0)
            else:
                enb.fading(tx, rx, self.nof_rx, fading, [1e-3 * (first + c0 + k) for k in range(m)], sigma,
                           (seed * 7919 + first + c0) & 0x7FFFFFFF)
            enb.gen_signal(rx, [self.iq_ptr(c0 + k, r) for k in range(m) for r in range(self.nof_rx)])
        lib().mi355_device_sync()

    def payloads(self, k0: int, n: int) -> np.ndarray:
        """Transmitted payload slots of resident subframes [k0, k0 + n) -> (n, 2, nbytes)."""
        out = np.zeros((n, 2, self.nbytes), np.uint8)
        lib().mi355_memcpy_d2h(out.ctypes.data, self.d_pl.ptr + k0 * 2 * self.nbytes, out.nbytes)
        return out

    def iq_host(self, k0: int, n: int) -> np.ndarray:
        out = np.zeros((n, self.nof_rx, self.sf_len), np.complex64)
        lib().mi355_memcpy_d2h(out.ctypes.data, self.iq_ptr(k0, 0), out.nbytes)
        return out

    def close(self):
        self.enb.close()


class DlReceiver:
    """The UE side of one batch of up to B subframes: srslte_ue_dl_t + softbuffers (2 per subframe) + grids /
    estimates / payload buffers.  Job tables are built per bind (no host work in a timed loop beyond the
    library calls)."""

    def __init__(self, cell: P.Cell, nof_rx: int, B: int, nbytes: int, device: int = 0, ctrl: bool = False,
                 max_cb: int = 16, ce_rows: int = 0):
        from .dlsch import SoftbufferPool
        from .tdec import DeviceBuffer
        from .ue_dl import ChestRes, UeDl, _declare, default_chest_cfg
        self.B, self.ctrl, self.cell, self.nof_rx = B, ctrl, cell, nof_rx
        self.np = cell.nof_ports
        self.G = 14 * 12 * cell.nof_prb
        self.plen = nbytes + 16
        self.d_grid = DeviceBuffer(B * nof_rx * self.G * 8, device)
        self.d_ce = DeviceBuffer(B * self.np * nof_rx * self.G * 8, device)
        self.d_pay = DeviceBuffer(B * 2 * self.plen, device)
        lib().mi355_memset_dev(self.d_pay.ptr, 0, B * 2 * self.plen)
        self.pool = SoftbufferPool(2 * B, max_cb=max_cb, device=device)
        self.ue = UeDl(cell, nof_rx, device)
        self.chest_cfg = default_chest_cfg()
        self.ce_rows = ce_rows  # 1: the AVERAGE estimate's row 0 only (the chain reads nothing else)
        self.ue.set_ce_rows(ce_rows)
        self.L = _declare()
        self.L.mi355_softbuffer_reset_range.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        self.chest = (ChestRes * B)()
        self.res = (P.PdschRes * (2 * B))()
        self.pays = (C.c_void_p * (2 * B))(*[self.d_pay.ptr + k * self.plen for k in range(2 * B)])
        if ctrl:
            from . import pdcch as Dc
            self.Lc = Dc._declare()
            self.ue_cfgs = (Dc.UeDlCfg * B)()
            self.ctrl_res = (Dc.CtrlRes * B)()
            self.dci = (Dc.DciDl * (B * Dc.MAX_DCI_MSG))()

    def grid_ptr(self, k: int, r: int) -> int:
        return self.d_grid.ptr + (k * self.nof_rx + r) * self.G * 8

    def ce_ptr(self, k: int, p: int, r: int) -> int:
        return self.d_ce.ptr + ((k * self.np + p) * self.nof_rx + r) * self.G * 8

    def bind(self, src: DlSource, k0: int, n: int, tb_major: bool = False):
        """Job tables for resident subframes [k0, k0 + n) of src (n <= B); softbuffers 2k, 2k + 1 (tb_major: k and
        B + k, so the first TBs' code blocks are contiguous in the pool)."""
        from .ue_dl import DlSfJob
        assert n <= self.B
        jobs, sfs, cfgs = (DlSfJob * n)(), (P.DlSfCfg * n)(), (P.PdschCfg * n)()
        for k in range(n):
            pl = src.plans[k0 + k]
            j = jobs[k]
            j.tti = pl.tti % 10
            for r in range(self.nof_rx):
                j.in_buffer[r] = src.iq_ptr(k0 + k, r)
                j.sf_symbols[r] = self.grid_ptr(k, r)
                for p in range(self.np):
                    j.ce[p][r] = self.ce_ptr(k, p, r)
            sfs[k] = P.DlSfCfg(pl.tti % 10, pl.cfi)
            cfgs[k] = pl.cfg
            cfgs[k].softbuffer[0], cfgs[k].softbuffer[1] = (k, self.B + k) if tb_major else (2 * k, 2 * k + 1)
            if self.ctrl:
                u = self.ue_cfgs[k]
                u.tm, u.use_tbs_index_alt = pl.tm, int(pl.tbs_alt)
        return (jobs, sfs, cfgs, n, k0)

    def step(self, bound, stages=None):
        """One batch: mi355_ue_dl_decode_batch (softbuffers of new TBs reset first: OFDM, estimation, PDSCH,
        DL-SCH) or, with the control channels, mi355_ue_dl_find_and_decode_batch.  With `stages` (dict) the
        two-call form (decode_fft_estimate, then decode_pdsch) is timed per stage instead."""
        self.last_bound = bound
        import time
        jobs, sfs, cfgs, n, _ = bound
        C.memset(self.res, 0, C.sizeof(self.res))
        if self.ctrl:
            # find_and_decode resets each TB's softbuffer itself (ue_dl.c:1522-1529)
            check(self.Lc.mi355_ue_dl_find_and_decode_batch(self.ue.h, self.pool.h, jobs, sfs, self.ue_cfgs, cfgs,
                                                            C.byref(self.chest_cfg), self.chest, self.pays, n,
                                                            self.ctrl_res, self.dci, self.res, None),
                  "ue_dl_find_and_decode_batch")
            return
        # on the decoder's own stream, in front of its decode (a NULL-stream reset would not be ordered against it)
        check(self.L.mi355_softbuffer_reset_range(self.pool.h, 0, 2 * n, self.ue.stream()), "softbuffer_reset_range")
        if stages is None:
            check(self.L.mi355_ue_dl_decode_batch(self.ue.h, self.pool.h, jobs, sfs, cfgs, C.byref(self.chest_cfg),
                                                  self.chest, self.pays, n, self.res, None), "ue_dl_decode_batch")
            return
        t0 = time.perf_counter()
        check(self.L.mi355_ue_dl_decode_fft_estimate_batch(self.ue.h, jobs, n, C.byref(self.chest_cfg), self.chest,
                                                           None), "decode_fft_estimate")
        t1 = time.perf_counter()
        check(self.L.mi355_ue_dl_decode_pdsch_batch(self.ue.h, self.pool.h, jobs, sfs, cfgs, self.chest, self.pays, n,
                                                    self.res, None), "decode_pdsch")
        lib().mi355_device_sync()
        t2 = time.perf_counter()
        stages["fft_chest_ms"] = stages.get("fft_chest_ms", 0) + (t1 - t0) * 1e3
        stages["pdsch_decode_ms"] = stages.get("pdsch_decode_ms", 0) + (t2 - t1) * 1e3

    def tb_enabled(self, bound) -> np.ndarray:
        """(n, 2) bool: TBs the bound subframes carry."""
        _, _, cfgs, n, _ = bound
        return np.array([[bool(cfgs[k].grant.tb[t].enabled) for t in range(2)] for k in range(n)])

    def crc_bits(self, n: int) -> np.ndarray:
        """2 bits per subframe (TB0, TB1 CRC ok; with the control channels also exactly one DCI found)."""
        r = np.ctypeslib.as_array(self.res)[: 2 * n]
        bits = (r["crc"] != 0) & (r["ret"] == 0)
        if self.ctrl:
            nd = np.ctypeslib.as_array(self.ctrl_res)[:n]["nof_dci"]
            bits &= np.repeat(nd == 1, 2)
        return bits.astype(np.uint8)

    def received(self, n: int) -> np.ndarray:
        host = np.zeros(n * 2 * self.plen, np.uint8)
        lib().mi355_memcpy_d2h(host.ctypes.data, self.d_pay.ptr, host.nbytes)
        return host.reshape(n, 2, self.plen)

    def payload_ok(self, src: DlSource, bound) -> int:
        """TBs whose CRC passed AND whose decoded bytes equal the transmitted payload."""
        _, _, cfgs, n, k0 = bound
        got = self.received(n)
        want = src.payloads(k0, n)
        bits = self.crc_bits(n).reshape(n, 2)
        ok = 0
        for k in range(n):
            nb = tb_bytes(src.plans[k0 + k].cfg)
            for t in range(2):
                if nb[t] and bits[k, t] and np.array_equal(got[k, t, : nb[t]], want[k, t, : nb[t]]):
                    ok += 1
        return ok

    def avg_its(self, n: int) -> float:
        return float(np.mean(np.ctypeslib.as_array(self.res)[: 2 * n]["avg_iterations_block"]))

    def close(self):
        self.pool.close()
        self.ue.close()


# ------------------------------------------------------------------ phy_dl_test's subframes (lib/test/phy/phy_dl_test.c)

def phy_dl_test_cell(nof_prb: int, tm: int, cell_id: int = 1) -> tuple[P.Cell, int]:
    """(cell, nof_rx_ant) as phy_dl_test's parse_args sets them: TM1 1 port / 1 rx, TM2-4 2 ports / 2 rx
    (phy_dl_test.c:86-107); tm is the 0-based index (SRSLTE_TM1 = 0)."""
    return P.make_cell(nof_prb, 1 if tm == 0 else 2, cell_id), 1 if tm == 0 else 2


def phy_dl_test_plans(cell: P.Cell, tm: int, mcs: int, enable_256qam: bool, nof_subframes: int | None = None,
                      cfi: int = 1, rnti: int = 0x1234, first: int = 0) -> list[SfPlan]:
    """The subframes phy_dl_test transmits (phy_dl_test.c:412-540): DCI format 1 (TM1/TM2), 2A (TM3) or 2 (TM4,
    pinfo 0), resource allocation type 0 over every RBG, rv 0, the DCI at UE-specific location
    (sf / 10) % nof_locations of subframe sf % 10, MCS 0 (6 PRB) / min(MCS, 27) (15 PRB) in subframes 0 and 5;
    eNodeB PDSCH p_a 0 dB, p_b 1 for TM2-4 (:173-175); the UE side as work_ue sets it (:213-219, :571-575:
    MMSE, power_scale on, CSI off, 10 iterations).  nof_subframes defaults to the number of UE locations over
    one frame, as the test does (:427-429); first: global index of the first subframe (a shard of a longer run)."""
    from . import pdcch as D
    nloc = [D.ue_locations(D.nof_cce(cell, cfi), sf, rnti) for sf in range(10)]
    if nof_subframes is None:
        nof_subframes = sum(len(v) for v in nloc)
    fmt = D.FORMAT1 if tm < 2 else (D.FORMAT2A if tm == 2 else D.FORMAT2)
    plans = []
    for sf_idx in range(first, first + nof_subframes):
        tti = sf_idx % 10
        d = D.DciDl()
        d.rnti, d.format, d.alloc_type = rnti, fmt, D.ALLOC_TYPE0
        d.type0_alloc.rbg_bitmask = 0xFFFFFFFF
        m_sf = mcs
        if cell.nof_prb == 6 and sf_idx % 5 == 0:
            m_sf = 0
        elif cell.nof_prb == 15 and sf_idx % 5 == 0:
            m_sf = min(mcs, 27)
        if tm < 2:
            d.tb[0].mcs_idx, d.tb[0].rv, d.tb[0].ndi, d.tb[0].cw_idx = m_sf, 0, 0, 0
            d.tb[1].mcs_idx, d.tb[1].rv = 0, 1
        else:
            for i in range(2):
                d.tb[i].mcs_idx, d.tb[i].rv, d.tb[i].ndi, d.tb[i].cw_idx = m_sf, 0, 0, i
        L, ncce = nloc[tti][(sf_idx // 10) % len(nloc[tti])]
        d.location = D.DciLocation(L, ncce)
        g = D.dci_to_grant(cell, d, tti, cfi, tm, enable_256qam)
        if g is None:
            raise ValueError(f"no grant for tm {tm + 1} mcs {m_sf} at {cell.nof_prb} PRB")
        msg = D.pack(cell, d, tti)
        msg.location, msg.rnti = D.DciLocation(L, ncce), rnti
        c = P.PdschCfg()
        c.grant = g
        c.rnti = rnti
        c.max_nof_iterations = 10
        c.decoder_type = P.MIMO_DECODER_MMSE
        c.p_a, c.p_b, c.power_scale = 0.0, 1 if tm > 0 else 0, 1
        c.csi_enable = 0
        plans.append(SfPlan(tti, cfi, c, msg, tm=tm, tbs_alt=enable_256qam))
    return plans


def phy_dl_test_matrix() -> list[tuple[int, bool, int, int]]:
    """lib/test/phy/CMakeLists.txt:33-58: (nof_prb, allow_256, tm 1..4, mcs) for the 240 phy_dl_test cases; with
    256QAM the MCS-28 case runs MCS 27 (26 at 15 PRB)."""
    out = []
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for allow_256 in (False, True):
            for tm in (1, 2, 3, 4):
                for mcs in range(0, 29, 7):
                    m = mcs
                    if allow_256 and mcs == 28:
                        m = 26 if nof_prb == 15 else 27
                    out.append((nof_prb, allow_256, tm, m))
    return out
