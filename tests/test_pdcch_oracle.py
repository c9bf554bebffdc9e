"""CPU tests of the downlink control path (no GPU):

* the oracle restatement (oracle/orc_pdcch.c + oracle/pdcch_chain.py) against the golden vectors recorded from
  the reference's own regs.c / pcfich.c / pdcch.c / viterbi37_avx2_16bit.c / rm_conv.c / crc.c
  (tests/golden/pdcch.npz, made by tests/golden/make_golden.py);
* the product library's host-side control functions (DCI sizes, packing / unpacking, DL grant, search spaces,
  REG map size, the eNodeB-side PCFICH / PDCCH encoder) against the oracle -- these run on the CPU.
"""
import numpy as np
import pytest

from golden_io import load
from oracle import pdcch_chain as P

Z = load("pdcch.npz")


def _ctrl_grid(k):
    nprb, ports, nrx = (int(v) for v in Z[f"sf{k}_cfg"][:3])
    glen = 14 * 12 * nprb
    y = np.zeros((nrx, glen), np.complex64)
    h = np.zeros((ports, nrx, glen), np.complex64)
    c = Z[f"sf{k}_y"].shape[1]
    y[:, :c] = Z[f"sf{k}_y"]
    h[:, :, :c] = Z[f"sf{k}_h"]
    return y, h


@pytest.mark.parametrize("k", range(int(Z["regs_n"])))
def test_regs_match_reference(k):
    nprb, ports, cid, res = (int(v) for v in Z[f"regs{k}_cell"])
    rg = P.regs(nprb, ports, cid, res)
    assert np.array_equal(rg.pcfich, Z[f"regs{k}_pcfich"])
    assert np.array_equal(rg.nregs, Z[f"regs{k}_nregs"])
    for c in range(3):
        assert np.array_equal(rg.pdcch[c], Z[f"regs{k}_pdcch{c}"])
    assert np.array_equal(rg.phich, Z[f"regs{k}_phich"])


def test_search_spaces_match_reference():
    for row in Z["locations"]:
        ncce, sf, rnti, n = (int(v) for v in row[:4])
        want = [(int(row[4 + 2 * i]), int(row[5 + 2 * i])) for i in range(n)]
        got = P.common_locations(ncce) if rnti == 0xFFFF else P.ue_locations(ncce, sf, rnti)
        assert got == want, (ncce, sf, rnti)


def test_crc16_matches_reference():
    L = P._lib()
    for k in range(int(Z["crc_n"])):
        b = Z[f"crc{k}_bits"]
        assert L.orc_crc16_bits(np.ascontiguousarray(b), b.size) == int(Z[f"crc{k}_crc"])


def test_viterbi_matches_reference():
    """Tail-biting K=7 decoder on u16 symbols: noisy code words, uniform random and saturated edge values."""
    L = P._lib()
    for k in range(int(Z["vit_n"])):
        sym = Z[f"vit{k}_sym"]
        F = sym.size // 3
        out = np.zeros(F, np.uint8)
        L.orc_viterbi37_tb_decode_us(np.ascontiguousarray(sym), F, out)
        assert np.array_equal(out, Z[f"vit{k}_bits"]), k


def test_dci_encode_decode_match_reference():
    L = P._lib()
    for k in range(int(Z["enc_n"])):
        bits, e_ref = Z[f"enc{k}_bits"], Z[f"enc{k}_e"]
        nb, E = bits.size, e_ref.size
        e = np.zeros(E, np.uint8)
        L.orc_pdcch_encode(np.ascontiguousarray(bits), nb, 0x1234, E, e)
        assert np.array_equal(e, e_ref)
        for snr in (0.4, 1.0, 2.5):
            llr = Z[f"dec{k}_{snr}_llr"]
            rm = np.zeros(3 * (nb + 16), np.float32)
            L.orc_rm_conv_rx(llr, E, rm, rm.size)
            q = np.zeros(rm.size, np.uint16)
            L.orc_viterbi_quant(rm, rm.size, q)
            out = np.zeros(nb + 16, np.uint8)
            L.orc_viterbi37_tb_decode_us(q, nb + 16, out)
            assert np.array_equal(out, Z[f"dec{k}_{snr}_out"]), (k, snr)
            p = int("".join(str(b) for b in out[nb:]), 2)
            assert p ^ L.orc_crc16_bits(out, nb) == int(Z[f"dec{k}_{snr}_crc"])


@pytest.mark.parametrize("k", range(8))
def test_control_region_matches_reference(k):
    """PCFICH CFI / correlation and PDCCH LLRs on synthetic control regions (1/2/4 ports, 1/2 rx, AWGN down to 3 dB)
    against srslte_pcfich_decode / srslte_pdcch_extract_llr: CFI exact, float values within 1e-5 of the range
    (the reference's AVX2 build vs the restatement's scalar order), and the SI-RNTI DCI found by the blind search."""
    nprb, ports, nrx, cid, sf, cfi = (int(v) for v in Z[f"sf{k}_cfg"])
    y, h = _ctrl_grid(k)
    noise = float(Z[f"sf{k}_noise"])
    rg = P.regs(nprb, ports, cid, 0)
    got_cfi, corr, _ = P.pcfich_decode(y, h, rg, cid, sf, noise)
    assert got_cfi == int(Z[f"sf{k}_cfi"])
    assert abs(float(corr.max()) - float(Z[f"sf{k}_corr"])) <= 1e-5 * abs(float(Z[f"sf{k}_corr"]))
    llr = P.pdcch_llr(y, h, rg, got_cfi, cid, sf, noise)
    ref = Z[f"sf{k}_llr"]
    assert llr.size == ref.size
    assert np.abs(llr - ref).max() <= 1e-5 * np.abs(ref).max()
    msg = Z[f"sf{k}_msg"]
    if msg.size and got_cfi == cfi:
        found = P.find_dl_dci(llr, rg.nof_cce(got_cfi), sf, P.SIRNTI, nprb, ports)
        on_ref = P.find_dl_dci(ref, rg.nof_cce(got_cfi), sf, P.SIRNTI, nprb, ports)
        assert [f["bits"].tolist() for f in found] == [f["bits"].tolist() for f in on_ref]
        if k != 6:  # case 6 (4 ports, 1 rx, per-RE Rayleigh, 12 dB) is a genuine decoding failure for both
            assert len(found) == 1 and np.array_equal(found[0]["bits"], msg)


# ------------------------------------------------------------------ product host functions vs the oracle

def _prod():
    from srsran_amd import pdcch as D
    from srsran_amd import pdsch as S
    return D, S


def test_tbs_table_transcription():
    D, _ = _prod()
    tbs, f1c = P.tbs_table()
    L = D._declare()
    for i in range(34):
        for n in range(1, 111):
            assert L.mi355_ra_tbs_from_idx(i, n) == tbs[i, n - 1]
    assert tbs[9, 99] == 15840 and tbs[33, 99] == 97896  # MCS 9 / MCS 27 alt at 100 PRB


def test_product_dci_sizes_and_search_spaces():
    D, S = _prod()
    for nprb in (6, 15, 25, 50, 75, 100, 110):
        for ports in (1, 2, 4):
            cell = S.make_cell(nprb, ports, 1)
            for fmt in (P.FORMAT0, P.FORMAT1, P.FORMAT1A, P.FORMAT1C, P.FORMAT1B, P.FORMAT1D, P.FORMAT2, P.FORMAT2A,
                        P.FORMAT2B):
                for csi, srs, ue in ((0, 0, 0), (1, 1, 0), (1, 1, 1), (0, 1, 0)):
                    c = D.DciCfg(csi, 0, 0, srs, 0, ue)
                    o = P.DciCfg(bool(csi), False, bool(srs), bool(ue))
                    assert D.dci_sizeof(cell, fmt, c) == P.dci_sizeof(fmt, nprb, ports, o), (nprb, ports, fmt, c)
            rg = P.regs(nprb, ports, 1, 0)
            for cfi in (1, 2, 3):
                assert D.nof_cce(cell, cfi) == rg.nof_cce(cfi)
    for ncce in (1, 5, 8, 21, 43, 87):
        assert D.common_locations(ncce) == P.common_locations(ncce)
        for sf in range(10):
            assert D.ue_locations(ncce, sf, 0x3C1A) == P.ue_locations(ncce, sf, 0x3C1A)


def _random_dci(rng, fmt, nprb, ports, rnti):
    d = dict(rnti=rnti, format=fmt, alloc_type=0, rbg_bitmask=0, vrb_bitmask=0, rbg_subset=0, shift=0, riv=0,
             n_prb1a=int(rng.integers(2)), n_gap=0, mode=0, pid=int(rng.integers(8)), tpc_pucch=int(rng.integers(4)),
             tb_cw_swap=int(rng.integers(2)), pinfo=0,
             tb=[dict(mcs_idx=int(rng.integers(29)), rv=int(rng.integers(4)), ndi=int(rng.integers(2)), cw_idx=0),
                 dict(mcs_idx=int(rng.integers(29)), rv=int(rng.integers(4)), ndi=int(rng.integers(2)), cw_idx=0)])
    Pg = P.ra_type0_P(nprb)
    nb = int(np.ceil(nprb / Pg))
    if fmt in (P.FORMAT1, P.FORMAT2, P.FORMAT2A):
        d["alloc_type"] = int(rng.integers(2)) if nprb > 10 else 0
        if d["alloc_type"] == 0:
            d["rbg_bitmask"] = int(rng.integers(1, 1 << nb))
        else:
            n1 = nb - int(np.ceil(np.log2(Pg))) - 1
            d["rbg_subset"], d["shift"] = int(rng.integers(Pg)), int(rng.integers(2))
            d["vrb_bitmask"] = int(rng.integers(1, 1 << n1))
        if fmt == P.FORMAT2:
            d["pinfo"] = int(rng.integers(2))
    elif fmt == P.FORMAT1A:
        d["alloc_type"], d["mode"] = 2, int(rng.integers(2)) if P.is_user(rnti) else 0
        L = int(rng.integers(1, nprb + 1))
        s = int(rng.integers(0, nprb - L + 1))
        if d["mode"] == 1:
            nvrb = P.ra_type2_n_vrb_dl(nprb, True)
            L = int(rng.integers(1, nvrb + 1))
            s = int(rng.integers(0, nvrb - L + 1))
        d["riv"] = P.type2_to_riv(L, s, nprb)
    elif fmt == P.FORMAT1C:
        d["alloc_type"], d["mode"] = 2, 1
        step = P.ra_type2_n_rb_step(nprb)
        nvrb = P.ra_type2_n_vrb_dl(nprb, True) // step
        L = int(rng.integers(1, nvrb + 1))
        s = int(rng.integers(0, nvrb - L + 1))
        d["riv"] = P.type2_to_riv(L, s, nvrb)
        d["tb"][0]["mcs_idx"] = int(rng.integers(32))
    return d


def _to_c(D, d):
    c = D.DciDl()
    c.rnti, c.format, c.alloc_type = d["rnti"], d["format"], d["alloc_type"]
    if d["alloc_type"] == 0:
        c.type0_alloc.rbg_bitmask = d["rbg_bitmask"]
    elif d["alloc_type"] == 1:
        c.type1_alloc.vrb_bitmask, c.type1_alloc.rbg_subset, c.type1_alloc.shift = (d["vrb_bitmask"],
                                                                                     d["rbg_subset"], d["shift"])
    else:
        c.type2_alloc.riv, c.type2_alloc.n_prb1a = d["riv"], d["n_prb1a"]
        c.type2_alloc.n_gap, c.type2_alloc.mode = d["n_gap"], d["mode"]
    for i in range(2):
        c.tb[i].mcs_idx, c.tb[i].rv, c.tb[i].ndi = d["tb"][i]["mcs_idx"], d["tb"][i]["rv"], d["tb"][i]["ndi"]
    c.pid, c.tpc_pucch, c.tb_cw_swap, c.pinfo = d["pid"], d["tpc_pucch"], d["tb_cw_swap"], d["pinfo"]
    return c


@pytest.mark.parametrize("nprb,ports", [(6, 1), (15, 2), (25, 2), (50, 1), (75, 4), (100, 2)])
def test_product_dci_pack_unpack_grant(nprb, ports):
    """Random DCIs of formats 1 / 1A / 1C / 2 / 2A: the product's packer equals the oracle's, its unpacker inverts
    it field by field and agrees with the oracle's, and the DL grants (PRB masks incl. distributed VRBs, TBS,
    modulation, scheme, layers, PMI) are the oracle's."""
    D, S = _prod()
    cell = S.make_cell(nprb, ports, 7)
    rng = np.random.default_rng(nprb * 10 + ports)
    tms = {P.FORMAT1: 0, P.FORMAT1A: 0, P.FORMAT1C: 0, P.FORMAT2: 3, P.FORMAT2A: 2}
    for _ in range(60):
        fmt = int(rng.choice([P.FORMAT1, P.FORMAT1A, P.FORMAT1C, P.FORMAT2, P.FORMAT2A]))
        rnti = 0xFFFF if fmt == P.FORMAT1C or (fmt == P.FORMAT1A and rng.integers(2)) else 0x4601
        d = _random_dci(rng, fmt, nprb, ports, rnti)
        bits_o = P.dci_pack(d, nprb, ports)
        m = D.pack(cell, _to_c(D, d))
        assert np.array_equal(D.msg_bits(m), bits_o), (fmt, d)
        u_o = P.dci_unpack(bits_o, fmt, rnti, nprb, ports)
        m.rnti = rnti
        u = D.unpack(cell, m)
        assert u is not None and u_o is not None
        assert (u.alloc_type, u.tb[0].mcs_idx, u.tb[0].rv, u.pid) == (u_o["alloc_type"], u_o["tb"][0]["mcs_idx"],
                                                                       u_o["tb"][0]["rv"], u_o["pid"])
        if u.alloc_type == 2:
            assert (u.type2_alloc.riv, u.type2_alloc.mode, u.type2_alloc.n_prb1a, u.type2_alloc.n_gap) == (
                u_o["riv"], u_o["mode"], u_o["n_prb1a"], u_o["n_gap"])
        cfi = 1 + int(rng.integers(3))
        tti = int(rng.integers(10))
        g = D.dci_to_grant(cell, u, tti, cfi, tms[fmt])
        g_o = P.dci_to_grant(u_o, nprb, ports, tms[fmt])
        assert (g is None) == (g_o is None), (fmt, d)
        if g is None:
            continue
        prb = np.array([[g.prb_idx[s][k] for k in range(nprb)] for s in range(2)], np.uint8)
        assert np.array_equal(prb, g_o["prb"]), (fmt, d)
        assert (g.tx_scheme, g.nof_layers, g.pmi, g.nof_tb) == (g_o["tx_scheme"], g_o["nof_layers"], g_o["pmi"],
                                                                g_o["nof_tb"])
        for i in range(2):
            if g_o["enabled"][i]:
                assert g.tb[i].tbs == g_o["tbs"][i] and [1, 2, 4, 6, 8][g.tb[i].mod] == g_o["qm"][i]
        assert g.nof_re == S.re_map(cell, g, cfi, tti).size


@pytest.mark.parametrize("ports", [1, 2, 4])
def test_product_ctrl_encoder_matches_oracle(ports):
    """The product's eNodeB-side PCFICH / PDCCH encoder writes the oracle's symbols to the same REs."""
    D, S = _prod()
    nprb, cid, tti, cfi = 50, 11, 6, 3
    cell = S.make_cell(nprb, ports, cid)
    rng = np.random.default_rng(ports)
    nb = P.dci_sizeof(P.FORMAT1A, nprb, ports)
    msgs = []
    for (L, n) in ((2, 0), (3, 8), (0, 20), (1, 22)):
        b = rng.integers(0, 2, nb, dtype=np.uint8)
        msgs.append(dict(bits=b, rnti=0x4601 + L, L=L, ncce=n))
    tx_o = np.zeros((ports, 14 * 12 * nprb), np.complex64)
    P.ctrl_tx(tx_o, P.regs(nprb, ports, cid, 0), cid, ports, tti, cfi, msgs)
    tx = np.zeros_like(tx_o)
    D.encode_ctrl_host(cell, tti, cfi, [D.dci_msg(m["bits"], P.FORMAT1A, m["rnti"], m["L"], m["ncce"]) for m in msgs],
                       tx)
    assert np.abs(tx - tx_o).max() <= 1e-6
    assert np.count_nonzero(tx[0]) > 0
