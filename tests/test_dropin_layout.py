"""The srslte_* drop-in boundary (include/srslte_mi355/srslte_mi355.h, srsran_amd/lib/libsrslte_mi355.so), CPU side.

* Every struct that crosses the boundary has the reference's size, alignment and field offsets: the probe
  tools/dropin_layout_probe.c compiled against our header must print exactly what it prints compiled against the
  reference headers.  The reference side is the committed fixture tests/golden/srslte_layout_ref.txt (written by
  tests/dropin/Makefile from /root/reference/lib/include); where the reference headers exist the fixture is
  regenerated and checked too.
* The header compiles as C and as C++.
* libsrslte_mi355.so exports every function the header declares, and resolves its own symbols
  (linked with --no-undefined); the reference-header caller library links against it.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "srslte_mi355", "srslte_mi355.h")
PROBE = os.path.join(ROOT, "tools", "dropin_layout_probe.c")
FIXTURE = os.path.join(ROOT, "tests", "golden", "srslte_layout_ref.txt")
LIB = os.path.join(ROOT, "srsran_amd", "lib", "libsrslte_mi355.so")
REF_INC = "/root/reference/lib/include"


def _probe(tmp_path, flags):
    exe = str(tmp_path / "probe")
    subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", *flags, "-o", exe, PROBE], check=True)
    return subprocess.run([exe], check=True, capture_output=True, text=True).stdout


def test_layout_matches_reference_fixture(tmp_path):
    ours = _probe(tmp_path, ["-I", os.path.join(ROOT, "include")])
    ref = open(FIXTURE).read()
    assert len(ref.splitlines()) > 200
    diff = [(a, b) for a, b in zip(ref.splitlines(), ours.splitlines()) if a != b]
    assert not diff, diff[:10]
    assert ours == ref


@pytest.mark.skipif(not os.path.isdir(REF_INC), reason="reference headers not present (GPU box)")
def test_fixture_is_the_reference_layout(tmp_path):
    assert _probe(tmp_path, ["-DUSE_REF", "-I", REF_INC]) == open(FIXTURE).read()


def test_header_compiles_as_c_and_cxx():
    for cmd in (["gcc", "-std=gnu11", "-x", "c"], ["g++", "-std=c++17", "-x", "c++"]):
        subprocess.run([*cmd, "-fsyntax-only", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), HDR],
                       check=True)


def _declared_functions():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    names = re.findall(r"^\s*(?:int|void|float|uint32_t)\s+\**\s*(srslte_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_function():
    assert os.path.exists(LIB), "build with make -C srsran_amd"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    declared = _declared_functions()
    assert len(declared) >= 40, declared
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    # the caller-visible API of the reference for this path (SURVEY 8b levels 2 and 4)
    for f in ("srslte_pdsch_decode", "srslte_ue_dl_decode_fft_estimate", "srslte_ue_dl_decode_pdsch",
              "srslte_ue_dl_find_dl_dci", "srslte_ue_dl_find_and_decode", "srslte_softbuffer_rx_init",
              "srslte_tdec_run_all", "srslte_tdec_iteration"):
        assert f in exported


def test_library_loads_without_a_gpu():
    import ctypes
    L = ctypes.CDLL(LIB)
    L.srslte_tdec_autoimp_get_subblocks.restype = ctypes.c_uint32
    L.srslte_tdec_autoimp_get_subblocks.argtypes = [ctypes.c_uint32]
    L.srslte_symbol_sz.argtypes = [ctypes.c_uint32]
    assert L.srslte_tdec_autoimp_get_subblocks(6144) == 16
    assert L.srslte_tdec_autoimp_get_subblocks(512) == 8
    assert L.srslte_tdec_autoimp_get_subblocks(40) == 0
    assert L.srslte_symbol_sz(100) == 1536 and L.srslte_symbol_sz(6) == 128


def test_reference_header_caller_links():
    caller = os.path.join(ROOT, "tests", "dropin", "libdropin_caller.so")
    if not os.path.exists(caller):
        pytest.skip("caller not built (needs the reference headers: make -C tests/dropin)")
    out = subprocess.run(["ldd", caller], check=True, capture_output=True, text=True).stdout
    assert "libsrslte_mi355.so" in out and "not found" not in out
    und = subprocess.run(["nm", "-D", "--undefined-only", caller], check=True, capture_output=True, text=True).stdout
    assert "srslte_ue_dl_find_dl_dci" in und and "srslte_pdsch_decode" in und


def test_tdec_shim_fits_reference_storage(tmp_path):
    """INTEGRATION 2.3's shim casts the caller's srslte_tdec_t* to mi355_srslte_tdec_t*: the reference object must
    be at least as large (its size from the reference-layout fixture)."""
    m = re.search(r"^srslte_tdec_t\s+size\s+(\d+)", open(FIXTURE).read(), flags=re.M)
    assert m, "srslte_tdec_t size missing from the fixture"
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "srsran_amd/srslte_tdec.h"\n'
                   'int main(void) { printf("%zu", sizeof(mi355_srslte_tdec_t)); return 0; }\n')
    exe = str(tmp_path / "sz")
    subprocess.run(["gcc", "-std=gnu11", "-I", os.path.join(ROOT, "include"), "-o", exe, str(src)], check=True)
    ours = int(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)
    assert ours <= int(m.group(1)), (ours, m.group(1))
