"""CPU: the C-ABI shared library loads and exports every symbol that include/srsran_amd/*.h declares
(no compute calls here -- there is no GPU in the build container)."""
import ctypes
import glob
import os
import re

import srsran_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "srsran_amd", "*.h")):
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"\b((?:mi355|srsran_amd)_\w+)\s*\(", txt):
            if not m.group(1).endswith("_t"):
                names.add(m.group(1))
    return sorted(names)


def test_headers_declare_api():
    names = declared_symbols()
    assert "mi355_tdec_batch_run_dev" in names and len(names) >= 10


def test_library_exports_every_declared_symbol():
    if not os.path.exists(srsran_amd.LIB_PATH):
        srsran_amd.build()
    lib = ctypes.CDLL(srsran_amd.LIB_PATH)
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    data = open(srsran_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in data
