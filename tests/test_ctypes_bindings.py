"""CPU guard against the round-2 crash class (a ctypes binding that declared 11 of its function's 12 argument types,
so a pointer went through as a 32-bit int): every `<lib>.<function>.argtypes = [...]` in the Python mirrors, tests,
bench and oracle glue is checked against the C prototype it binds --

* same number of arguments;
* a pointer type (POINTER, c_void_p, c_char_p, ndpointer, CFUNCTYPE, a ctypes array) exactly where the C parameter
  is a pointer, an array or a function-pointer typedef (`*_fn`), and a 64-bit scalar where the C parameter is size_t / 64-bit;
* every function the Python side CALLS through a library handle has its argtypes declared somewhere, and one that
  returns a pointer or a 64-bit value has its restype declared.

Prototypes come from include/srsran_amd/*.h, include/srslte_mi355/srslte_mi355.h, tests/dropin/caller.c and the
exported definitions of oracle/*.c and oracle/ref/*.c."""
from __future__ import annotations

import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C_SOURCES = (glob.glob(os.path.join(ROOT, "include", "srsran_amd", "*.h")) +
             [os.path.join(ROOT, "include", "srslte_mi355", "srslte_mi355.h"),
              os.path.join(ROOT, "tests", "dropin", "caller.c")] +
             glob.glob(os.path.join(ROOT, "oracle", "*.c")) + glob.glob(os.path.join(ROOT, "oracle", "*.cpp")) +
             glob.glob(os.path.join(ROOT, "oracle", "ref", "*.c")))
PY_SOURCES = (glob.glob(os.path.join(ROOT, "srsran_amd", "*.py")) + glob.glob(os.path.join(ROOT, "tests", "*.py")) +
              glob.glob(os.path.join(ROOT, "oracle", "*.py")) + [os.path.join(ROOT, "bench.py")])
PY_SOURCES = [p for p in PY_SOURCES if not p.endswith("test_ctypes_bindings.py")]
PREFIXES = ("mi355_", "srslte_", "orc_", "ref_", "caller_")
WIDE = re.compile(r"\b(size_t|uint64_t|int64_t|double|ptrdiff_t|long)\b")


def _strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def _split_top(s: str) -> list[str]:
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [x.strip() for x in out if x.strip()]


def c_prototypes() -> dict[str, tuple[str, list[str]]]:
    """name -> (return type, parameter texts) for every prototype / non-static definition."""
    protos: dict[str, tuple[str, list[str]]] = {}
    pat = re.compile(r"(?:^|[;}\n])\s*((?:extern\s+\"C\"\s+)?(?:const\s+)?[A-Za-z_][\w\s\*]*?[\s\*])"
                     r"((?:" + "|".join(PREFIXES) + r")\w*)\s*\(([^;{)]*(?:\([^)]*\)[^;{)]*)*)\)\s*[;{]")
    for path in C_SOURCES:
        src = _strip_comments(open(path).read())
        for m in pat.finditer(src):
            ret, name, params = m.group(1), m.group(2), m.group(3)
            if "static" in ret or "return" in ret or "typedef" in ret:
                continue
            ps = _split_top(params)
            if ps == ["void"]:
                ps = []
            protos.setdefault(name, (" ".join(ret.split()), ps))
    return protos


def _aliases(src: str) -> dict[str, str]:
    al: dict[str, str] = {}
    for m in re.finditer(r"^[ \t]*([A-Za-z_][\w \t,]*?)[ \t]*=[ \t]*(.+)$", src, flags=re.M):
        names = [n.strip() for n in m.group(1).split(",")]
        vals = _split_top(m.group(2))
        if len(names) == len(vals) and all(n.isidentifier() for n in names):
            for n, v in zip(names, vals):
                al[n] = v
    return al


def _expand(tok: str, al: dict[str, str]) -> str:
    for _ in range(3):
        tok = re.sub(r"\b([A-Za-z_]\w*)\b", lambda m: al.get(m.group(1), m.group(1)) if m.group(1) in al and
                     len(al[m.group(1)]) < 80 else m.group(1), tok)
    return tok


def _is_ptr_py(tok: str) -> bool:
    # ndpointer aliases of oracle/__init__.py (i16p, u8p, f32p ...) count as pointers wherever they are imported from
    return bool(re.search(r"POINTER|c_void_p|c_char_p|ndpointer|CFUNCTYPE|\*\s*\w|\b[iuf]\d+p\b", tok))


def _is_wide_py(tok: str) -> bool:
    return bool(re.search(r"c_size_t|c_uint64|c_int64|c_double|c_ulonglong|c_longlong|c_ssize_t", tok))


class _Sym:
    def __init__(self, name):
        self.name = name

    def __getattr__(self, a):
        return _Sym(f"{self.name}.{a}")

    def __call__(self, *a):
        return _Sym(f"{self.name}({', '.join(map(str, a))})")

    def __mul__(self, n):
        return _Sym(f"{self.name} * {n}")

    def __str__(self):
        return self.name


class _SymNS(dict):
    def __missing__(self, key):
        return _Sym(key)


def py_bindings():
    """(file, line, name, [expanded argtype texts]) for every argtypes assignment, restype names, called names."""
    binds, restypes, calls = [], set(), {}
    for path in PY_SOURCES:
        src = open(path).read()
        al = _aliases(src)
        for m in re.finditer(r"\.((?:" + "|".join(PREFIXES) + r")\w*)\.argtypes\s*=\s*\[", src):
            i, depth = m.end(), 1
            while depth:
                depth += {"[": 1, "]": -1}.get(src[i], 0)
                i += 1
            body = src[m.end(): i - 1]
            line = src.count("\n", 0, m.start()) + 1
            rest = src[i: src.index("\n", i)].strip()
            if rest.startswith(("*", "+")):  # a list expression ([...] * n + [...]): evaluate it symbolically
                args = [_expand(str(t), al) for t in eval("[" + body + "]" + rest, {}, _SymNS())]
            else:
                args = [_expand(t, al) for t in _split_top(body)]
            binds.append((os.path.relpath(path, ROOT), line, m.group(1), args))
        # _bind(L, "name", restype, [argtypes]) helpers (oracle/pdcch_chain.py)
        for m in re.finditer(r"_bind\(\w+,\s*\"(\w+)\",\s*([^,]+),\s*", src):
            i = m.end()
            j, depth = i, 0
            while True:
                ch = src[j]
                depth += {"[": 1, "(": 1, "]": -1, ")": -1}.get(ch, 0)
                if depth < 0:
                    break
                j += 1
            expr = src[i:j]
            args = [_expand(str(t), al) for t in eval(expr, {}, _SymNS())]
            binds.append((os.path.relpath(path, ROOT), src.count("\n", 0, m.start()) + 1, m.group(1), args))
            if m.group(2).strip() != "None":
                restypes.add(m.group(1))
        for m in re.finditer(r"\.((?:" + "|".join(PREFIXES) + r")\w*)\.restype\s*=", src):
            restypes.add(m.group(1))
        for m in re.finditer(r"\.((?:" + "|".join(PREFIXES) + r")\w*)\(", src):
            calls.setdefault(m.group(1), f"{os.path.relpath(path, ROOT)}:{src.count(chr(10), 0, m.start()) + 1}")
    return binds, restypes, calls


def test_prototypes_parsed():
    protos = c_prototypes()
    for name in ("mi355_ue_dl_find_and_decode_batch", "srslte_pdsch_decode", "mi355_tdec_batch_run_dev",
                 "caller_pdsch_decode", "orc_ue_dl_rx_batch", "ref_tdec_run_batch", "mi355_ue_dl_set_chunks"):
        assert name in protos, name
    assert len(protos["mi355_ue_dl_find_and_decode_batch"][1]) == 14


def test_argtypes_match_prototypes():
    protos = c_prototypes()
    binds, _, _ = py_bindings()
    assert len(binds) > 100
    bad = []
    for path, line, name, args in binds:
        if name not in protos:
            bad.append(f"{path}:{line} {name}: no C prototype found")
            continue
        cparams = protos[name][1]
        if len(args) != len(cparams):
            bad.append(f"{path}:{line} {name}: {len(args)} argtypes for {len(cparams)} C parameters")
            continue
        for k, (a, c) in enumerate(zip(args, cparams)):
            c_ptr = "*" in c or "[" in c or bool(re.search(r"\w+_fn\b", c))  # (function-pointer typedefs: *_fn)
            if c_ptr != _is_ptr_py(a):
                bad.append(f"{path}:{line} {name} arg {k}: C `{c}` vs ctypes `{a}`")
            elif not c_ptr and bool(WIDE.search(c)) and not _is_wide_py(a):
                bad.append(f"{path}:{line} {name} arg {k}: 64-bit C `{c}` declared as `{a}`")
    assert not bad, "\n".join(bad)


def test_every_called_function_is_declared():
    protos = c_prototypes()
    binds, restypes, calls = py_bindings()
    declared = {b[2] for b in binds}
    bad = []
    for name, where in sorted(calls.items()):
        if name not in protos:
            continue  # Python-side names that share a prefix
        nparams = len(protos[name][1])
        if name not in declared and nparams:
            bad.append(f"{where} {name}: called without argtypes")
        ret = protos[name][0]
        if ("*" in ret or WIDE.search(ret)) and name not in restypes:
            bad.append(f"{where} {name}: returns `{ret}` without restype")
    assert not bad, "\n".join(bad)
