"""Static check of the scripts the round-end driver runs (bench.py, __graft_entry__.py): every name a function reads
as a global must be bound at module level or be a builtin.  Round 4's default bench crashed on a NameError inside a
probe that only a GPU run reaches (map_probe read a local of another function); this catches that class on CPU."""
import builtins
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _unbound_globals(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    known = module_names | set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    bad = []

    def walk(tab, where):
        for s in tab.get_symbols():
            # a read resolved to module scope (implicit global) that nothing binds there
            if s.is_referenced() and (s.is_global() or s.is_declared_global()) and s.get_name() not in known:
                bad.append(f"{where}: {s.get_name()}")
        for ch in tab.get_children():
            walk(ch, f"{where}.{ch.get_name()}" if where else ch.get_name())

    for ch in top.get_children():
        walk(ch, ch.get_name())
    return bad


@pytest.mark.parametrize("name", ["bench.py", "__graft_entry__.py"])
def test_no_unbound_global_reads(name):
    assert _unbound_globals(os.path.join(ROOT, name)) == []


def test_checker_catches_a_stray_local(tmp_path):
    p = tmp_path / "m.py"
    p.write_text("import os\n\ndef f():\n    x = 1\n    return x\n\ndef g(a):\n    return d_in.ptr + a + os.sep\n")
    assert _unbound_globals(str(p)) == ["g: d_in"]
