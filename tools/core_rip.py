#!/usr/bin/env python3
"""Poor man's backtrace from an x86-64 Linux core file (no gdb on the box):  tools/core_rip.py <core> [nstack]

For every thread (NT_PRSTATUS): signal, rip and the mapped file + file-relative address of rip; for the first
(faulting) thread also the return-address candidates found scanning its stack (values that point into executable
file mappings), each symbolized with llvm-symbolizer when available."""
import os
import struct
import subprocess
import sys

NT_PRSTATUS, NT_FILE = 1, 0x46494C45
SYMB = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def main():
    path = sys.argv[1]
    nstack = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    f = open(path, "rb")
    eh = f.read(64)
    assert eh[:4] == b"\x7fELF" and eh[4] == 2, "not an ELF64 core"
    phoff, = struct.unpack_from("<Q", eh, 32)
    phentsize, phnum = struct.unpack_from("<HH", eh, 54)
    loads, notes = [], []
    for i in range(phnum):
        f.seek(phoff + i * phentsize)
        p_type, p_flags, p_offset, p_vaddr, _pa, p_filesz, p_memsz, _al = struct.unpack("<IIQQQQQQ", f.read(56))
        if p_type == 1:
            loads.append((p_vaddr, p_memsz, p_offset, p_filesz))
        elif p_type == 4:
            f.seek(p_offset)
            notes.append(f.read(p_filesz))
    threads, files = [], []
    for blob in notes:
        o = 0
        while o + 12 <= len(blob):
            namesz, descsz, ntype = struct.unpack_from("<III", blob, o)
            o += 12
            o += (namesz + 3) & ~3
            desc = blob[o: o + descsz]
            o += (descsz + 3) & ~3
            if ntype == NT_PRSTATUS:
                signo = struct.unpack_from("<i", desc, 0)[0]
                pid = struct.unpack_from("<i", desc, 32)[0]
                rip, = struct.unpack_from("<Q", desc, 112 + 16 * 8)
                rsp, = struct.unpack_from("<Q", desc, 112 + 19 * 8)
                threads.append((pid, signo, rip, rsp))
            elif ntype == NT_FILE:
                count, _page = struct.unpack_from("<QQ", desc, 0)
                ents = [struct.unpack_from("<QQQ", desc, 16 + 24 * k) for k in range(count)]
                names = desc[16 + 24 * count:].split(b"\0")
                files = [(s, e, off * _page, names[k].decode(errors="replace")) for k, (s, e, off) in enumerate(ents)]

    def where(addr):
        for s, e, off, name in files:
            if s <= addr < e:
                base = min(s2 - o2 for s2, _e2, o2, n2 in files if n2 == name)
                return name, addr - base
        return None, None

    def symb(name, rel):
        if not name or not os.path.exists(SYMB) or not os.path.exists(name):
            return ""
        try:
            out = subprocess.run([SYMB, "--obj=" + name, hex(rel)], capture_output=True, text=True, timeout=20).stdout
            return " ".join(out.split("\n")[:2])
        except Exception:
            return ""

    def read(addr, n):
        for v, msz, off, fsz in loads:
            if v <= addr < v + fsz:
                f.seek(off + addr - v)
                return f.read(min(n, v + fsz - addr))
        return b""

    for k, (pid, signo, rip, rsp) in enumerate(threads):
        name, rel = where(rip)
        print(f"thread {k} lwp {pid} signal {signo} rip {rip:#x} {name}+{rel:#x}" if name else
              f"thread {k} lwp {pid} signal {signo} rip {rip:#x} (unmapped)")
        if k == 0 or signo == 11:
            print("   ", symb(name, rel))
    if threads:
        pid, signo, rip, rsp = next((t for t in threads if t[1] == 11), threads[0])
        print(f"stack scan of lwp {pid} from rsp {rsp:#x}:")
        data = read(rsp, 8 * nstack)
        shown = 0
        for i in range(0, len(data) - 7, 8):
            v, = struct.unpack_from("<Q", data, i)
            name, rel = where(v)
            if name and (name.endswith(".so") or ".so." in name or "python" in name):
                print(f"  [rsp+{i:#x}] {v:#x} {os.path.basename(name)}+{rel:#x} {symb(name, rel)}")
                shown += 1
                if shown >= 40:
                    break


if __name__ == "__main__":
    main()
