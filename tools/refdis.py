"""Condensed float-arithmetic disassembly of one function of the reference's
debug build (test-infrastructure tool for the FMA-contraction map):

  python tools/refdis.py <exe> <symbol-regex> [--all]

Intel syntax (destination first), one instruction a line, prefixed by the
source line the debug info gives (the innermost frame, glm / libstdc++ frames
shown by file name).  Without --all only arithmetic, compares, conversions,
shuffles and loads/stores of xmm registers are kept."""
from __future__ import annotations

import re
import subprocess
import sys

KEEP = re.compile(r"^v?(add|sub|mul|div|fmadd|fmsub|fnmadd|fnmsub|sqrt|min|max|xorp|andp|andnp|orp|cvt|comi|ucomi|"
                  r"mov|blend|shuf|unpck|perm|insert|extract|broadcast|rcp|rsqrt|round|hadd|dpp|cmp|j|call)")


def main(exe, sym_re, show_all=False):
    nm = subprocess.run(["nm", "-C", "--defined-only", exe], capture_output=True, text=True).stdout
    syms = subprocess.run(["nm", "--defined-only", "-S", exe], capture_output=True, text=True).stdout
    dem = {}
    for line in subprocess.run(["nm", "-C", "--defined-only", "-S", exe], capture_output=True, text=True).stdout.splitlines():
        p = line.split(" ", 3)
        if len(p) == 4 and re.search(sym_re, p[3]):
            dem[p[3]] = (int(p[0], 16), int(p[1], 16))
    for name, (addr, size) in sorted(dem.items(), key=lambda kv: kv[1][0]):
        if "cold" in name:
            continue
        print(f"==== {name} @ {addr:#x} ({size} B)")
        out = subprocess.run(["objdump", "-d", "-C", "-l", "-M", "intel", "--no-show-raw-insn",
                              f"--start-address={addr:#x}", f"--stop-address={addr + size:#x}", exe],
                             capture_output=True, text=True).stdout
        loc = ""
        last = None
        for line in out.splitlines():
            m = re.match(r"^(/\S+):(\d+)", line)
            if m:
                f = m.group(1).replace("/root/reference/", "")
                f = f.split("/")[-1] if ("glm" in f or "/usr/" in f) else f
                loc = f"{f}:{m.group(2)}"
                continue
            m = re.match(r"^\s+([0-9a-f]+):\s+(\S+)\s*(.*)$", line)
            if not m:
                continue
            op, args = m.group(2), m.group(3)
            if not show_all and not KEEP.match(op):
                continue
            if not show_all and op.startswith(("mov", "vmov")) and "xmm" not in args and "ymm" not in args:
                continue
            args = re.sub(r"\s+#.*$", "", args)
            tag = loc if loc != last else ""
            last = loc
            print(f"{m.group(1):>6s} {tag:34s} {op:14s} {args}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "--all" in sys.argv)
