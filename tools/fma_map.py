"""Where the reference build fuses multiply-adds (test-infrastructure tool).

The reference is compiled with GCC's default contraction (-ffp-contract=fast
under gnu++20, -march=native): a product whose only uses are adds becomes an
FMA, across statements and through inlined glm helpers.  Parity of the device
and the oracle with the reference needs the same fused operations spelled out
(fma_ / rmul).  This tool maps every FMA instruction of a debug build of the
reference harness (oracle/Makefile `refdbg`: the reference's own flags + -g,
which does not change code generation) to its inline chain and reports, per
reference expression site (the innermost frame outside glm and libstdc++),
how many FMAs the build emitted there and through which helper lines.

  python tools/fma_map.py oracle/_ref/dbg/ref_harness_g [symbol-regex]
"""
from __future__ import annotations

import collections
import re
import subprocess
import sys

LIB = ("/glm/", "/usr/include/", "/usr/lib/")


def main(exe: str, sym_re: str = "", helpers: str = "") -> None:
    """helpers: regex of function names treated like glm (inlined vector
    helpers); the site is the innermost frame outside them."""
    dis = subprocess.run(["objdump", "-d", "-C", "--no-show-raw-insn", exe], capture_output=True, text=True).stdout
    fn, addrs = None, []
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:", line)
        if m:
            fn = m.group(2)
            continue
        m = re.match(r"^\s+([0-9a-f]+):\s+(vf(n)?m(add|sub)\S*)\s+(.*)$", line)
        if m and fn and (not sym_re or re.search(sym_re, fn)):
            addrs.append((m.group(1), fn, m.group(2), m.group(5)))
    if not addrs:
        return
    # one addr2line call: -a prints each address before its frames (innermost first)
    out = subprocess.run(["addr2line", "-a", "-i", "-f", "-C", "-e", exe] + ["0x" + a for a, *_ in addrs],
                         capture_output=True, text=True).stdout.splitlines()
    groups, cur = {}, None
    i = 0
    while i < len(out):
        if re.match(r"^0x[0-9a-f]+$", out[i]):
            cur = int(out[i], 16)
            groups[cur] = []
            i += 1
            continue
        groups[cur].append((out[i], out[i + 1].split(" (")[0]))
        i += 2
    sites = collections.defaultdict(list)
    for a, fn, op, ops in addrs:
        frames = groups.get(int(a, 16), [])
        site = next((loc for f, loc in frames if not any(s in loc for s in LIB)
                     and not (helpers and re.fullmatch(helpers, f.split("(")[0].strip()))),
                    frames[-1][1] if frames else "?")
        chain = " <- ".join(f"{f.split('(')[0]}@{loc.split('/')[-1]}" for f, loc in frames)
        sites[site].append((fn.split("(")[0], op, ops, chain))
    for site in sorted(sites, key=lambda s: (s.split(":")[0], int(s.split(":")[1]) if s.split(":")[-1].isdigit() else 0)):
        print(f"{site.replace('/root/reference/', '')}: {len(sites[site])}")
        for fn, op, ops, chain in sites[site]:
            print(f"    {op:14s} {ops:28s} {chain}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "", sys.argv[3] if len(sys.argv) > 3 else "")
