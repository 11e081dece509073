"""Static instruction audit of one kernel from the device assembly
(hipcc --offload-device-only -S, the product flags): per basic block, the
instruction mix (VALU, SALU, vector memory loads / stores, LDS, waits,
branches) and the loop the block belongs to, plus the totals over the
kernel's outermost loop.  Test/measurement tool.

  python tools/isa_audit.py <file.s> <kernel-symbol-regex> [out.txt]
"""
from __future__ import annotations

import re
import sys
from collections import OrderedDict

CLASSES = [
    ("vmem_load", re.compile(r"^\s+(buffer_load|global_load|flat_load)")),
    ("vmem_store", re.compile(r"^\s+(buffer_store|global_store|flat_store|buffer_atomic|global_atomic)")),
    ("smem", re.compile(r"^\s+s_(load|buffer_load)")),
    ("lds", re.compile(r"^\s+ds_")),
    ("wait", re.compile(r"^\s+s_waitcnt")),
    ("branch", re.compile(r"^\s+s_(cbranch|branch)")),
    ("valu", re.compile(r"^\s+v_")),
    ("salu", re.compile(r"^\s+s_")),
]


def blocks(lines):
    cur, name, loop = [], "entry", ""
    for ln in lines:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)$", ln)
        if m:
            yield name, loop, cur
            name, cur = m.group(1), []
            loop = m.group(2).strip().lstrip(";").strip()
            continue
        if ln.startswith("\t") and not ln.strip().startswith(";") and not ln.strip().startswith("."):
            cur.append(ln)
    yield name, loop, cur


def classify(ins):
    c = OrderedDict((k, 0) for k, _ in CLASSES)
    for ln in ins:
        for k, rx in CLASSES:
            if rx.match(ln):
                c[k] += 1
                break
    return c


def main(path, sym, out=None):
    text = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(text) if re.match(rf"^{sym}.*:", ln))
    end = next(i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end"))
    rows, tot, loop_tot = [], classify([]), classify([])
    for name, loop, ins in blocks(text[start + 1:end]):
        c = classify(ins)
        rows.append((name, loop, len(ins), c))
        for k in tot:
            tot[k] += c[k]
            if loop:
                loop_tot[k] += c[k]
    lines = [f"# static instruction mix of {text[start].split(':')[0]}", f"# source: {path}",
             "# block  insts  " + "  ".join(k for k, _ in CLASSES) + "  loop"]
    for name, loop, n, c in rows:
        lines.append(f"{name:14s} {n:5d}  " + "  ".join(f"{c[k]:4d}" for k, _ in CLASSES) + f"  {loop}")
    lines.append("total          " + "  ".join(f"{k}={v}" for k, v in tot.items()))
    lines.append("in loops       " + "  ".join(f"{k}={v}" for k, v in loop_tot.items()))
    report = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(report)
    print(report)


if __name__ == "__main__":
    main(*sys.argv[1:])
