"""Parse tools/gather_rate's report into profiles/r05_gather_rate.json (the
measured ceiling of the traversal's access pattern that bench.py prices the
traversal kernels against: bench.gather_ceiling).

  python tools/gather_rate_json.py gpurun_out/<run>/gather_rate.txt profiles/r05_gather_rate.json
"""
from __future__ import annotations

import json
import re
import sys
from pathlib import Path

ROW = re.compile(r"^(\w+)\s+(P\d+|C\d+)\s+waves/SIMD\s+(\d+)\s+([\d.]+) ms\s+([\d.]+) G wave-steps/s\s+"
                 r"([\d.]+) lane-loads/clk/CU\s+(\d+) clk/step/wave")


def parse(text: str) -> dict:
    rows = []
    for line in text.splitlines():
        m = ROW.match(line.strip())
        if m:
            rows.append({"level": m.group(1), "pattern": m.group(2), "waves_per_simd": int(m.group(3)),
                         "ms": float(m.group(4)), "g_wave_steps_per_s": float(m.group(5)),
                         "lane_loads_per_clk_cu": float(m.group(6)), "clk_per_step_wave": int(m.group(7))})
    head = [ln for ln in text.splitlines() if "CUs" in ln or "clock" in ln]
    return {"_meta": {"tool": "tools/gather_rate.hip", "header": head[:2],
                      "patterns": {"P1": "one 16-B load per lane per step",
                                   "P3": "three 16-B loads of one 48-B record (the PT_Q48 node / slot step)",
                                   "P4": "four 16-B loads of one 64-B node",
                                   "P7": "a 64-B node and a 48-B slot from two independent chains",
                                   "P5": "see tools/gather_rate.hip"}},
            "rows": rows}


if __name__ == "__main__":
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    out = parse(src.read_text())
    if not out["rows"]:
        sys.exit(f"no rows in {src}")
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(f"{len(out['rows'])} rows -> {dst}")
