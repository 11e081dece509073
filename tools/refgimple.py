"""GCC's optimized GIMPLE of one reference function, as the reference build
compiles it (test-infrastructure tool for the FMA-contraction map).

The dump is made by the reference's own flags plus -fdump-tree-optimized-lineno
(which does not change code generation: the objects compare equal), into
oracle/_ref/gimple/ (`make -C oracle gimple`).  Contractions show as .FMA /
.FMS / .FNMA / .FNMS internal calls, SLP-vectorised lanes as vector(2) /
vector(4) operations; the lines printed are the function body with PHIs, the
source locations shortened to file:line.

  python tools/refgimple.py <name-regex> [TU ...]"""
from __future__ import annotations

import re
import sys
from pathlib import Path

DUMPS = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "gimple"


def functions(tu: Path):
    s = tu.read_text()
    for part in re.split(r"\n(?=;; Function )", s):
        m = re.match(r";; Function (.*?) \((\S+?),", part)
        if m:
            yield m.group(1), m.group(2), part


def clean(body: str) -> str:
    out = []
    started = False
    for line in body.splitlines():
        if line.startswith("{"):
            started = True
        if not started or "DEBUG" in line or "CLOBBER" in line or not line.strip():
            continue
        if re.match(r"^\s+(float|double|int|unsigned|bool|struct|vector|long|const|char|_Bool|sizetype|void)\b.*;$", line):
            continue  # declarations
        line = re.sub(r"\[(/[^\]]*?)/([^/\]:]+):(\d+):\d+( discrim \d+)?\] ", lambda m: f"[{m.group(2)}:{m.group(3)}] ", line)
        # keep one location per statement (the first)
        locs = re.findall(r"\[([^\]]+:\d+)\] ", line)
        line = re.sub(r"\[[^\]]+:\d+\] ", "", line)
        if locs:
            line = f"{line:90s} // {locs[0]}"
        out.append(line)
    return "\n".join(out)


# the reference harness's link order (oracle/Makefile REFSRC, then the harness):
# an inline function emitted by several objects resolves to the first one
LINK_ORDER = ["Texture", "ResourceManager", "Primitive", "Shape", "Light", "LightSampler", "Scene", "Integrators",
              "PhaseFunction", "stb_image", "stb_image_write", "ref_harness"]


def main(name_re: str, tus=()):
    files = [DUMPS / f"{t}.optimized" for t in (tus or LINK_ORDER) if (DUMPS / f"{t}.optimized").exists()]
    seen = set()
    for f in files:
        for name, mangled, body in functions(f):
            if re.search(name_re, name) and mangled not in seen:
                seen.add(mangled)
                print(f"==== {name}   [{f.stem}] {mangled}")
                print(clean(body))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
