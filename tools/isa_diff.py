"""Compare the gfx950 device code of two builds of pt_runtime.hip, kernel by
kernel (a refactor that only removes dead compile-time variants must leave the
default kernels' instructions unchanged).

  python tools/isa_diff.py snap <name> [-D...]   build the device code object, keep <name>.fn.json
  python tools/isa_diff.py diff <a> <b>           kernels whose normalized instructions differ

Runs here on the CPU (hipcc cross-compiles); outputs under /tmp/isa.
"""
from __future__ import annotations

import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = Path("/tmp/isa")
LLVM = Path("/opt/rocm/lib/llvm/bin")


def snap(name: str, defines: list[str]) -> None:
    OUT.mkdir(exist_ok=True)
    co, elf, dis = OUT / f"{name}.co", OUT / f"{name}.elf", OUT / f"{name}.dis"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--offload-device-only", "-O3", "-fPIC",
                    "-std=c++20", "-munsafe-fp-atomics", "-Wno-unused-result", "-Wno-unused-value",
                    "-ffp-contract=off", *defines, "-c", str(ROOT / "pathtracing_amd/csrc/pt_runtime.hip"),
                    "-o", str(co), "-I", str(ROOT / "include"), "-I", str(ROOT / "pathtracing_amd/csrc")],
                   check=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={co}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"], check=True)
    with open(dis, "w") as f:
        subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", str(elf)],
                       check=True, stdout=f)
    fns: dict[str, list[str]] = {}
    cur = None
    for line in dis.read_text().splitlines():
        m = re.match(r"^<(.+)>:$", line)
        if m:
            cur = m.group(1)
            fns[cur] = []
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith(";"):
            continue
        s = re.sub(r"\s*//.*$", "", s)            # encodings / comments
        s = re.sub(r"<[^>]*>", "<L>", s)          # branch targets
        s = re.sub(r"0x[0-9a-f]+", "X", s) if s.startswith(("s_branch", "s_cbranch")) else s
        fns[cur].append(s)
    (OUT / f"{name}.fn.json").write_text(json.dumps(fns))
    print(f"{name}: {len(fns)} functions")


def diff(a: str, b: str) -> int:
    fa = json.loads((OUT / f"{a}.fn.json").read_text())
    fb = json.loads((OUT / f"{b}.fn.json").read_text())
    bad = 0
    for k in sorted(set(fa) | set(fb)):
        if k not in fa or k not in fb:
            print(f"{'only in ' + a if k in fa else 'only in ' + b}: {k}")
            continue
        if fa[k] != fb[k]:
            bad += 1
            print(f"DIFF {k}: {len(fa[k])} vs {len(fb[k])} instructions")
    print(f"{bad} differing of {len(set(fa) & set(fb))} common functions")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "snap":
        snap(sys.argv[2], sys.argv[3:])
    else:
        sys.exit(1 if diff(sys.argv[2], sys.argv[3]) else 0)
