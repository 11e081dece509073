"""Build the in-tree native libraries.

  pathtracing_amd/_lib/libpt_hip.so   product: HIP kernels (gfx950) + C ABI
                                      + host BVH builder
  oracle/_build/liboracle.so          test infrastructure: C restatement
  oracle/_ref/ref_harness             test infrastructure: the reference
                                      itself (only where /root/reference exists)

hipcc cross-compiles gfx950 code objects without a GPU.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "pathtracing_amd" / "csrc"
LIBDIR = ROOT / "pathtracing_amd" / "_lib"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# device float semantics: no implicit contraction — every fused multiply-add
# the reference's GCC build forms is spelled out (fma_ in pt_device.h), so
# the device rounds exactly as the reference does; see DESIGN.md §4
FP_FLAGS: list[str] = ["-ffp-contract=off"]
ARCH = os.environ.get("PT_OFFLOAD_ARCH", "gfx950")


def _run(cmd, cwd=None):
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True, cwd=cwd)


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build_product(force: bool = False, variant: str = "", defines=()) -> Path:
    """The product library; `variant` + `defines` (-D flags) build an A/B
    copy under pathtracing_amd/_lib/variants/ for tuning runs (PT_HIP_LIB)."""
    libdir = LIBDIR / "variants" if variant else LIBDIR
    libdir.mkdir(parents=True, exist_ok=True)
    out = libdir / (f"libpt_hip_{variant}.so" if variant else "libpt_hip.so")
    deps = list(CSRC.glob("*")) + [ROOT / "include" / "pt_api.h"]
    if not force and not _stale(out, deps):
        return out
    build = ROOT / "build" / variant if variant else ROOT / "build"
    build.mkdir(parents=True, exist_ok=True)
    inc = ["-I", ROOT / "include", "-I", CSRC]
    # Host BVH builder: GNU dialect keeps GCC's default FP contraction, as the
    # reference's own -std=gnu++20 build; x86-64-v3 (AVX2+FMA) is portable to
    # the GPU hosts while contracting like the reference's -march=native build.
    bvh_o = build / "pt_bvh.o"
    _run(["g++", "-std=gnu++20", "-O3", "-march=x86-64-v3", "-fPIC", "-c", CSRC / "pt_bvh.cpp", "-o", bvh_o, *inc])
    # TextureInfiniteLight pre-process (host): no contraction, every fused
    # multiply-add of the reference build is spelled out
    env_o = build / "pt_envmap.o"
    _run(["g++", "-std=gnu++20", "-O3", "-march=x86-64-v3", "-ffp-contract=off", "-fPIC", "-c",
          CSRC / "pt_envmap.cpp", "-o", env_o, *inc])
    # alpha coverage masks (host, upload time; pt_alpha_cov.h)
    cov_o = build / "pt_alpha_cov.o"
    _run(["g++", "-std=gnu++20", "-O2", "-march=x86-64-v3", "-ffp-contract=off", "-fPIC", "-c",
          CSRC / "pt_alpha_cov.cpp", "-o", cov_o, *inc])
    rt_o = build / "pt_runtime.o"
    extra = [d for d in defines if d.startswith("-")]  # raw compiler flags of a tuning variant
    defs = [f"-D{d}" for d in defines if not d.startswith("-")]
    _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++20", "-munsafe-fp-atomics",
          "-Wno-unused-result", "-Wno-unused-value", *FP_FLAGS, *extra, *defs,
          "-c", CSRC / "pt_runtime.hip", "-o", rt_o, *inc])
    tmp = out.with_suffix(".so.tmp")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", rt_o, bvh_o, env_o, cov_o, "-o", tmp, "-lrccl", "-lpthread"])
    os.replace(tmp, out)
    return out


def build_tools() -> None:
    """Measurement helpers run on the GPU box (tools/_bin/, git-ignored):
    the FETCH_SIZE calibration and the gather-rate ceiling of the traversal's
    access pattern (profiles/r05_gather_rate.json)."""
    for name in ("fetch_calib", "gather_rate"):
        src = ROOT / "tools" / f"{name}.hip"
        out = ROOT / "tools" / "_bin" / name
        out.parent.mkdir(parents=True, exist_ok=True)
        if _stale(out, [src]):
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", src, "-o", out])


def build_oracle() -> Path:
    _run(["make", "-s", "-C", ROOT / "oracle"])
    return ROOT / "oracle" / "_build" / "liboracle.so"


def build_reference_harness():
    """The reference itself, compiled from /root/reference (test infrastructure)."""
    if not Path("/root/reference/Integrators.cpp").exists():
        return None
    _run(["make", "-s", "-j8", "-C", ROOT / "oracle", "ref"])
    # the same harness driving the C++ drop-in integrator (integration/) on
    # libpt_hip.so, for the GPU tests of the drop-in (tests/test_gpu_integration.py)
    _run(["make", "-s", "-j8", "-C", ROOT / "oracle", "hip"])
    return ROOT / "oracle" / "_ref" / "ref_harness"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    force = "--force" in argv
    variants = [a.split("=", 1)[1] for a in argv if a.startswith("--variant=")]
    if variants:  # --variant=name:DEF1,DEF2=3 ...  (tuning builds only)
        for v in variants:
            name, _, defs = v.partition(":")
            build_product(True, name, [d for d in defs.split(",") if d])
        return
    build_product(force)
    build_tools()
    build_oracle()
    if "--no-ref" not in argv:
        build_reference_harness()


if __name__ == "__main__":
    main()
