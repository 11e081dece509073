"""The C++ drop-in (integration/HipIntegrator.cpp) compiles against the
reference's headers with PT_WITH_MODEL, the exporter's unwrap of the
reference's Model (Model.hpp) that every main.cpp scene needs
(ResourceManager::CacheModel<BLAS4>, main.cpp:290, 376, 483).  The
hip_harness the GPU tests run is built with it (oracle/Makefile HIPFLAGS);
this CPU test checks that build line in this container, where the reference
headers exist, and that the built object carries the Model path."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")

needs_ref = pytest.mark.skipif(not (REF / "Model.hpp").exists() or shutil.which("g++") is None,
                               reason="needs the reference headers (build container only)")


@needs_ref
@pytest.mark.parametrize("with_model", [True, False])
def test_drop_in_compiles_with_and_without_the_model_unwrap(with_model):
    cmd = ["g++", "-std=gnu++20", "-fsyntax-only", "-include", str(ROOT / "oracle" / "chrono_shim.hpp"),
           f"-I{REF}", f"-I{ROOT / 'integration'}", f"-I{ROOT / 'include'}", "-I/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", "-w", str(ROOT / "integration" / "HipIntegrator.cpp")]
    if with_model:
        cmd.insert(1, "-DPT_WITH_MODEL")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


@needs_ref
def test_hip_harness_object_unwraps_models():
    obj = ROOT / "oracle" / "_ref" / "hip" / "HipIntegrator.o"
    if not obj.exists():
        pytest.skip("hip_harness not built")
    flags = (ROOT / "oracle" / "Makefile").read_text()
    assert "-DPT_WITH_MODEL" in flags
    syms = subprocess.run(["nm", "-C", str(obj)], capture_output=True, text=True, check=True).stdout
    # the exporter's dynamic_cast<const Model*> needs Model's type info
    assert "typeinfo for Model" in syms
