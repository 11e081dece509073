"""The device's sinf/cosf (pathtracing_amd/csrc/pt_sincosf.h) against the
host libm the reference and the oracle call: bit-identical on a strided
sample of every float in (-120, 120) (tools/check_sincosf.c; stride 1 is the
exhaustive run)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_sincosf_matches_host_libm(tmp_path):
    exe = tmp_path / "check_sincosf"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-o", str(exe), str(ROOT / "tools" / "check_sincosf.c"),
                    "-lm"], check=True)
    out = subprocess.run([str(exe), "257"], check=True, capture_output=True, text=True).stdout.split()
    total, bad = int(out[0]), int(out[1])
    assert total > 10_000_000 and bad == 0
