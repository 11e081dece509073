"""The device's expf / acosf / atanf / atan2f / powf and double log
(pathtracing_amd/csrc/pt_libmf.h) against the host libm the reference and the
oracle call: bit-identical on a strided sample of every float, plus random
(y, x) pairs for atan2f and powf, and log over the medium sampler's inputs
1 - k 2^-24 and random doubles (tools/check_libmf.c; stride 1 is the
exhaustive run: 0 mismatches of 4.3e9 per float function, and of all 2^24
medium inputs + 1e8 random doubles for log, when last run)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_libmf_matches_host_libm(tmp_path):
    exe = tmp_path / "check_libmf"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-o", str(exe), str(ROOT / "tools" / "check_libmf.c"),
                    "-lm"], check=True)
    res = subprocess.run([str(exe), "1021", "2000000"], capture_output=True, text=True)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "expf table in libm: 1" in res.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_u8_unit_is_the_division_for_every_byte(tmp_path):
    """pt_shading.h u8_unit (texel byte / 255 as mul + fma correction) equals
    the IEEE division for all 256 bytes."""
    exe = tmp_path / "check_u8unit"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-o", str(exe), str(ROOT / "tools" / "check_u8unit.c"),
                    "-lm"], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "mismatches: 0 of 256" in res.stdout
