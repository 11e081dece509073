import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle", ROOT / "tests" / "golden"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the native kernels")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the in-tree libraries once if they are missing (hipcc cross-compiles here)."""
    lib = ROOT / "pathtracing_amd" / "_lib" / "libpt_hip.so"
    orc = ROOT / "oracle" / "_build" / "liboracle.so"
    if not lib.exists() or not orc.exists():
        sys.path.insert(0, str(ROOT / "tools"))
        import build_native
        build_native.main(["--no-ref"])
    yield


def record_parity(test: str, key: str, value: float):
    """Append a measured parity fraction to $PT_PARITY_LOG (JSON lines) when
    set: the GPU runs that pin the per-scene bars collect them this way."""
    path = os.environ.get("PT_PARITY_LOG")
    if path:
        import json
        with open(path, "a") as f:
            f.write(json.dumps({"test": test, "key": key, "value": float(value)}) + "\n")
