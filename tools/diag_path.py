"""Per-path debugging aid: renders the mini C4 scene at max depth D with a
library built with -DPT_DEBUG_KEY (PT_HIP_LIB=...), so the device prints the
traced path's bounces; the oracle prints the same path with ORACLE_DEBUG_KEY."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from pathtracing_amd import scenes  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 2
setup = scenes.sanmiguel(W=48, H=27, spp=2, detail=0.02, tex_size=64, max_depth=depth)
L = setup.make_integrator().RenderSamples()
pix, s = (int(x) for x in sys.argv[2:4]) if len(sys.argv) > 3 else (158, 0)
print("L", L[pix, s].tolist())
