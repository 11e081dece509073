"""Diagnostics: BVH4 node visits a wide (up to 8-slot) node that absorbs its
children's children would save, in the reference's visit order, over a
sample of a scene's frame (oracle built with -DORACLE_WIDE_STATS).

    python tools/wide_stats.py [c4|c4small] [rows]"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]


def main(which="c4small", rows=8):
    out = ROOT / "oracle" / "_build" / "liboracle_wide.so"
    subprocess.run(["gcc", "-std=gnu11", "-O3", "-fPIC", "-march=x86-64-v3", "-ffp-contract=off", "-fno-math-errno",
                    "-DORACLE_WIDE_STATS", "-shared", "-o", str(out), str(ROOT / "oracle" / "pt_oracle.c"), "-lm",
                    "-lpthread"], check=True)
    import oracle
    oracle.LIB = out
    lib = oracle.lib()
    lib.oracle_wide_stats.argtypes = [C.c_void_p]
    from pathtracing_amd import scenes
    setup = (scenes.sanmiguel(W=192, H=108, spp=2) if which == "c4" else
             scenes.sanmiguel(W=160, H=90, spp=2, detail=0.02, tex_size=64))
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    y0 = H // 2 - rows // 2
    _, _, cnt = oracle.li(integ, pixel_begin=y0 * W, pixel_end=(y0 + rows) * W)
    w = (C.c_ulonglong * 2)()
    lib.oracle_wide_stats(w)
    nc, na = cnt["nodes_closest"], cnt["nodes_any"]
    print(f"{which}: closest rays {cnt['closest']}: BVH4 nodes/ray {nc / cnt['closest']:.2f}, absorbed "
          f"{w[0] / cnt['closest']:.2f} -> wide {(nc - w[0]) / cnt['closest']:.2f}; tris/ray "
          f"{cnt['tris_closest'] / cnt['closest']:.2f}")
    print(f"   any rays {cnt['any']}: BVH4 nodes/ray {na / max(1, cnt['any']):.2f}, absorbed "
          f"{w[1] / max(1, cnt['any']):.2f} -> wide {(na - w[1]) / max(1, cnt['any']):.2f}; tris/ray "
          f"{cnt['tris_any'] / max(1, cnt['any']):.2f}")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["c4small"]), *(int(a) for a in sys.argv[2:3]))
