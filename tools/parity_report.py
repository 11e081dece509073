"""Measured parity fractions per golden scene (GPU box), the numbers the
per-scene bars in tests/test_gpu_parity.py are pinned to.

    python3 tools/parity_report.py <out.json> [--c4]

For every fixture scene: closest-hit / any-hit agreement with the oracle and
with the reference's own records for both pool node formats (the 128-B
reference clusters and the 64-B quantized nodes), per-sample Li agreement
(|dL| <= 1e-4 max(1, |L|)) with the oracle and the reference fixtures, the
film bar (per-pixel relative L2 <= 1e-3) against both, and whether the pool
traversal over quantized nodes gives the same radiance as the full nodes.
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle", ROOT / "tests" / "golden"):
    sys.path.insert(0, str(p))

import oracle  # noqa: E402
from fixtures import NAMES, load  # noqa: E402
from pathtracing_amd import native as N  # noqa: E402


def li_frac(got, ref):
    err = np.abs(got - ref).max(-1)
    return float((err <= 1e-4 * np.maximum(1.0, np.abs(ref).max(-1))).mean())


def film_frac(film, ref):
    num = np.linalg.norm(film[..., :3] - ref[..., :3], axis=-1)
    den = np.maximum(np.linalg.norm(ref[..., :3], axis=-1), 1e-3 * ref[..., 3])
    return float((num <= 1e-3 * den + 1e-7).mean())


def rays_of(fx):
    rays = np.zeros(fx["rays"].shape[0], dtype=N.RAY)
    rays["o"], rays["d"], rays["tmax"] = fx["rays"][:, :3], fx["rays"][:, 3:6], fx["rays"][:, 6]
    return rays


def scene_report(name):
    setup, integ, fx = load(name)
    ctx = integ.context()
    rays = rays_of(fx)
    ref = oracle.trace(integ.flat, rays, any_hit=False)
    out = {}
    for fmt, tag in ((N.PT_NODES_FULL, "full"), (N.PT_NODES_QUANTIZED, "quant")):
        ctx.set_node_format(fmt)
        hits, _ = ctx.trace(rays, any_hit=False)
        anyh, _ = ctx.trace(rays, any_hit=True)
        agree = (hits["prim"] >= 0) == (ref["hit"] > 0)
        both = agree & (ref["hit"] > 0)
        out[f"hit_oracle_{tag}"] = float(agree.mean())
        out[f"prim_oracle_{tag}"] = float((hits["prim"][both] == ref["prim"][both]).mean())
        out[f"hit_ref_{tag}"] = float(((hits["prim"] >= 0) == (fx["hits"][:, 0] > 0)).mean())
        out[f"any_ref_{tag}"] = float(((anyh["prim"] > 0) == (fx["any"] > 0)).mean())
    ctx.set_node_format(N.PT_NODES_AUTO)
    L = integ.RenderSamples()
    Lo, _, _ = oracle.li(integ)
    out["li_oracle"] = li_frac(L, Lo)
    out["li_ref"] = li_frac(L, fx["li_L"])
    Lq = integ.RenderSamples(flags=N.PT_RENDER_TRAVERSAL_POOL | N.PT_RENDER_NODES_QUANTIZED)
    Lf = integ.RenderSamples(flags=N.PT_RENDER_TRAVERSAL_POOL | N.PT_RENDER_NODES_FULL)
    out["li_quant_vs_full_identical"] = float((Lq == Lf).all(-1).mean())
    out["li_quant_oracle"] = li_frac(Lq, Lo)
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render()
    fo, _ = oracle.render(integ, threads=8)
    out["film_oracle"] = film_frac(film.accum, fo)
    out["film_ref"] = film_frac(film.accum, fx["film"])
    out["samples"] = int(L.shape[0] * L.shape[1])
    return out


def c4_report():
    from pathtracing_amd import scenes
    setup = scenes.sanmiguel(W=192, H=108, spp=2)
    integ = setup.make_integrator()
    b, e = 192 * 40, 192 * 48
    Lo, _, _ = oracle.li(integ, pixel_begin=b, pixel_end=e)
    res = {}
    for f, tag in ((N.PT_RENDER_NODES_QUANTIZED, "quant"), (N.PT_RENDER_NODES_FULL, "full")):
        L = integ.RenderSamples(pixel_begin=b, pixel_end=e, flags=f)
        res[f"li_oracle_{tag}"] = li_frac(L, Lo)
        res[f"L_{tag}"] = L
    res["li_quant_vs_full_identical"] = float((res.pop("L_quant") == res.pop("L_full")).all(-1).mean())
    return res


def main(out, c4=False):
    rep = {}
    for name in NAMES:
        rep[name] = scene_report(name)
        print(name, json.dumps(rep[name]), flush=True)
    if c4:
        rep["c4_band"] = c4_report()
        print("c4_band", json.dumps(rep["c4_band"]), flush=True)
    Path(out).write_text(json.dumps(rep, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], "--c4" in sys.argv)
