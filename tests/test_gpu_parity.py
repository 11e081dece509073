"""GPU parity tests: the HIP path (through the C ABI) against the oracle and
the reference's golden vectors.

Bars.  The device is built with -ffp-contract=off and
spells out every fused multiply-add the reference's GCC build forms (DESIGN.md
§4), and restates the host libm's sinf / cosf / expf / powf / acosf / atan2f,
so it rounds exactly as the reference does:
  - closest hits exact: hit / miss, primitive and t bit for bit against the
    oracle, hit / miss and t bit for bit against the reference's own hits,
    any-hit answers exact (both node layouts of the pool traversal);
  - per-sample Li, BSDF cases, light cases and surface interactions
    bit-identical to the oracle and to the reference's own values, on every
    parity scene, the 2 %-detail C4 recipe and the full ~10 M-triangle C4
    band (gpurun_out/r3d, round 3);
  - film per-pixel relative L2 <= 1e-3 on every pixel (the f64 splat sums
    in a different order than the reference's FilmTile).
"""
import numpy as np
import pytest

import oracle
from conftest import record_parity
from fixtures import GOLDEN, NAMES, load, rescaled_reference_film
from pathtracing_amd import native as N
from pathtracing_amd import scenes

pytestmark = pytest.mark.gpu

HIT_MIN = 0.9999


@pytest.fixture(scope="module", params=NAMES)
def case(request):
    setup, integ, fx = load(request.param)
    return request.param, setup, integ, fx


def _rays(fx):
    rays = np.zeros(fx["rays"].shape[0], dtype=N.RAY)
    rays["o"], rays["d"], rays["tmax"] = fx["rays"][:, :3], fx["rays"][:, 3:6], fx["rays"][:, 6]
    if "ray_times" in fx:  # a shutter scene's rays, each at its own time
        rays["time"] = fx["ray_times"]
    return rays


def _li_close(got, ref, frac_min=0.999, tag=None):
    err = np.abs(got - ref).max(-1)
    tol = 1e-4 * np.maximum(1.0, np.abs(ref).max(-1))
    frac = (err <= tol).mean()
    if tag:
        record_parity(tag, "li", frac)
    assert frac >= frac_min, f"{frac:.5f} of samples within tolerance (bar {frac_min})"
    np.testing.assert_allclose(got.astype(np.float64).mean((0, 1)), ref.astype(np.float64).mean((0, 1)),
                               rtol=5e-3, atol=1e-6)


def _li_bits(got, ref, tag=None):
    """Per-sample radiance bit for bit."""
    got = np.ascontiguousarray(got, np.float32)
    ref = np.ascontiguousarray(ref, np.float32).reshape(got.shape)
    same = (got.view(np.uint32) == ref.view(np.uint32)).all(-1)
    if tag:
        record_parity(tag, "li", same.mean())
    assert same.all(), f"{same.mean():.5f} of samples bit-identical; first {np.argwhere(~same)[:4].tolist()}"


def _film_close(film, ref, frac_min=0.999, tag=None):
    np.testing.assert_allclose(film[..., 3], ref[..., 3], rtol=1e-9, atol=1e-12)
    num = np.linalg.norm(film[..., :3] - ref[..., :3], axis=-1)
    den = np.maximum(np.linalg.norm(ref[..., :3], axis=-1), 1e-3 * ref[..., 3])
    frac = (num <= 1e-3 * den + 1e-7).mean()
    if tag:
        record_parity(tag, "film", frac)
    assert frac >= frac_min, f"film pixels within 1e-3 rel L2: {frac:.5f} (bar {frac_min})"


@pytest.mark.parametrize("nodes", [N.PT_NODES_FULL, N.PT_NODES_QUANTIZED])
def test_gpu_trace_matches_oracle_and_reference(case, nodes):
    """pt_trace runs the pool traversal, over the reference's 128-B clusters
    or over the 64-B quantized nodes."""
    name, setup, integ, fx = case
    ctx = integ.context()
    ctx.set_node_format(nodes)
    try:
        rays = _rays(fx)
        hits, st = ctx.trace(rays, any_hit=False)
        ref = oracle.trace(integ.flat, rays, any_hit=False)
        # exact: hit / miss, the primitive hit, and t bit for bit (the Li
        # built on these hits is already asserted bit-exact)
        got_hit, ref_hit = hits["prim"] >= 0, ref["hit"] > 0
        bad = np.nonzero(got_hit != ref_hit)[0]
        assert bad.size == 0, f"hit/miss differs from the oracle on rays {bad[:8].tolist()}"
        both = np.nonzero(ref_hit)[0]
        badp = both[hits["prim"][both] != ref["prim"][both]]
        assert badp.size == 0, f"primitive differs from the oracle on rays {badp[:8].tolist()}"
        badt = both[hits["t"][both].view(np.uint32) != ref["t"][both].view(np.uint32)]
        assert badt.size == 0, f"t differs from the oracle on rays {badt[:8].tolist()}"
        # against the reference's own hits: hit / miss and t bit for bit
        fh = fx["hits"]
        bad = np.nonzero(got_hit != (fh[:, 0] > 0))[0]
        assert bad.size == 0, f"hit/miss differs from the reference on rays {bad[:8].tolist()}"
        fb = np.nonzero(fh[:, 0] > 0)[0]
        badt = fb[hits["t"][fb].view(np.uint32) != fh[fb, 1].astype(np.float32).view(np.uint32)]
        assert badt.size == 0, f"t differs from the reference on rays {badt[:8].tolist()}"
        anyh, _ = ctx.trace(rays, any_hit=True)
        bad = np.nonzero((anyh["prim"] > 0) != (fx["any"] > 0))[0]
        assert bad.size == 0, f"any-hit differs from the reference on rays {bad[:8].tolist()}"
        assert st["rays_closest"] == len(rays) and st["nodes_closest"] > 0
        # no exact-t tie was dropped from the re-trace list (pt_stats::
        # tie_overflows; tie_models / tie_instances put ties on every wall hit)
        assert st["tie_overflows"] == 0 and st["stack_overflows"] == 0
    finally:
        ctx.set_node_format(N.PT_NODES_AUTO)


def test_gpu_li_matches_oracle_and_reference(case):
    name, setup, integ, fx = case
    L = integ.RenderSamples()
    Lo, _, _ = oracle.li(integ)
    _li_bits(L, Lo, f"li_oracle/{name}")
    _li_bits(L, fx["li_L"], f"li_ref/{name}")


def test_gpu_film_matches_oracle_and_reference(case):
    name, setup, integ, fx = case
    film = setup.camera.GetFilm()
    film.Clear()
    st = integ.Render()
    ref, cnt = oracle.render(integ, threads=4)
    _film_close(film.accum, ref, 1.0, f"film_oracle/{name}")
    _film_close(film.accum, rescaled_reference_film(name, fx["film"], film.accum), 1.0, f"film_ref/{name}")
    assert st["paths"] == cnt["paths"]
    # the wavefront traces exactly the reference's closest-hit queries
    assert st["rays_closest"] == cnt["closest"]
    # NEE rays whose contribution is already zero are not traced, so never
    # more than the reference's
    assert st["rays_any"] <= cnt["any"]
    assert st["tie_overflows"] == 0 and st["stack_overflows"] == 0


@pytest.mark.parametrize("name", ["lens_box", "lens_gauss", "mitchell2", "cornell_c3"])
def test_gpu_tiled_and_per_pixel_gathers_agree(name, monkeypatch):
    """The tiled separable gather (k_gather_tile, radius 1 and 2 instances)
    against the per-pixel gather (k_gather, PT_GATHER_PIXEL=1) on Box 0.5,
    Gaussian 1.5 and Mitchell 2.0 / 1.5 footprints: same samples, same
    weights, each pixel summed in the same footprint order."""
    setup, integ, fx = load(name)
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render()
    tiled = film.accum.copy()
    monkeypatch.setenv("PT_GATHER_PIXEL", "1")
    film.Clear()
    integ.Render()
    np.testing.assert_allclose(film.accum, tiled, rtol=1e-12, atol=1e-300)
    assert tiled[..., 3].min() > 0


def test_gpu_sharded_films_sum_to_the_frame():
    setup = scenes.cornell(W=64, H=48, spp=6, config="c3")
    integ = setup.make_integrator()
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render()
    full = film.accum.copy()
    parts = []
    for r in range(3):
        film.Clear()
        integ.Render(shard_index=r, shard_count=3)
        parts.append(film.accum.copy())
    np.testing.assert_allclose(sum(parts), full, rtol=1e-9, atol=1e-12)
    ref, _ = oracle.render(integ, threads=4)
    _film_close(full, ref, 0.999, "film_oracle/sharded_c3")


@pytest.mark.parametrize("W,H,pif", [(37, 23, 0), (64, 64, 256), (8, 8, 64)])
def test_gpu_odd_sizes_and_tiny_wavefronts(W, H, pif):
    """Untiled (W, H not multiples of 8) and tiled orders; a wavefront far
    smaller than the frame forces thousands of refills."""
    setup = scenes.example_1(W=W, H=H, spp=3)
    integ = setup.make_integrator()
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render(paths_in_flight=pif)
    ref, _ = oracle.render(integ, threads=4)
    _film_close(film.accum, ref, 0.999, f"film_oracle/odd_{W}x{H}_{pif}")


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_gpu_shallow_depths(depth):
    setup = scenes.material_zoo(W=16, H=16, spp=2, max_depth=depth)
    integ = setup.make_integrator()
    L = integ.RenderSamples()
    Lo, _, _ = oracle.li(integ)
    _li_bits(L, Lo, f"li_oracle/zoo_depth{depth}")
    if depth == 0:
        assert not L.any()


def test_gpu_counters_and_timing():
    setup = scenes.heightfield(n=200, W=64, H=64, spp=2)
    integ = setup.make_integrator()
    st = integ.Render(flags=N.PT_RENDER_COUNT_NODES | N.PT_RENDER_TIMING)
    assert st["nodes_closest"] > st["rays_closest"] > 0
    assert st["tris_closest"] > 0 and st["ms_closest"] > 0 and st["launches_closest"] > 0
    _, cnt = oracle.render(integ, threads=4)
    # node visits per ray of the GPU order vs the reference order (same tree)
    g = st["nodes_closest"] / st["rays_closest"]
    o = cnt["nodes_closest"] / cnt["closest"]
    assert 0.5 * o <= g <= 1.5 * o


def test_gpu_sanmiguel_small_matches_oracle():
    """C4 generator at 2 % detail (≈ 0.2 M triangles, all materials, foliage
    alpha masks, ~200 emissive triangles, sky + sun, depth 128)."""
    setup = scenes.sanmiguel(W=48, H=27, spp=2, detail=0.02, tex_size=64)
    integ = setup.make_integrator()
    L = integ.RenderSamples()
    Lo, _, _ = oracle.li(integ)
    _li_bits(L, Lo, "li_oracle/sanmiguel_2pct")


@pytest.fixture(scope="module")
def c4_full():
    setup = scenes.sanmiguel(W=192, H=108, spp=2)
    return setup, setup.make_integrator()


def test_gpu_sanmiguel_full_size_per_sample_parity(c4_full):
    """The full ~10 M-triangle C4 scene: per-sample Li of a pixel band against
    the oracle over the same BVH, through the default big-scene path (pool
    traversal over quantized nodes), and the same band over the reference's
    full clusters: bit for bit (3,072 / 3,072 samples; depth-128 paths through
    ~10 M triangles)."""
    setup, integ = c4_full
    assert integ.flat.tri_flags.shape[0] > 9_000_000
    b, e = 192 * 40, 192 * 48
    L = integ.RenderSamples(pixel_begin=b, pixel_end=e)
    Lo, _, _ = oracle.li(integ, pixel_begin=b, pixel_end=e)
    _li_bits(L, Lo, "li_oracle/c4_band")
    Lf = integ.RenderSamples(pixel_begin=b, pixel_end=e, flags=N.PT_RENDER_NODES_FULL)
    np.testing.assert_array_equal(L, Lf)


def test_gpu_overlapped_any_hit_stream_is_bit_identical(c4_full):
    """Bounce k's any-hit rays on a second stream beside bounce k+1's
    closest-hit rays (PT_RENDER_OVERLAP_SHADOW) against one stream
    (PT_RENDER_SERIAL_SHADOW): the same per-sample Li and the same film, bit
    for bit, on the full C4 scene (pool traversal)."""
    setup, integ = c4_full
    b, e = 192 * 40, 192 * 48
    Ls = integ.RenderSamples(pixel_begin=b, pixel_end=e, flags=N.PT_RENDER_SERIAL_SHADOW)
    Lo = integ.RenderSamples(pixel_begin=b, pixel_end=e, flags=N.PT_RENDER_OVERLAP_SHADOW)
    np.testing.assert_array_equal(Ls, Lo)
    film = setup.camera.GetFilm()
    films = []
    for f in (N.PT_RENDER_SERIAL_SHADOW, N.PT_RENDER_OVERLAP_SHADOW):
        film.Clear()
        st = integ.Render(flags=f)
        films.append((film.accum.copy(), st["rays_any"], st["rays_closest"]))
    np.testing.assert_array_equal(films[0][0], films[1][0])
    assert films[0][1:] == films[1][1:]


def test_gpu_tail_kernel_is_bit_identical(c4_full):
    """The last bounces of a fixed-SPP chunk in one launch (k_tail: each lane
    loops over its path's bounces) against a wavefront iteration per bounce
    (PT_RENDER_NO_TAIL): the same per-sample Li and film bit for bit, and the
    same closest-hit / NEE query counts, on the full C4 scene."""
    setup, integ = c4_full
    b, e = 192 * 40, 192 * 48
    Lt = integ.RenderSamples(pixel_begin=b, pixel_end=e)
    Ln = integ.RenderSamples(pixel_begin=b, pixel_end=e, flags=N.PT_RENDER_NO_TAIL)
    np.testing.assert_array_equal(Lt, Ln)
    film = setup.camera.GetFilm()
    films = []
    for f in (0, N.PT_RENDER_NO_TAIL):
        film.Clear()
        st = integ.Render(flags=f)
        films.append((film.accum.copy(), st["rays_any"], st["rays_closest"], st["paths"]))
    np.testing.assert_array_equal(films[0][0], films[1][0])
    assert films[0][1:] == films[1][1:]


@pytest.mark.parametrize("name", ["zoo", "sanmiguel", "cornell_c2", "alpha_maps", "example1"])
def test_gpu_tail_kernel_matches_the_wavefront_on_parity_scenes(name):
    """Small scenes reach the tail after a few bounces (a sixteenth of the
    wavefront left): with and without it, the same Li and query counts."""
    setup, integ, fx = load(name)
    Lt = integ.RenderSamples()
    Ln = integ.RenderSamples(flags=N.PT_RENDER_NO_TAIL)
    np.testing.assert_array_equal(Lt, Ln)
    sts = []
    for f in (0, N.PT_RENDER_NO_TAIL):
        setup.camera.GetFilm().Clear()
        st = integ.Render(flags=f)
        sts.append((st["rays_closest"], st["rays_any"], st["paths"]))
    assert sts[0] == sts[1]


def test_gpu_sanmiguel_full_size_matches_reference_band(c4_full):
    """The full ~10 M-triangle C4 scene against the reference's own per-sample
    Li (tests/golden/c4_band.npz: ref_harness li over pixel rows 40..47 at
    192 x 108, 2 spp, through the reference's BVH4 and integrator), with the
    sky power of that reference run: bit for bit."""
    from fixtures import GOLDEN
    from pathtracing_amd.scene import FunctionInfiniteLight
    setup, integ = c4_full
    fx = np.load(GOLDEN / "c4_band.npz", allow_pickle=False)
    lights = list(setup.scene.GetLights()) + list(setup.extra_lights)
    for l, p in zip(lights, fx["light_power"]):
        if isinstance(l, FunctionInfiniteLight):
            l.power_override = float(p)
    fresh = type(setup.light_sampler)()
    fresh.Add(lights)
    fresh.PreProcess(setup.scene.BoundingBox())
    setup.light_sampler = fresh
    integ2 = setup.make_integrator()
    np.testing.assert_allclose(integ2.flat.lights["power"][:len(fx["light_power"])], fx["light_power"], rtol=2e-6)
    b, e = 192 * 40, 192 * 48
    L = integ2.RenderSamples(pixel_begin=b, pixel_end=e)
    _li_bits(L, fx["li_L"], "li_ref/c4_band")


def _frame_pairs(W, H, spp, shard=(0, 1), n=96, seed=7):
    rng = np.random.default_rng(seed)
    own = np.arange(shard[0], spp, shard[1])
    pix = rng.integers(0, W * H, size=n).astype(np.uint32)
    smp = np.concatenate([rng.choice(own, size=n // 2), own[-1:].repeat(n - n // 2)]).astype(np.uint32)
    return pix, smp


@pytest.mark.parametrize("W,H,shard", [(64, 48, (0, 1)), (37, 23, (0, 1)), (64, 48, (1, 3))])
def test_gpu_frame_samples_are_the_oracle_li(W, H, shard):
    """pt_frame_samples reads the per-sample radiance the last pt_render
    splatted (tiled 8x8 and linear pixel orders, a sample shard): equal to the
    oracle's Li of the same (pixel, sample) bit for bit -- bench.py's check of
    the frame it times.  Samples of another shard are refused."""
    setup = scenes.cornell(W=W, H=H, spp=7, config="c3")
    integ = setup.make_integrator()
    setup.camera.GetFilm().Clear()
    integ.Render(shard_index=shard[0], shard_count=shard[1])
    ctx = integ.context()
    pix, smp = _frame_pairs(W, H, 7, shard)
    got = ctx.frame_samples(pix, smp)
    want, _ = oracle.li_pairs(integ, pix, smp)
    _li_bits(got, want, f"frame_samples/{W}x{H}_{shard[0]}of{shard[1]}")
    # one chunk holds the whole frame here: the range is the shard's samples
    own = np.arange(shard[0], 7, shard[1])
    assert ctx.frame_sample_range() == (int(own[0]), int(own[-1]))
    with pytest.raises(N.NativeError):  # a pixel past the film (the tiled work order pads it)
        ctx.frame_samples(np.array([W * H], np.uint32), np.array([shard[0]], np.uint32))
    if shard[1] > 1:
        with pytest.raises(N.NativeError):
            ctx.frame_samples(np.array([0], np.uint32), np.array([shard[0] + 1], np.uint32))
    # any other render replaces the buffer: the record is gone
    integ.RenderSamples(pixel_begin=0, pixel_end=4)
    with pytest.raises(N.NativeError):
        ctx.frame_samples(pix[:1], smp[:1])


def test_gpu_frame_samples_full_size_c4(c4_full):
    """The same check on the full ~10 M-triangle C4 scene (pool traversal,
    quantized nodes, spatial hit sort: the benched path)."""
    setup, integ = c4_full
    setup.camera.GetFilm().Clear()
    integ.Render()
    pix, smp = _frame_pairs(192, 108, 2, n=64)
    got = integ.context().frame_samples(pix, smp)
    want, _ = oracle.li_pairs(integ, pix, smp)
    _li_bits(got, want, "frame_samples/c4_full")


def test_gpu_sanmiguel_full_size_shards_sum(c4_full):
    setup, integ = c4_full
    film = setup.camera.GetFilm()
    film.Clear()
    st = integ.Render(flags=N.PT_RENDER_COUNT_NODES)
    full = film.accum.copy()
    assert st["paths"] == 192 * 108 * 2 and st["rays_any"] > 0
    # no traversal stack push was dropped (pt_stats::stack_overflows: the
    # pool kernels' 48-entry stack, LDS + HBM)
    assert st["stack_overflows"] == 0
    # ... and no exact-t tie was dropped from the re-trace list
    # (pt_stats::tie_overflows, Shape.cpp:204)
    assert st["tie_overflows"] == 0
    parts = []
    for r in range(2):
        film.Clear()
        parts.append(integ.Render(shard_index=r, shard_count=2))
        parts[-1] = (film.accum.copy(), parts[-1])
    np.testing.assert_allclose(parts[0][0] + parts[1][0], full, rtol=1e-9, atol=1e-12)
    assert parts[0][1]["paths"] + parts[1][1]["paths"] == st["paths"]


def _bits_equal(a, b):
    return (a == b) | (np.isnan(a) & np.isnan(b))


def test_gpu_interactions_are_bit_identical_to_the_reference(case):
    """The device's SurfaceInteraction (p, n, ns, uv, tangent) for the
    fixture rays, against the reference's own records, bit for bit."""
    name, setup, integ, fx = case
    rec = integ.context().interact(_rays(fx))
    ref = fx["hits"]
    both = (rec[:, 0] > 0) & (ref[:, 0] > 0)
    assert ((rec[:, 0] > 0) == (ref[:, 0] > 0)).mean() >= 0.999
    # every field bit-identical, sphere uvs included (SphereShape::GetSphereUV's
    # acosf / atan2f are glibc's, restated in pt_libmf.h)
    exact = _bits_equal(rec[both][:, 1:16], ref[both][:, 1:16]).all(1)
    assert exact.all(), f"{name}: {exact.mean():.4f} bit-identical interactions"


def test_gpu_bsdf_matches_oracle_and_reference(case):
    """Material scatter / attenuation / PDF on the fixture cases: the device
    against the oracle and against the reference's own values, every output
    word bit for bit."""
    name, setup, integ, fx = case
    ctx = integ.context()
    cases = fx["bsdf_cases"]
    for m, fid in enumerate(fx["bsdf_flat_ids"]):
        got = np.asarray(ctx.bsdf_cases(int(fid), cases), np.float32)
        orc = np.asarray(oracle.bsdf(integ.flat, int(fid), cases), np.float32)
        same = _bits_equal(got, orc).all(1)
        assert same.all(), f"material {m}: {same.mean():.4f} of cases bit-identical to the oracle"
        ref = np.asarray(fx[f"bsdf{m}"], np.float32)
        same = _bits_equal(got[:, :ref.shape[1]], ref).all(1)
        assert same.all(), f"material {m}: {same.mean():.4f} of cases bit-identical to the reference"


def test_gpu_light_sampler_picks_match_the_running_sum_scan(case):
    """LightSampler::Sample(u) on the device (pt_light_picks: guide table +
    search over the float running sums) against the reference's scan
    restated in numpy (UniformLightSampler: min(u*n, n-1); PowerLightSampler:
    first running sum >= u*total, LightSampler.cpp:7-11, 34-46), on random
    draws, both sides of every guide-bucket edge and the draws whose u*total
    lands on a running sum: identical picks."""
    name, setup, integ, fx = case
    flat = integ.flat
    sl = np.asarray(flat.sampler_lights, np.int64)
    rng = np.random.default_rng(7)
    one = np.float32(1.0)
    u = [rng.integers(0, 1 << 24, 100_000) * np.float32(2.0 ** -24)]
    edges = np.arange(4096, dtype=np.float32) / np.float32(4096)
    u += [edges, np.nextafter(edges, np.float32(0)), np.nextafter(edges, one)]
    n = len(sl)
    if n:
        pw = flat.lights["power"][sl].astype(np.float32)
        cdf = np.cumsum(pw, dtype=np.float32)
        uc = (cdf / cdf[-1]).astype(np.float32)
        u += [uc, np.nextafter(uc, np.float32(0)), np.nextafter(uc, one)]
    u = np.clip(np.concatenate(u).astype(np.float32), 0, np.float32(1 - 2.0 ** -24))
    got = integ.context().light_picks(u)
    if n == 0:
        assert (got == -1).all()
        return
    if flat.light_sampler == 0:
        i = np.minimum((u * np.float32(n)).astype(np.int64), n - 1)
    else:
        target = (u * cdf[-1]).astype(np.float32)
        i = np.minimum(np.searchsorted(cdf, target, side="left"), n - 1)
    np.testing.assert_array_equal(got, sl[i])


def test_gpu_light_samples_match_oracle_and_reference(case):
    """Light::sample / PDF / L on the fixture cases, device vs oracle and vs
    the reference's own values, every output word bit for bit (uvs through
    the restated glibc acosf / atan2f, transformed lights' normals through the
    normal matrix with the build's FNMA cofactors)."""
    name, setup, integ, fx = case
    nc = fx["lsample_cases"].shape[0]
    got = np.asarray(integ.context().light_cases(fx["lsample_cases"], integ.flat.lights.shape[0]), np.float32)
    orc = np.asarray(oracle.lights(integ.flat, fx["lsample_cases"]), np.float32)
    same = _bits_equal(got, orc).all(1)
    assert same.all(), f"{same.mean():.4f} of light cases bit-identical to the oracle; first {np.nonzero(~same)[0][:4]}"
    g, r = got.reshape(-1, nc, 18), fx["lsample"].reshape(-1, nc, 18)
    if "lsample_lights" in fx.files:
        sel = fx["lsample_lights"]
        keep = sel < g.shape[0]
        g, r = g[sel[keep]], r[keep]
    else:
        g = g[:r.shape[0]]  # inner lights of instances (hit identity only) are not Light::sample'd
        r = r[:g.shape[0]]
    same = _bits_equal(g.reshape(-1, 18), np.asarray(r, np.float32).reshape(-1, 18)).all(1)
    assert same.all(), f"{same.mean():.4f} of light cases bit-identical to the reference"


@pytest.mark.parametrize("name", ["cornell_c3", "zoo", "sanmiguel", "instances", "nested_instances"])
@pytest.mark.parametrize("nodes", [N.PT_RENDER_NODES_FULL, N.PT_RENDER_NODES_QUANTIZED])
def test_gpu_pool_and_simple_traversal_agree_bit_for_bit(name, nodes):
    """The persistent refilling traversal (pt_pool.h) and the one-ray-per-lane
    one visit the same nodes in the same order per ray: identical radiance.
    Over the quantized nodes the pool traversal visits a superset of nodes
    (outward-rounded boxes) in the same order, with the same result here."""
    setup, integ, fx = load(name)
    a = integ.RenderSamples(flags=N.PT_RENDER_TRAVERSAL_POOL | nodes)
    b = integ.RenderSamples(flags=N.PT_RENDER_TRAVERSAL_SIMPLE)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", ["zoo", "sanmiguel", "lit_instances", "fog", "nested_instances"])
@pytest.mark.parametrize("flag", [N.PT_RENDER_SORT_MATERIAL, N.PT_RENDER_SORT_SPATIAL,
                                  N.PT_RENDER_SORT_RAYS | N.PT_RENDER_TRAVERSAL_POOL])
def test_gpu_hit_sorted_shading_is_identical(name, flag):
    """PT_RENDER_SORT_MATERIAL / _SPATIAL only change which lane shades which
    path: the per-sample radiance is bit-identical to the unsorted wavefront."""
    setup, integ, fx = load(name)
    a = integ.RenderSamples(flags=flag)
    b = integ.RenderSamples(flags=N.PT_RENDER_NO_SORT)
    np.testing.assert_array_equal(a, b)


# ---------------------------------------------------------------- film resolve (pt_film_resolve)
@pytest.mark.parametrize("film", ["example1", "cornell_c3", "fog", "sanmiguel", "synthetic"])
@pytest.mark.parametrize("tonemap,key", [("reinhard_jodie", "jodie"), ("aces", "aces")])
def test_gpu_film_resolve_matches_reference(film, tonemap, key):
    """The device tone map + sRGB + u8 against Film::WritePNG's pixels computed
    by the reference's own functions; the device contracts its double FMAs
    where GCC may not, so a truncation boundary may move one code value on a
    rare pixel."""
    from fixtures import GOLDEN
    from pathtracing_amd.scene import Film
    fx = np.load(GOLDEN / "film_resolve.npz", allow_pickle=False)
    acc = fx[f"{film}_film"]
    f = Film((acc.shape[1], acc.shape[0]))
    got = f.Resolve(tonemap, accum=acc).astype(int)
    ref = fx[f"{film}_{key}"].astype(int)
    d = np.abs(got - ref)
    assert d.max() <= 1 and (d == 0).mean() >= 0.999, f"{film}/{tonemap}: {(d == 0).mean():.5f} exact, max {d.max()}"


def test_gpu_film_resolve_full_size_matches_oracle():
    """C4's film size (1920x1080) from a device tensor: the same image as the
    oracle's restatement of the writer."""
    import torch
    from pathtracing_amd.scene import Film
    rng = np.random.default_rng(5)
    H, W = 1080, 1920
    acc = np.concatenate([np.exp(rng.uniform(-9, 9, (H, W, 3))), rng.uniform(0.5, 40, (H, W, 1))], -1)
    acc[..., :3] *= acc[..., 3:]
    acc[0, :16] = 0.0
    dev = torch.from_numpy(acc).to("cuda:0")
    f = Film((W, H))
    for tm, t in ((0, "reinhard_jodie"), (1, "aces")):
        got = f.Resolve(t, accum=dev).astype(int)
        ref = oracle.resolve(acc, tm).astype(int)
        d = np.abs(got - ref)
        assert d.max() <= 1 and (d == 0).mean() >= 0.999


# ---------------------------------------------------------------- adaptive sampling (pt_render_adaptive)
ADAPTIVE = ["cornell_c3", "example1", "example1_simple", "zoo", "fog", "lens_box", "instances", "mitchell2",
            "stratified", "motion_path"]


@pytest.mark.parametrize("name", ADAPTIVE)
def test_gpu_adaptive_matches_reference_render(name):
    """pt_render_adaptive against the reference's own TileIntegrator::Render
    with its adaptive rounds (tests/golden/adaptive.npz, ref_harness
    `adaptive`) and against the oracle: per-pixel sample counts identical
    (every stop decision of the f64 Welford estimators), film within the
    film tolerance on every pixel."""
    from fixtures import GOLDEN
    setup, integ, _ = load(name)
    fx = np.load(GOLDEN / "adaptive.npz", allow_pickle=False)
    film = setup.camera.GetFilm()
    film.Clear()
    st = integ.Render(adaptive=True)
    counts = integ.last_sample_counts
    ref_counts = fx[f"{name}_counts"]
    same = (counts == ref_counts).mean()
    record_parity(f"adaptive_counts_ref/{name}", "counts", same)
    np.testing.assert_array_equal(counts, ref_counts)
    assert st["paths"] == int(counts.sum())
    _film_close(film.accum, fx[f"{name}_film"], 1.0, f"adaptive_film_ref/{name}")
    ofilm, ocounts, _ = oracle.render_adaptive(integ, threads=4)
    np.testing.assert_array_equal(counts, ocounts)
    _film_close(film.accum, ofilm, 1.0, f"adaptive_film_oracle/{name}")


def test_gpu_adaptive_tile_shards_and_device_film():
    """Tile shards (32 x 32, Integrators.cpp:33) sum to the unsharded frame;
    the device-film path gives the same film and counts as the host one; a
    sample chunk smaller than a round (tiny wavefront) changes nothing."""
    import torch
    setup = scenes.cornell(W=80, H=72, spp=3, config="c3")
    integ = setup.make_integrator()
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render(adaptive=True)
    full, counts = film.accum.copy(), integ.last_sample_counts.copy()
    assert counts.max() > 3 * 2, "some pixel needs more than one round"
    parts = []
    for r in range(3):
        film.Clear()
        integ.Render(adaptive=True, shard_index=r, shard_count=3)
        parts.append((film.accum.copy(), integ.last_sample_counts.copy()))
    np.testing.assert_allclose(sum(p[0] for p in parts), full, rtol=1e-12, atol=1e-300)
    np.testing.assert_array_equal(sum(p[1] for p in parts), counts)
    dev = torch.zeros((72, 80, 4), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    integ.Render(adaptive=True, film_ptr=dev.data_ptr(), paths_in_flight=256)
    np.testing.assert_allclose(dev.cpu().numpy(), full, rtol=1e-12, atol=1e-300)
    np.testing.assert_array_equal(integ.last_sample_counts, counts)
    ofilm, ocounts, _ = oracle.render_adaptive(integ, threads=4)
    np.testing.assert_array_equal(counts, ocounts)
    _film_close(full, ofilm, 1.0, "adaptive_film_oracle/c3_80x72")


def test_gpu_adaptive_one_sample_rounds():
    """spp = 1: the first round has one sample and Variance() = 0, so every
    pixel stops after one round (the 128 * spp cap itself is reached by
    cornell_c3 / mitchell2 pixels in the fixture test)."""
    setup = scenes.cornell(W=40, H=40, spp=1, config="c3")
    integ = setup.make_integrator()
    ofilm, ocounts, _ = oracle.render_adaptive(integ, threads=4)
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render(adaptive=True)
    np.testing.assert_array_equal(integ.last_sample_counts, ocounts)
    assert ocounts.max() == 1 and ocounts.min() == 1
    _film_close(film.accum, ofilm, 1.0, "adaptive_film_oracle/c3_spp1")


# ---------------------------------------------------------------- F8: vs the reference's own random Render
@pytest.mark.parametrize("name", ["example1", "cornell_c3", "blend_box", "envmap", "sanmiguel_c4"])
def test_gpu_matches_reference_render_statistically(name):
    """pt_render_samples at 1024 spp against the reference's own Render with
    its StratifiedSampler(32, 32) and unseeded RNGs (tests/golden/stats.npz):
    per-pixel means within 4 standard errors on >= 99 % of pixel channels
    (measured 100 %, 100 %, 99.97 %).  sanmiguel_c4 is the C4 recipe class
    (textures, masked foliage, sun + sky + lamps, glass, depth 128) at 2 %
    detail, 64 x 64 pixels."""
    from fixtures import stats_scenes, z_test
    setup = stats_scenes()[name]()
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    L = integ.RenderSamples()
    ok = z_test(L.reshape(H, W, setup.spp, 3), np.load(GOLDEN / "stats.npz", allow_pickle=False)[name])
    record_parity(f"ztest_ref/{name}", "pixels", ok.mean())
    assert ok.mean() >= 0.99, f"{ok.mean():.4f} of pixel channels within 4 sigma"


def test_gpu_blend_alpha_accept_rate():
    """AlphaTester Blend (Material.hpp:189): a ray crossing the alpha-0.35
    panel stops there with probability 0.35 -- device and oracle draw the same
    ray hash, and the rate over 200k camera rays is within 4 binomial sigma."""
    setup = scenes.blend_box(W=8, H=8, spp=1)
    integ = setup.make_integrator()
    rng = np.random.default_rng(11)
    n = 200_000
    rays = np.zeros(n, dtype=N.RAY)
    rays["o"] = setup.camera.lookFrom
    tgt = np.stack([rng.uniform(-0.45, 0.45, n), rng.uniform(-0.5, 0.4, n), np.full(n, 1.2)], 1)
    d = tgt - rays["o"]
    rays["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays["tmax"] = np.inf
    hits, _ = integ.context().trace(rays, any_hit=False)
    ref = oracle.trace(integ.flat, rays, any_hit=False)
    t_panel = (1.2 - setup.camera.lookFrom[2]) / rays["d"][:, 2]
    on_panel = np.abs(hits["t"] - t_panel) < 1e-3
    np.testing.assert_array_equal(hits["prim"], ref["prim"])
    rate = on_panel.mean()
    assert abs(rate - 0.35) <= 4 * np.sqrt(0.35 * 0.65 / n), f"accept rate {rate:.4f}"


# ---------------------------------------------------------------- TextureInfiniteLight (f4)
@pytest.mark.parametrize("integrator", ["path", "simple"])
def test_gpu_envmap_matches_oracle(integrator):
    """A FloatImageTexture environment (TextureInfiniteLight): the device's
    Le / cell pick / PDF (NEE and the escape MIS weight) against the oracle
    per sample and per film pixel, on the same cell running sums."""
    setup = scenes.envmap(W=32, H=32, spp=8, integrator=integrator)
    integ = setup.make_integrator()
    L = integ.RenderSamples()
    Lo, _, _ = oracle.li(integ)
    _li_bits(L, Lo, f"li_oracle/envmap_{integrator}")
    film = setup.camera.GetFilm()
    film.Clear()
    integ.Render()
    ref, _ = oracle.render(integ, threads=4)
    _film_close(film.accum, ref, 1.0, f"film_oracle/envmap_{integrator}")


def test_gpu_frame_sample_range_of_a_multi_chunk_frame(monkeypatch):
    """A frame rendered in several sample chunks keeps only the last one:
    pt_frame_sample_range names it, frame_samples serves it (bit-exact against
    the oracle) and refuses the earlier chunks' samples (bench.py's check draws
    its pairs from the range)."""
    monkeypatch.setenv("PT_SAMPLE_CHUNK", "2")
    setup = scenes.cornell(W=24, H=16, spp=9, config="c3")
    integ = setup.make_integrator()
    setup.camera.GetFilm().Clear()
    integ.Render(shard_index=1, shard_count=2)  # local samples 1, 3 | 5, 7
    ctx = integ.context()
    assert ctx.frame_sample_range() == (5, 7)
    pix = np.arange(0, 24 * 16, 7, dtype=np.uint32)
    smp = np.where(np.arange(pix.size) % 2 == 0, 5, 7).astype(np.uint32)
    want, _ = oracle.li_pairs(integ, pix, smp)
    _li_bits(ctx.frame_samples(pix, smp), want, "frame_samples/multi_chunk")
    with pytest.raises(N.NativeError):
        ctx.frame_samples(pix[:1], np.array([3], np.uint32))


def test_gpu_stratified_camera_lowers_the_pixel_variance():
    """StratifiedSampler(4, 4) on the GPU: over 8 seeds, the per-pixel
    estimate of a 16-spp frame (thin lens, the sky's edges) varies less than with
    the plain stream -- the camera strata take effect (Sampler.hpp:73-151);
    the per-sample bit-exactness is test_gpu_li_matches_oracle_and_reference
    on the `stratified` scenes."""
    def frames(strata):
        out = []
        for k in range(8):
            # depth 1: the sky seen past the sphere and floor, so the pixel's
            # estimate varies with the camera draws only
            setup = scenes.example_1(W=48, H=48, spp=16, max_depth=1, medium=False, seed=0x5EED0900 + k,
                                     lens=(0.3, 1.2))
            setup.strata = strata
            integ = setup.make_integrator()
            film = setup.camera.GetFilm()
            film.Clear()
            integ.Render()
            out.append(film.accum[..., :3] / film.accum[..., 3:4])
        return np.stack(out)
    v_plain = frames(None).var(0).mean(-1)
    v_strat = frames((4, 4)).var(0).mean(-1)
    edge = v_plain > np.percentile(v_plain, 75)  # pixels whose estimate the camera draws move most
    assert v_strat[edge].mean() < 0.7 * v_plain[edge].mean(), (v_strat[edge].mean(), v_plain[edge].mean())


def test_gpu_upload_rejects_an_image_past_the_texel_buffer():
    """pt_scene_upload checks every image lies inside the texel buffer (the
    alpha test reads an image's texels without a bound check): an image whose
    texels run past the buffer is PT_ERR_ARG, the unmodified scene uploads."""
    import copy
    setup = scenes.alpha_maps(W=16, H=16, spp=1)
    integ = setup.make_integrator()
    ctx = integ.context()
    flat = integ.flat
    assert flat.images.shape[0] > 0
    bad = copy.copy(flat)
    bad.images = flat.images.copy()
    bad.images["offset"][0] = flat.texels.size  # its texels start at the buffer's end
    with pytest.raises(N.NativeError):
        ctx.upload(bad)
    ctx.upload(flat)  # and the real one again


@pytest.mark.gpu
@pytest.mark.parametrize("defect", ["cycle", "backward", "other_bvh", "tlas_names_level", "too_deep"])
def test_gpu_upload_rejects_a_malformed_instance_chain(defect):
    """pt_scene_upload validates nested wrappers (pt_instance.inner): a level
    record must come after the record that names it (no cycles), share its
    chain's bvh, never be a TLAS slot's instance, and a chain holds at most
    PT_MAX_INSTANCE_DEPTH levels; each defect is PT_ERR_ARG and the
    unmodified scene uploads afterwards."""
    import copy
    setup = scenes.nested_instances(W=16, H=16, spp=1)
    integ = setup.make_integrator()
    ctx = integ.context()
    flat = integ.flat
    ins = flat.instances
    top = np.nonzero(np.isin(np.arange(len(ins)), flat.prims["index"][flat.prims["kind"] == N.PT_PRIM_INSTANCE]))[0]
    deep = max(top, key=lambda k: _chain_len(ins, k))  # the four-level pane
    assert _chain_len(ins, deep) == 4
    bad = copy.copy(flat)
    bad.instances = ins.copy()
    first = int(ins["inner"][deep])
    if defect == "cycle":  # the innermost level points back at the chain's second record
        last = first
        while bad.instances["inner"][last] >= 0:
            last = int(bad.instances["inner"][last])
        bad.instances["inner"][last] = first
    elif defect == "backward":  # a level record before the record that names it
        bad.instances["inner"][first] = deep
    elif defect == "other_bvh":
        other = next(int(b) for b in np.unique(ins["bvh"]) if b != ins["bvh"][deep])
        bad.instances["bvh"][first] = other
    elif defect == "tlas_names_level":
        bad.prims = flat.prims.copy()
        slot = int(np.nonzero((flat.prims["kind"] == N.PT_PRIM_INSTANCE))[0][0])
        bad.prims["index"][slot] = first
    else:  # a fifth level: the innermost record chains to a copy of itself
        extra = bad.instances[first:first + 1].copy()
        last = first
        while bad.instances["inner"][last] >= 0:
            last = int(bad.instances["inner"][last])
        extra["inner"] = -1
        bad.instances["inner"][last] = len(bad.instances)
        bad.instances = np.concatenate([bad.instances, extra])
    with pytest.raises(N.NativeError):
        ctx.upload(bad)
    ctx.upload(flat)


def _chain_len(ins, k):
    n = 1
    while ins["inner"][k] >= 0:
        k = int(ins["inner"][k])
        n += 1
    return n


# ---------------------------------------------------------------- AnimatedPrimitive inverse (anim_inverse)
def test_gpu_anim_inverse_bit_exact_vs_reference_glm():
    """The device's closed-form inverse of an AnimatedPrimitive's matrix at a
    ray's time (pt_shading.h anim_inverse, through pt_anim_inverse_cases)
    against glm::inverse as the reference's own build computes it
    (tests/golden/anim_inverse.npz): every sign pattern of +0 and
    +-{denormal, tiny, unit, large, near-max} translations, and random ones
    over 20 decades -- all 16 entries bit for bit, the zeros' signs included."""
    from fixtures import GOLDEN
    from pathtracing_amd.integrator import Context
    fx = np.load(GOLDEN / "anim_inverse.npz", allow_pickle=False)
    ctx = Context(0)
    got = ctx.anim_inverse(fx["t"])
    want = fx["inv"]
    bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)).any(1))[0]
    assert bad.size == 0, f"{bad.size} of {len(want)} differ; first t {fx['t'][bad[:4]].tolist()}"


# ---------------------------------------------------------------- stackless any hit (PT_RENDER_ANY_STACKLESS)
STACKLESS_SCENES = [n for n in NAMES if n not in ("instances", "tie_instances", "lit_instances", "motion_blur",
                                                  "motion_path", "motion_simple", "stratified_motion",
                                                  "nested_instances", "ref_transformed_models")]


@pytest.mark.parametrize("name", STACKLESS_SCENES)
def test_gpu_stackless_any_hit_matches_the_reference(name):
    """The stackless any-hit traversal (escape links, no stack; pt_trace
    any_hit 2) answers every fixture ray as the reference's IntersectPred does
    (BVH.hpp:1019-1109), over the quantized records of the scenes without
    instances (the traversal's domain): TLAS leaves with BLAS hops, BLAS-root
    copies, one-leaf BVHs, alpha-tested triangles, quads and spheres."""
    setup, integ, fx = load(name)
    ctx = integ.context()
    ctx.set_node_format(N.PT_NODES_QUANTIZED)
    try:
        rays = _rays(fx)
        sl, st = ctx.trace(rays, any_hit=True, stackless=True)
        bad = np.nonzero((sl["prim"] > 0) != (fx["any"] > 0))[0]
        assert bad.size == 0, f"any-hit differs from the reference on rays {bad[:8].tolist()}"
        stack, _ = ctx.trace(rays, any_hit=True)
        np.testing.assert_array_equal(sl["prim"], stack["prim"])
        assert st["stack_overflows"] == 0 and st["nodes_any"] > 0
    finally:
        ctx.set_node_format(N.PT_NODES_AUTO)


@pytest.mark.parametrize("name", ["sanmiguel", "cornell_c3", "tie_models", "ref_models", "alpha_maps"])
def test_gpu_stackless_any_hit_li_bit_identical(name):
    """Per-sample Li with the NEE rays through the stackless traversal, over
    the pool kernels and quantized records: bit for bit the oracle's."""
    setup, integ, fx = load(name)
    L = integ.RenderSamples(flags=N.PT_RENDER_ANY_STACKLESS | N.PT_RENDER_TRAVERSAL_POOL |
                            N.PT_RENDER_NODES_QUANTIZED)
    Lo, _, _ = oracle.li(integ)
    _li_bits(L, Lo, f"li_stackless/{name}")


def test_gpu_stackless_any_hit_full_size_c4(c4_full):
    """The full ~10 M-triangle C4 band with the stackless any-hit kernel
    (the benched scene): every sample bit-exact against the oracle, no ray
    abandoned (the kernel's step bound counts into stack_overflows)."""
    setup, integ = c4_full
    b, e = 192 * 40, 192 * 48
    L = integ.RenderSamples(pixel_begin=b, pixel_end=e, flags=N.PT_RENDER_ANY_STACKLESS)
    assert integ.last_stats["stack_overflows"] == 0
    Lo, _, _ = oracle.li(integ, pixel_begin=b, pixel_end=e)
    _li_bits(L, Lo, "li_stackless/c4_band")
