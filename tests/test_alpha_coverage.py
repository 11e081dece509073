"""The conservative alpha coverage masks (pt_alpha_coverage, host code: runs
here without a GPU).  Every cell a mask decides must decide it as the exact
alpha test does (GeometricPrimitive::Intersect -> Material::Alpha,
Primitive.cpp:6-26, Material.hpp:181-198, ImageTexture::alpha
Texture.cpp:46-62) at every barycentric point that falls into it -- checked
on sampled points (random, cell corners and edges) with a float64
restatement of the device test (tri_alpha_rec, pt_trace.h), against which the
masks' 1e-6 value margin and 1e-4 texel margin are far from tight.  The GPU
side (same Li with and without the masks) is the parity suite's
alpha scenes and the full C4 band (tests/test_gpu_parity.py)."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import pytest

from pathtracing_amd import native as N
from pathtracing_amd import scenes
from pathtracing_amd.flatten import bind_lights
from pathtracing_amd.scene import (AlphaMode, AlphaTester, ImageTexture, Mesh, MicrofacetDiffuse, Model,
                                   SolidColor)

ALPHA_IMAGE_TEX = 1  # pt_api.h PT_TEX_IMAGE


def _lib():
    try:
        return N.lib()
    except N.NativeError as e:  # pragma: no cover - the library is built by build()
        pytest.skip(str(e))


def coverage(setup):
    sc = setup.scene
    flat = sc.flat if sc.flat is not None else sc.BuildTlas()
    flat = bind_lights(flat, sc, setup.light_sampler)
    d = flat.desc()
    out = np.zeros((flat.n_prims, 1025), np.uint32)
    assert _lib().pt_alpha_coverage(C.byref(d), N.ptr(out)) == 0
    return flat, out


NONE = 0xFFFFFFFF


def set_n(handle) -> int:
    return 4 << (int(handle) >> 29)


def cell_bits(row, cell):
    """(accept, reject) bits of cells `cell` in a hook row."""
    w, b = cell >> 5, (cell & 31).astype(np.uint32)
    return (row[1 + w] >> b) & 1, (row[513 + w] >> b) & 1


def alpha_cell(u, v, n=4):
    """pt_device.h alpha_cell<n>, vectorised (float32 inputs)."""
    a = np.float32(n) * u.astype(np.float32)
    b = np.float32(n) * v.astype(np.float32)
    fi = np.clip(np.floor(a), 0, n - 1)
    fj = np.clip(np.floor(b), 0, n - 1)
    i, j = fi.astype(np.int64), fj.astype(np.int64)
    im = n - 1 - j
    up = ((a - fi) + (b - fj) > 1.0) & (i < im)
    return j * (2 * n - j) + 2 * np.minimum(i, im) + up


def exact_alpha(flat, slot, u, v):
    """The alpha test's value a and verdict at barycentrics (u, v) of slot's
    triangle, float64 (tri_alpha_rec's algorithm)."""
    p = flat.prims[slot]
    m = flat.materials[p["material"]]
    vid = flat.tri_vidx.reshape(-1, 3)[p["index"]]
    uv = flat.uvs.reshape(-1, 2)[vid].astype(np.float64)
    w = 1.0 - u - v
    tu = u * uv[1, 0] + v * uv[2, 0] + w * uv[0, 0]
    tv = u * uv[1, 1] + v * uv[2, 1] + w * uv[0, 1]
    tid = m["alpha"] if m["alpha"] >= 0 else m["tex"]
    t = flat.textures[tid]
    assert t["kind"] == ALPHA_IMAGE_TEX
    im = flat.images[t["image"]]
    W, H, Ch = int(im["width"]), int(im["height"]), int(im["channels"])
    ch = 3 if m["alpha"] < 0 else 0
    px = flat.texels[int(im["offset"]):int(im["offset"]) + W * H * Ch].reshape(H, W, Ch)[..., ch]
    x, y = tu * W - 0.5, tv * H - 0.5
    xi, yi = np.floor(x).astype(np.int64), np.floor(y).astype(np.int64)
    dx, dy = x - xi, y - yi
    x0, x1, y0, y1 = xi % W, (xi + 1) % W, yi % H, (yi + 1) % H
    f = lambda yy, xx: px[yy, xx].astype(np.float64) / 255.0
    a = (1 - dx) * (1 - dy) * f(y0, x0) + dx * (1 - dy) * f(y0, x1) + (1 - dx) * dy * f(y1, x0) + dx * dy * f(y1, x1)
    if m["alpha"] >= 0:
        a = a * float(t["scale"][0])
    mode = int(m["alpha_mode"])
    if mode == 0:
        return np.ones_like(a, bool), np.zeros_like(a, bool)
    if mode == 2:
        return a > m["alpha_cutoff"], a <= m["alpha_cutoff"]
    return a >= 1.0, a <= 0.0  # Blend: certainly true / certainly false


def sample_points(rng, n, k=4):
    """Random barycentrics in the triangle plus every cell corner and edge
    midpoint of the k x k subdivision."""
    r1, r2 = rng.random(n), rng.random(n)
    s = np.sqrt(r1)
    u, v = s * (1 - r2), s * r2
    m = 2 * k
    g = np.array([(a / m, b / m) for a in range(m + 1) for b in range(m + 1 - a)])
    return np.concatenate([u, g[:, 0]]), np.concatenate([v, g[:, 1]])


def check_scene(setup, rng, min_decided=None, n=400):
    """Every decided cell agrees with the exact test at every sampled point;
    returns the decided fraction of the points."""
    flat, masks = coverage(setup)
    decided = total = 0
    for slot in range(flat.n_prims):
        if flat.prims[slot]["kind"] != 0 or flat.prims[slot]["material"] < 0 or masks[slot, 0] == NONE:
            continue
        mat = flat.materials[flat.prims[slot]["material"]]
        tid = mat["alpha"] if mat["alpha"] >= 0 else mat["tex"]
        if flat.textures[tid]["kind"] != ALPHA_IMAGE_TEX:
            continue  # constant alpha: decided whole (test_alpha_maps_masks_hold)
        k = set_n(masks[slot, 0])
        u, v = sample_points(rng, n, k)
        sure_pass, sure_fail = exact_alpha(flat, slot, u, v)
        total += u.size
        acc, rej = cell_bits(masks[slot], alpha_cell(u, v, k))
        assert not np.any(acc & rej), f"slot {slot}: a {k}x{k} cell both accepted and rejected"
        bad = (acc == 1) & ~sure_pass | (rej == 1) & ~sure_fail
        assert not bad.any(), f"slot {slot} {k}x{k}: wrong at {u[bad][:4]}, {v[bad][:4]}"
        decided += int(((acc | rej) == 1).sum())
    frac = decided / total if total else None
    if min_decided is not None:
        assert frac is not None and frac >= min_decided, frac
    return flat, masks, frac


@pytest.mark.parametrize("k", [4, 8, 16, 32, 64, 128])
def test_alpha_cell_covers_the_cells_once(k):
    # the sub-triangle centroids land in k * k distinct cells, in the row order
    cents = []
    for j in range(k):
        for i in range(k - j):
            cents.append(((i + 1 / 3) / k, (j + 1 / 3) / k))
            if i < k - 1 - j:
                cents.append(((i + 2 / 3) / k, (j + 2 / 3) / k))
    c = np.array(cents)
    cells = alpha_cell(c[:, 0], c[:, 1], k)
    assert sorted(cells.tolist()) == list(range(k * k))


def test_alpha_cell_stays_in_range():
    # vertices and points past the hypotenuse (rounding) stay in range
    u = np.array([0, 1, 0, 0.5000001, 0.25, 1.0000001, -1e-9])
    v = np.array([0, 0, 1, 0.5, 0.7500001, 0, 0.3])
    assert ((alpha_cell(u, v) >= 0) & (alpha_cell(u, v) < 16)).all()


def test_alpha_maps_masks_hold():
    """alpha_maps: every deterministic alpha source (RGB alpha texture with a
    colorScale, one-channel alpha texture, RGBA albedo, solid below cutoff)."""
    flat, masks, _ = check_scene(scenes.alpha_maps(), np.random.default_rng(1))
    # the solid alpha below the cutoff: every cell rejected
    solid = [s for s in range(flat.n_prims) if flat.prims[s]["kind"] == 0 and flat.prims[s]["material"] >= 0 and
             flat.materials[flat.prims[s]["material"]]["alpha"] >= 0 and
             flat.textures[flat.materials[flat.prims[s]["material"]]["alpha"]]["kind"] == 0]
    assert solid
    for s in solid:  # one shared 4 x 4 set, all cells rejected
        assert set_n(masks[s, 0]) == 4 and masks[s, 1] == 0 and masks[s, 513] == 0xFFFF
    assert len({int(masks[s, 0]) for s in solid}) == 1


def leaf_scene(uv_scale=1.0, uv_offset=(0.0, 0.0), mode=AlphaMode.Mask, cutoff=0.5, size=256, n=60, seed=7):
    rng = np.random.default_rng(seed)
    setup = scenes.cornell(W=16, H=16, spp=1, config="c3", max_depth=2, seed=seed)
    img = ImageTexture(scenes._leaf_image(rng, size))
    m = MicrofacetDiffuse(img)
    m.setAlphaTester(AlphaTester(mode, cutoff))
    idx, v, _, nr, uv = scenes._leaf_cards(rng, (0.0, 0.0, 0.0), 0.8, n, 0.15)
    uv = uv * np.float32(uv_scale) + np.asarray(uv_offset, np.float32)
    setup.scene.Add(Model([Mesh(idx, v, None, nr, uv.astype(np.float32), m)]))
    return setup.finish()


def test_leaf_card_masks_hold_and_decide_most_hits():
    """C4's leaf cards (the ellipse mask of scenes._leaf_image): most of the
    area is decided -- what saves the traversal its texel reads."""
    flat, masks, frac = check_scene(leaf_scene(size=1024), np.random.default_rng(2), min_decided=0.95)
    # the cards share two uv layouts: two mask sets, 128 x 128 cells each
    sets = {int(h) for h in masks[:, 0] if h != NONE}
    assert len(sets) == 2 and all(set_n(h) == 128 for h in sets)


@pytest.mark.parametrize("scale,offset", [(2.5, (-0.3, 0.7)), (0.3, (3.9, -2.2)), (40.0, (0.0, 0.0))])
def test_wrapped_footprints_hold(scale, offset):
    """uvs outside [0, 1] (repeat wrap), footprints split at the image edge
    and footprints larger than the image."""
    check_scene(leaf_scene(scale, offset, size=64), np.random.default_rng(3))


def test_blend_masks_hold():
    """Blend: only alpha 0 (reject) and alpha >= 1 cells are decided."""
    check_scene(leaf_scene(mode=AlphaMode.Blend, size=64), np.random.default_rng(4))


def test_masks_are_deterministic_and_memoised_identically():
    a = coverage(leaf_scene(seed=9))[1]
    b = coverage(leaf_scene(seed=9))[1]
    assert np.array_equal(a, b)


def alpha_tex_scene(scale, cutoff, mode=AlphaMode.Mask, size=48, seed=11):
    """Cards whose alpha is a separate one-channel texture with a colorScale
    (Evaluate(uv).x * colorScale.x, the CH1 source), random uvs per card."""
    rng = np.random.default_rng(seed)
    setup = scenes.cornell(W=16, H=16, spp=1, config="c3", max_depth=2, seed=seed)
    a = scenes._noise_img(rng, size, size, 1, 0, 255, smooth=12)
    a = np.where(a > 140, 255, np.where(a < 110, 0, a)).astype(np.uint8)  # large flat regions
    alpha = ImageTexture(a, colorScale=(scale, 1, 1))
    m = MicrofacetDiffuse(SolidColor((0.3, 0.6, 0.2)), None, None, None, alpha)
    m.setAlphaTester(AlphaTester(mode, cutoff))
    idx, v, _, nr, uv = scenes._leaf_cards(rng, (0.0, 0.0, 0.0), 0.8, 40, 0.15)
    uv = uv * rng.uniform(0.3, 2.5, (uv.shape[0], 1)).astype(np.float32) + rng.uniform(-2, 2, (1, 2)).astype(
        np.float32)
    setup.scene.Add(Model([Mesh(idx, v, None, nr, uv.astype(np.float32), m)]))
    return setup.finish()


@pytest.mark.parametrize("scale,cutoff", [(1.25, 0.5), (-0.8, -0.3), (0.7, 0.0)])
def test_scaled_alpha_texture_masks_hold(scale, cutoff):
    """The CH1 source with positive and negative colorScale: the value range
    is scaled (and flipped) before the cutoff decision."""
    _, masks, frac = check_scene(alpha_tex_scene(scale, cutoff), np.random.default_rng(5))
    assert frac is not None and frac > 0.05  # the flat regions decide cells


def test_blend_scaled_alpha_texture_masks_hold():
    check_scene(alpha_tex_scene(1.0, 0.5, mode=AlphaMode.Blend), np.random.default_rng(6))
