"""bench.verify_frame's film check: a non-finite film pixel passes only when a
sample in its filter footprint is non-finite in the oracle's Li as well (the
reference itself produces it, as C3's rough-dielectric NaN samples do:
profiles/r05_small_configs.json); a non-finite sample the oracle computes
finite, or a non-finite pixel with no such sample, fails."""
import sys
import types
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _setup(W=6, H=5, spp=4, radius=1.5):
    film = types.SimpleNamespace(Resolution=lambda: (W, H), filter=types.SimpleNamespace(radius=np.array([radius] * 2)))
    return types.SimpleNamespace(camera=types.SimpleNamespace(GetFilm=lambda: film), spp=spp)


def _case(oracle_nan: bool, nan_pixel=(2, 3), film_nan=((2, 3), (3, 3))):
    setup = _setup()
    W, H = 6, 5
    film = torch.ones((H, W, 4), dtype=torch.float64)
    for x, y in film_nan:
        film[y, x, :3] = float("nan")
    bad_p = nan_pixel[1] * W + nan_pixel[0]

    def frame_samples(pix, smp):
        L = np.ones((pix.shape[0], 3), np.float32)
        L[(pix == bad_p) & (smp == 2)] = np.nan
        return L

    def li_pairs(integ, pix, smp):
        L = np.ones((pix.shape[0], 3), np.float32)
        if oracle_nan:
            L[(pix == bad_p) & (smp == 2)] = np.nan
        return L, None

    oracle = types.SimpleNamespace(li_pairs=li_pairs)
    return bench._nonfinite_vs_oracle(setup, None, film, frame_samples, None, oracle)


def test_nonfinite_pixels_explained_by_the_oracle():
    r = _case(oracle_nan=True)
    assert r["explained"] and r["pixels"] == 2 and r["samples_checked"] == 1 and r["samples_as_oracle"] == 1


def test_nonfinite_sample_the_oracle_computes_finite_fails():
    assert not _case(oracle_nan=False)["explained"]


def test_nonfinite_pixel_outside_every_footprint_fails():
    # a NaN pixel two columns away from the only NaN sample's pixel (radius 1)
    assert not _case(oracle_nan=True, film_nan=((2, 3), (5, 0)))["explained"]


def _case2(bug_nan_pixel=None, sample_range=None, film_nan=((2, 3), (3, 3)), max_pixels=64):
    """A genuine NaN sample (the oracle's too) at pixel (2, 3) sample 2, and
    optionally a second non-finite sample the oracle computes finite."""
    setup = _setup()
    W, H = 6, 5
    film = torch.ones((H, W, 4), dtype=torch.float64)
    for x, y in film_nan:
        film[y, x, :3] = float("nan")
    good_p = 3 * W + 2
    bug_p = None if bug_nan_pixel is None else bug_nan_pixel[1] * W + bug_nan_pixel[0]

    def frame_samples(pix, smp):
        L = np.ones((pix.shape[0], 3), np.float32)
        L[(pix == good_p) & (smp == 2)] = np.nan
        if bug_p is not None:
            L[(pix == bug_p) & (smp == 1)] = np.nan
        return L

    def li_pairs(integ, pix, smp):
        L = np.ones((pix.shape[0], 3), np.float32)
        L[(pix == good_p) & (smp == 2)] = np.nan
        return L, None

    oracle = types.SimpleNamespace(li_pairs=li_pairs)
    return bench._nonfinite_vs_oracle(setup, None, film, frame_samples, sample_range, oracle, max_pixels=max_pixels)


def test_a_buggy_nan_beside_a_genuine_one_fails():
    # the bug's NaN sample sits in the same footprint as the reference's own
    assert _case2()["explained"]
    assert not _case2(bug_nan_pixel=(3, 3))["explained"]


def test_more_non_finite_pixels_than_checked_fails():
    assert not _case2(max_pixels=1)["explained"]


def test_a_multi_chunk_frame_cannot_explain_a_nan():
    # the sample buffer holds only the last chunk (samples 2..3 of 4)
    assert not _case2(sample_range=(2, 3))["explained"]
    assert _case2(sample_range=(0, 3))["explained"]


def test_overflows_fail_the_frame_check():
    setup = _setup()
    r = bench.verify_frame(setup, None, 0, 1, 0, None, None, overflows={"stack_overflows": 0, "tie_overflows": 1})
    assert not r["ok"] and r["tie_overflows"] == 1
    r = bench.verify_frame(setup, None, 0, 1, 0, None, None, overflows={"stack_overflows": 0, "tie_overflows": 0})
    assert r["ok"]
