"""Integrators backed by the HIP wavefront tracer (libpt_hip.so).

Mirrors the reference's `Integrator` interface (Integrators.hpp:10-67):
PathIntegrator(scene, camera, sampler, lightSampler, maxDepth) and
SimplePathIntegrator(scene, camera, sampler, maxDepth); Render() fills the
camera's Film (sum RGB*w, sum w per pixel, Film.hpp:227-253).

The sample stream is the deterministic counter-based PCG stream of DESIGN.md
(`PCGSampler`); the reference's `UniformSampler` name is accepted for its
samples-per-pixel count (its RNG is unseeded, so no frame of it is
reproducible anyway: SURVEY.md §0.4).  `StratifiedSampler(xSamples,
ySamples)` stratifies the camera draws as the reference's does on Render's
per-thread clone (Sampler.hpp:73-151): pixel, time and lens strata from
PermutationElement / Hash, the stream as the jitter.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import native as N
from .flatten import bind_lights, camera_desc
from .scene import BoxFilter, Camera, GaussianFilter, LightSampler, MitchellFilter, Scene


class Sampler:
    def __init__(self, samples: int, seed: int = 0x5EED0001):
        self.samples = int(samples)
        self.seed = int(seed) & 0xFFFFFFFF

    def SamplesPerPixel(self) -> int:
        return self.samples


class PCGSampler(Sampler):
    pass


class UniformSampler(Sampler):
    pass


class StratifiedSampler(Sampler):
    """StratifiedSampler(xSamples, ySamples) (Sampler.hpp:73-151).  Render's
    camera draws go through its per-thread clone (Integrators.cpp:39, 61-64):
    sample index i of pixel (px, py) takes the stratum
    PermutationElement(i, spp, Hash(px, py, dimension)) (Util.hpp:45-73,
    160-168) of the pixel (dimension 0), time (2) and lens (3) draws, jittered
    by the stream's draw of that dimension (the reference's random_float()).
    The path's own draws come from the stream (the reference's Li draws from
    the integrator's shared sampler)."""

    def __init__(self, xSamples: int, ySamples: int, seed: int = 0x5EED0001):
        super().__init__(int(xSamples) * int(ySamples), seed)
        self.xSamples, self.ySamples = int(xSamples), int(ySamples)

    @property
    def strata(self) -> tuple[int, int]:
        return self.xSamples, self.ySamples


class Context:
    """One libpt context: one GPU, or several (`devices`) with the library's
    own RCCL film reduce (pt_create(ctx, n_devices, device_ids)).  Fails
    loudly if HIP or the library is missing."""

    def __init__(self, device: int = 0, devices: Optional[list[int]] = None):
        self._lib = N.lib()
        self.ptr = C.c_void_p()
        ids = [int(device)] if devices is None else [int(d) for d in devices]
        arr = (C.c_int * len(ids))(*ids)
        N.check(self._lib.pt_create(C.byref(self.ptr), len(ids), arr))
        self.device = ids[0]
        self.devices = ids
        self.scene_key = None
        self.comm_ranks = 0

    @staticmethod
    def comm_unique_id() -> bytes:
        """pt_comm_unique_id: the RCCL id rank 0 broadcasts (PT_COMM_ID_BYTES)."""
        buf = (C.c_uint8 * N.PT_COMM_ID_BYTES)()
        N.check(N.lib().pt_comm_unique_id(buf))
        return bytes(buf)

    def comm_init_rank(self, n_ranks: int, rank: int, uid: bytes):
        """pt_comm_init_rank: join the film-reduce communicator (one process per GPU)."""
        buf = (C.c_uint8 * N.PT_COMM_ID_BYTES).from_buffer_copy(uid)
        N.check(self._lib.pt_comm_init_rank(self.ptr, int(n_ranks), int(rank), buf), self.ptr)
        self.comm_ranks = int(n_ranks)

    def film_reduce(self, film_ptr: int, n_doubles: int, root: int = 0):
        """pt_film_reduce: in-place ncclReduce(SUM) of a device film onto `root`."""
        N.check(self._lib.pt_film_reduce(self.ptr, C.c_void_p(film_ptr), int(n_doubles), int(root)), self.ptr)

    def comm_destroy(self):
        """pt_comm_destroy: drop this process's film-reduce communicator."""
        N.check(self._lib.pt_comm_destroy(self.ptr), self.ptr)
        self.comm_ranks = 0

    def frame_sample_range(self) -> tuple[int, int]:
        """pt_frame_sample_range: (first, last) frame sample indices of this
        shard that frame_samples can serve (the last sample chunk)."""
        a, b = C.c_uint32(0), C.c_uint32(0)
        N.check(self._lib.pt_frame_sample_range(self.ptr, C.byref(a), C.byref(b)), self.ptr)
        return int(a.value), int(b.value)

    def frame_samples(self, pixels: np.ndarray, samples: np.ndarray) -> np.ndarray:
        """pt_frame_samples: per-sample radiance (n, 3) float32 of the last
        fixed-SPP frame rendered on this context, for (pixel, sample) pairs
        (pixel = y * width + x, sample = the frame's sample index)."""
        pix = np.ascontiguousarray(pixels, np.uint32)
        smp = np.ascontiguousarray(samples, np.uint32)
        if pix.shape != smp.shape or pix.ndim != 1:
            raise ValueError("pixels and samples must be 1-D arrays of one length")
        out = np.zeros((pix.shape[0], 3), np.float32)
        N.check(self._lib.pt_frame_samples(self.ptr, pix.ctypes.data, smp.ctypes.data, pix.shape[0], out.ctypes.data),
                self.ptr)
        return out

    def close(self):
        if self.ptr:
            self._lib.pt_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, flat, key=None):
        d = flat.desc()
        N.check(self._lib.pt_scene_upload(self.ptr, C.byref(d)), self.ptr)
        self.scene_key = key

    def set_stream(self, stream_ptr: int | None):
        N.check(self._lib.pt_set_stream(self.ptr, C.c_void_p(stream_ptr) if stream_ptr else None), self.ptr)

    def set_node_format(self, fmt: int):
        """pt_set_node_format: N.PT_NODES_AUTO / _FULL / _QUANTIZED (pool traversal node layout)."""
        N.check(self._lib.pt_set_node_format(self.ptr, int(fmt)), self.ptr)

    def render(self, cam: N.CameraDesc, rd: N.RenderDesc, film_ptr: int) -> dict:
        st = N.Stats()
        N.check(self._lib.pt_render(self.ptr, C.byref(cam), C.byref(rd), C.c_void_p(film_ptr), C.byref(st)), self.ptr)
        return st.as_dict()

    def render_adaptive(self, cam: N.CameraDesc, rd: N.RenderDesc, film_ptr: int) -> tuple[dict, np.ndarray]:
        """pt_render_adaptive: (stats, per-pixel sample counts (H, W) u32)."""
        st = N.Stats()
        counts = np.zeros((cam.height, cam.width), np.uint32)
        N.check(self._lib.pt_render_adaptive(self.ptr, C.byref(cam), C.byref(rd), C.c_void_p(film_ptr),
                                             counts.ctypes.data, C.byref(st)), self.ptr)
        return st.as_dict(), counts

    def render_samples(self, cam: N.CameraDesc, rd: N.RenderDesc, npix: int) -> tuple[np.ndarray, dict]:
        out = np.zeros((npix, rd.spp, 3), dtype=np.float32)
        st = N.Stats()
        L = self._lib
        L.pt_render_samples.argtypes = [C.c_void_p, C.POINTER(N.CameraDesc), C.POINTER(N.RenderDesc), C.c_void_p,
                                        C.POINTER(N.Stats)]
        L.pt_render_samples.restype = C.c_int32
        N.check(L.pt_render_samples(self.ptr, C.byref(cam), C.byref(rd), out.ctypes.data, C.byref(st)), self.ptr)
        return out, st.as_dict()

    def trace(self, rays: np.ndarray, any_hit: bool, stackless: bool = False) -> tuple[np.ndarray, dict]:
        """pt_trace: closest or any hit per ray (test hook); stackless: any hit
        through the stackless traversal (pt_trace any_hit 2)."""
        rays = np.ascontiguousarray(rays, dtype=N.RAY)
        hits = np.zeros(rays.shape[0], dtype=N.HIT)
        st = N.Stats()
        mode = (2 if stackless else 1) if any_hit else 0
        N.check(self._lib.pt_trace(self.ptr, rays.ctypes.data, rays.shape[0], mode, hits.ctypes.data,
                                   C.byref(st)), self.ptr)
        return hits, st.as_dict()


    def interact(self, rays: np.ndarray) -> np.ndarray:
        """Closest hit + reconstructed SurfaceInteraction per ray: (n, 16)
        {hit, t, p, n, ns, uv, tangent} (test hook)."""
        rays = np.ascontiguousarray(rays, dtype=N.RAY)
        out = np.zeros((rays.shape[0], 16), np.float32)
        N.check(self._lib.pt_interact(self.ptr, rays.ctypes.data, rays.shape[0], out.ctypes.data), self.ptr)
        return out

    def bsdf_cases(self, material: int, cases: np.ndarray) -> np.ndarray:
        """Material scatter / f / pdf on (n, 27) cases -> (n, 20) (test hook)."""
        cases = np.ascontiguousarray(cases, np.float32)
        out = np.zeros((cases.shape[0], 20), np.float32)
        N.check(self._lib.pt_bsdf_cases(self.ptr, int(material), cases.ctypes.data, cases.shape[0],
                                        out.ctypes.data), self.ptr)
        return out

    def light_picks(self, u: np.ndarray) -> np.ndarray:
        """LightSampler::Sample(u) on the device: picked light index per u (test hook)."""
        u = np.ascontiguousarray(u, np.float32)
        out = np.zeros(u.shape[0], np.int32)
        N.check(self._lib.pt_light_picks(self.ptr, u.ctypes.data, u.shape[0], out.ctypes.data), self.ptr)
        return out

    def anim_inverse(self, t: np.ndarray) -> np.ndarray:
        """The device's inverse of identity + translation t (AnimatedPrimitive's
        glm::inverse at a ray's time), (n, 3) -> (n, 16) column-major (test hook)."""
        t = np.ascontiguousarray(t, np.float32).reshape(-1, 3)
        out = np.zeros((t.shape[0], 16), np.float32)
        N.check(self._lib.pt_anim_inverse_cases(self.ptr, t.ctypes.data, t.shape[0], out.ctypes.data), self.ptr)
        return out

    def light_cases(self, cases: np.ndarray, n_lights: int) -> np.ndarray:
        """Light sample / PDF / L for every light x case: (n_lights*n, 18) (test hook)."""
        cases = np.ascontiguousarray(cases, np.float32)
        out = np.zeros((n_lights * cases.shape[0], 18), np.float32)
        N.check(self._lib.pt_light_cases(self.ptr, cases.ctypes.data, cases.shape[0], out.ctypes.data), self.ptr)
        return out


_contexts: dict[int, Context] = {}


def get_context(device: int = 0) -> Context:
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]


def render_desc(integrator: int, spp: int, max_depth: int, seed: int, film_filter, shard_index: int = 0,
                shard_count: int = 1, flags: int = 0, paths_in_flight: int = 0, pixel_begin: int = 0,
                pixel_end: int = 0, strata=(0, 0)) -> N.RenderDesc:
    rd = N.RenderDesc()
    rd.integrator = integrator
    rd.spp = int(spp)
    rd.max_depth = int(max_depth)
    rd.seed = int(seed) & 0xFFFFFFFF
    rd.filter = film_filter.kind
    rd.filter_radius[0] = float(film_filter.radius[0])
    rd.filter_radius[1] = float(film_filter.radius[1])
    p = film_filter.params()
    rd.filter_params[0] = float(p[0])
    rd.filter_params[1] = float(p[1])
    rd.shard_index = int(shard_index)
    rd.shard_count = int(shard_count)
    rd.flags = int(flags)
    rd.paths_in_flight = int(paths_in_flight)
    rd.pixel_begin = int(pixel_begin)
    rd.pixel_end = int(pixel_end)
    rd.strata[0], rd.strata[1] = int(strata[0]), int(strata[1])
    return rd


class Integrator:
    kind = N.PT_INTEGRATOR_PATH

    def __init__(self, scene: Scene, camera: Camera, sampler: Sampler, lightSampler: Optional[LightSampler],
                 maxDepth: int):
        self.scene = scene
        self.camera = camera
        self.sampler = sampler
        self.lightSampler = lightSampler
        self.maxDepth = int(maxDepth)
        if scene.flat is None:
            scene.BuildTlas()
        self.flat = bind_lights(scene.flat, scene, lightSampler)
        self.flat.medium_id(camera.GetMedium())  # registered before upload
        self.last_stats: dict = {}

    def context(self, device: int = 0) -> Context:
        ctx = get_context(device)
        key = (id(self.flat), id(self.lightSampler), len(self.flat.medium_ids))
        if ctx.scene_key != key:
            ctx.upload(self.flat, key)
        return ctx

    def desc(self, **kw) -> tuple[N.CameraDesc, N.RenderDesc]:
        film = self.camera.GetFilm()
        spp = kw.pop("spp", self.sampler.SamplesPerPixel())
        # a StratifiedSampler's strata, while its own sample count is rendered
        strata = getattr(self.sampler, "strata", (0, 0))
        if strata[0] * strata[1] != spp:
            strata = (0, 0)
        rd = render_desc(self.kind, spp, self.maxDepth, kw.pop("seed", self.sampler.seed), film.filter,
                         strata=kw.pop("strata", strata), **kw)
        return camera_desc(self.camera, self.flat), rd

    def Render(self, device: int = 0, shard_index: int = 0, shard_count: int = 1, flags: int = 0,
               film_ptr: int | None = None, paths_in_flight: int = 0, adaptive: bool = False) -> dict:
        """TileIntegrator::Render equivalent: accumulates into camera.GetFilm().accum
        (or into the float64 device buffer at film_ptr).

        adaptive=False renders exactly spp samples per pixel (the benchmark's
        fixed-SPP frame); adaptive=True runs the reference's own loop
        (Integrators.cpp:55-86): rounds of spp samples per pixel until the
        luminance-weighted relative variance of every channel is <= 1.5, at
        most 128*spp samples; the per-pixel sample counts land in
        `last_sample_counts` (H, W).  Shards then own 32x32 tiles, not samples."""
        ctx = self.context(device)
        cam, rd = self.desc(shard_index=shard_index, shard_count=shard_count, flags=flags,
                            paths_in_flight=paths_in_flight)
        film = self.camera.GetFilm()
        ptr = film_ptr if film_ptr is not None else film.accum.ctypes.data
        if adaptive:
            self.last_stats, self.last_sample_counts = ctx.render_adaptive(cam, rd, ptr)
        else:
            self.last_stats = ctx.render(cam, rd, ptr)
        return self.last_stats

    def RenderSamples(self, pixel_begin: int = 0, pixel_end: int = 0, spp: Optional[int] = None,
                      device: int = 0, flags: int = 0) -> np.ndarray:
        """Per-sample Li for pixels [pixel_begin, pixel_end): (npix, spp, 3) float32."""
        ctx = self.context(device)
        W, H = self.camera.GetFilm().Resolution()
        if pixel_begin == 0 and pixel_end == 0:
            pixel_end = W * H
        kw = {} if spp is None else {"spp": spp}
        cam, rd = self.desc(pixel_begin=pixel_begin, pixel_end=pixel_end, flags=flags, **kw)
        out, self.last_stats = ctx.render_samples(cam, rd, pixel_end - pixel_begin)
        return out


class PathIntegrator(Integrator):
    """PathIntegrator (Integrators.hpp:43-54): NEE + MIS (power heuristic) + RR."""
    kind = N.PT_INTEGRATOR_PATH


class VolPathIntegrator(Integrator):
    """VolPathIntegrator (Integrators.hpp:56-67, Integrators.cpp:296-479):
    PathIntegrator plus homogeneous media (Medium.hpp), Henyey-Greenstein
    phase sampling, NEE from medium points and transmittance along shadow rays
    (Scene::IntersectTr, Scene.cpp:8-29).  The medium's two hidden
    random_float() draws (Medium.hpp:28-30) come from the sample stream, right
    before the bounce's nine draws."""
    kind = N.PT_INTEGRATOR_VOLPATH


class SimplePathIntegrator(Integrator):
    """SimplePathIntegrator (Integrators.hpp:33-41): BSDF sampling + RR."""
    kind = N.PT_INTEGRATOR_SIMPLE

    def __init__(self, scene: Scene, camera: Camera, sampler: Sampler, maxDepth: int):
        super().__init__(scene, camera, sampler, None, maxDepth)
