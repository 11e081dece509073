"""MI355X-native wavefront path tracer with the API of marko176/PathTracing.

The scene API (pathtracing_amd.scene) mirrors the reference's classes; the
per-sample hot loop (integrator + BVH4 traversal + material/light evaluation)
runs as hand-written HIP kernels for gfx950 behind the C ABI of
include/pt_api.h (libpt_hip.so).  See DESIGN.md.
"""
from .scene import (AlphaMode, AlphaTester, AreaLight, BoxFilter, Camera, CheckerTexture, DistantLight, Film,
                    FunctionInfiniteLight, GaussianFilter, LanczosFilter, GeometricPrimitive, HenyeyGreenstein, HomogeneusMedium,
                    ImageTexture,
                    MicrofacetDielectric, MicrofacetDiffuse, MitchellFilter, Mesh, Model, PointLight,
                    PowerLightSampler, QuadShape, Scene, SolidColor, SpecularConductor, SphereShape, ThinDielectric,
                    UniformInfiniteLight, UniformLightSampler)
from .integrator import (PathIntegrator, PCGSampler, SimplePathIntegrator, StratifiedSampler, UniformSampler,
                         VolPathIntegrator,
                         get_context)

__all__ = [n for n in dir() if not n.startswith("_")]
