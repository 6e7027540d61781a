"""MI355X-native Monte Carlo path tracer: the per-pixel, per-sample hot path of
SiodomeHuu/MonteCarloPathTracing (generateRay -> [intersect -> shade] x depth ->
history accumulate) as hand-written HIP kernels for gfx950 behind a C ABI
(include/mcpt_hip.h), with the reference's config.json / OBJ+MTL / .hdr surface.

Modules mirror the reference's host modules:
    config  - MCPT::Config           (config.cpp)
    scene   - ThirdPartyWrapper, Auxiliary::parseCamera, SceneCL packing, HLBVH
    render  - OpenCLBasic/RayGeneration/SceneBuild/ColorOut device side
    app     - OpenCL::init/update frame loop + .hdr dump (OpenCLApp.cpp, colorout.cpp)
    dist    - one-process-per-GPU tile sharding + RCCL reduce
"""
from . import _lib
from ._lib import MCPTError, lib

__all__ = ["MCPTError", "lib", "_lib"]
