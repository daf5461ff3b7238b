"""MI355X-native sparse-voxel-octree primary-ray caster.

Drop-in for the SVO ray path of epitaque/RaytracingTest: the Unity host
driver RaytracingMaster + the HLSL IntersectSVO kernel become a C-ABI plugin
(include/svo_rt.h, libsvo_rt.so) launching hand-written gfx950 HIP kernels.
"""
from ._lib import HIT_DTYPE, STACK_EXACT, STACK_HLSL, SvoError
from .svo_data import SVOData, SVOFormatError
from .raytracing_master import RaytracingMaster, band_rows

__all__ = ["HIT_DTYPE", "STACK_EXACT", "STACK_HLSL", "SvoError", "SVOData", "SVOFormatError",
           "RaytracingMaster", "band_rows"]
