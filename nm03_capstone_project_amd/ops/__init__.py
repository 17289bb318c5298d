"""torch-tensor entry points of the gfx950 kernels (K1a median, K1b sharpen+band, K2 SRG+morph,
K4 JPEG, K5 3D SRG + cube dilation, K6 threshold) and plain-PyTorch fp32 references of the same ops (ops.reference).

Every wrapper takes CUDA (HIP) tensors, passes raw device pointers and the current torch stream to
the native launcher and returns torch tensors — there is no CPU/Python fallback: without the
native extension the call raises.
"""
from .kernels import (dilate3d, jpeg_encode, median2d, pack_bits, region_grow, region_grow3d,  # noqa: F401
                      sharpen_band, threshold, unpack_bits)
from . import reference  # noqa: F401
