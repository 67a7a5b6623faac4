"""uasl_motion_estimation_amd — MI355X-native stereo-VO hot path.

A from-scratch HIP/CDNA4 implementation of the inner loop of
abeauvisage/uasl_motion_estimation: mutual-information patch scores and the
MI stereo-scale optimiser, KLT track updates, scanline NMS and the windowed
stereo bundle adjuster (residual/Jacobian kernels + on-device Schur on FP64
MFMA), behind the C ABI of include/me_hip.h (libme_hip.so).
"""
from ._lib import Context, MEError, default_context, device_count, load_library  # noqa: F401

__all__ = ["Context", "MEError", "default_context", "device_count", "load_library"]
