"""sqrtlm — MI355X-native square-root Levenberg–Marquardt bundle adjustment.

Python surface over libsqrtlm.so (include/sqrtlm.h). The compute path is the
HIP library; this package only marshals arrays and mirrors the reference's
``Optimizer`` BA entry points.
"""
from .problem import BAProblem, HUBER_MONO_GBA, HUBER_MONO_LBA, CHI2_MONO  # noqa: F401

__all__ = ["BAProblem", "HUBER_MONO_GBA", "HUBER_MONO_LBA", "CHI2_MONO", "Context", "Optimizer"]


def __getattr__(name):
    if name in ("Context", "Optimizer", "comm_unique_id", "pose_from_Tcw_f32", "pose_to_Tcw_f32"):
        from . import optimizer
        return getattr(optimizer, name)
    raise AttributeError(name)
