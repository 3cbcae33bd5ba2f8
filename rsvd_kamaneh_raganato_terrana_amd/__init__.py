"""rsvd_kamaneh_raganato_terrana_amd -- MI355X-native randomized SVD.

Drop-in for the rSVD() / intermediate_step() / generateOmega() / QR() / SVD<method> path of
AMSC22-23/rSVD_Kamaneh_Raganato_Terrana: a C ABI (include/rsvd_c.h, librsvd_hip.so) over
hand-written gfx950 HIP kernels; this package is the Python host front end over that ABI.
"""
from ._capi import build, row_partition, RSVDError, LIB_PATH  # noqa: F401
from .api import (  # noqa: F401
    Engine,
    QRMode,
    SVD,
    SVDMethod,
    colmajor,
    default_engine,
    empty_colmajor,
    generateOmega,
    intermediate_step,
    make_allreduce_hook,
    make_collective_hook,
    qr_decomposition_full,
    qr_decomposition_reduced,
    rSVD,
    rSVD_image_compression,
)

__all__ = [
    "build", "row_partition", "RSVDError", "Engine", "QRMode", "SVDMethod", "colmajor",
    "default_engine", "empty_colmajor", "generateOmega", "intermediate_step", "make_allreduce_hook",
    "make_collective_hook", "rSVD",
    "rSVD_image_compression",
    "SVD", "qr_decomposition_full", "qr_decomposition_reduced",
]
