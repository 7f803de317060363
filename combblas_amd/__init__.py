"""combblas_amd -- MI355X (gfx950) semiring SpGEMM hot path of CombBLAS.

Python host mirror of the reference's local SpGEMM interface over the C-ABI in
include/combblas_hip.h. The compute path is HIP only (libcombblas_hip.so); importing the
kernels' entry points without the library raises.
"""
from .semirings import MinPlusSRing, OrAndSRing, PlusTimesSRing, SelectMaxSRing  # noqa: F401
from .spdccols import Context, HostDcsc, SpDCCols  # noqa: F401
from .mtspgemm import (EstimateLocalFLOP, LocalHybridSpGEMM, LocalSpGEMM, LocalSpGEMMHash,  # noqa: F401
                       MultiwayMerge, PhasedSpGEMM, SpGEMMPlan, estimateFLOPandNNZ)
from .rmat import rmat, rmat_edges  # noqa: F401

__all__ = ["Context", "HostDcsc", "SpDCCols", "PlusTimesSRing", "SelectMaxSRing", "MinPlusSRing", "OrAndSRing",
           "LocalHybridSpGEMM", "LocalSpGEMMHash", "LocalSpGEMM", "MultiwayMerge", "EstimateLocalFLOP",
           "estimateFLOPandNNZ", "PhasedSpGEMM", "rmat", "rmat_edges"]
