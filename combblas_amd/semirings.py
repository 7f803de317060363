"""Semiring descriptors of the device path (reference: include/CombBLAS/Semirings.h).

A descriptor names a device functor compiled into libcombblas_hip.so (combblas_amd/csrc/
semiring.h); the element type comes from the operands, as with the reference's
SR<T1,T2> where T1 == T2 == T_promote on every hot-path call site.
"""
from __future__ import annotations


class Semiring:
    def __init__(self, name, code, ref, commutative=True):
        self.name, self.code, self.ref, self.commutative = name, code, ref, commutative

    def __repr__(self):
        return f"<{self.name} ({self.ref})>"


PlusTimesSRing = Semiring("PlusTimesSRing", 0, "Semirings.h:212-232")
SelectMaxSRing = Semiring("SelectMaxSRing", 1, "Semirings.h:165-187")
MinPlusSRing = Semiring("MinPlusSRing", 2, "Semirings.h:235-255")
# boolean OR-AND (PlusTimesSRing<bool,bool>, ReleaseTests/KTipsTest.cpp:12-20 KTipsSR)
OrAndSRing = Semiring("OrAndSRing", 3, "KTipsTest.cpp:12-20")

ALL = {s.name: s for s in (PlusTimesSRing, SelectMaxSRing, MinPlusSRing, OrAndSRing)}
