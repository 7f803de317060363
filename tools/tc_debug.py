#!/usr/bin/env python3
"""Dev tool: consistency checks of the dot-form TC path at a given scale (GPU box).
    python tools/tc_debug.py 20 22
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import combblas_amd as cb
    from bench_tc import host_check
    from combblas_amd.apps import MaskedSpGEMM, TCLower, Transpose
    from combblas_amd.semirings import PlusTimesSRing

    ctx = cb.Context(0)
    for s in [int(x) for x in sys.argv[1:]]:
        L = TCLower(ctx, s)
        L2 = TCLower(ctx, s)
        cp, jc, ir, num = L.tensors()
        colof = torch.repeat_interleave(jc, cp[1:] - cp[:-1])
        ok_l = bool((num == (ir.long() > colof).long()).all().item())
        AT = Transpose(L)
        tcp, tjc, tir, tnum = AT.tensors()
        ok_t = bool(torch.equal(tcp, cp) and torch.equal(tjc, jc) and torch.equal(tir, ir)
                    and torch.equal(tnum, (colof > ir.long()).long()))
        AT.free()
        print(f"scale {s}: nnzL {L.nnz} L values ok {ok_l}; transpose ok {ok_t}", flush=True)
        C = MaskedSpGEMM(PlusTimesSRing, L, L2, L, method="dot")
        ctx.synchronize()
        tri = int(C.tensors()[3].sum().item())
        checked, bad = host_check(L, C, 100)
        print(f"scale {s}: nnzC {C.nnz} triangles {tri} sampled columns {checked} mismatches {bad}", flush=True)
        for S in (C, L, L2):
            S.free()
    ctx.close()


if __name__ == "__main__":
    main()
