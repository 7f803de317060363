"""GPU: the reference's UNCHANGED Mult_AnXBn_Synch (PSpGEMM's driver) instantiated with
COMBBLAS_HIP_INSTANTIATE runs on the gfx950 kernels and matches the stock OpenMP path exactly
(tests/dropin/dropin_harness.cpp, built by `make -C oracle ref` where the reference exists)."""
import os
import subprocess

import pytest

import helpers as H

pytestmark = pytest.mark.gpu

HARNESS = os.path.join(H.REPO, "oracle", "_ref", "dropin_harness")


@pytest.mark.parametrize("scale", [8, 12, 16])  # 16: config C1 (MultTest plumbing, R-MAT scale 16)
def test_reference_driver_uses_hip_kernels(scale):
    assert os.path.exists(HARNESS), "oracle/_ref/dropin_harness missing: run __graft_entry__.build() with the reference"
    env = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib", OMP_NUM_THREADS="8")
    r = subprocess.run([HARNESS, str(scale)], env=env, capture_output=True, text=True, timeout=240, cwd="/tmp")
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    lines = [l for l in out.splitlines() if l.startswith("DROPIN")]
    # built-in PlusTimes<double> / SelectMax<int64> (library kernels, arrival order: exact on integer-valued
    # inputs), user KTips bool and promoted PlusTimes<double,int64> (default reference order), user struct
    # MinMax (arrival_order_ok opt-in), Select2nd (non-commutative add), marked PlusTimes f64 and an unmarked
    # non-commutative affine f64 semiring on non-dyadic values (reference order), and the built-in
    # PlusTimes<double> on non-dyadic values with COMBBLAS_HIP_ORDER=reference -- all bit-identical to the
    # stock driver (at scale 16: config C1 in the reference's own order, no tolerance)
    assert len(lines) == 9 and all(" OK " in l for l in lines), out
