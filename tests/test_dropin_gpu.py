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
    r = subprocess.run([HARNESS, str(scale)], env=env, capture_output=True, text=True, timeout=150, cwd="/tmp")
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    lines = [l for l in out.splitlines() if l.startswith("DROPIN")]
    # 5 arrival-order cases + Select2nd (non-commutative add) and non-dyadic f64 in reference order
    assert len(lines) == 7 and all(" OK " in l for l in lines), out
