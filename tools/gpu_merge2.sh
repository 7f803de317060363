#!/bin/bash
# merge-path MultiwayMerge (k = 2): the merge tests, then the bench's merge sample A/B
set -o pipefail
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_dist_gpu.py tests/test_devpath_gpu.py tests/test_devpath3d_gpu.py tests/test_dropin3d_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_merge.log 2>&1 || { tail -40 $OUT/pytest_merge.log; exit 1; }
tail -1 $OUT/pytest_merge.log
timeout -k 10 300 python -u - > $OUT/merge_ab.txt 2>&1 <<'PY' || { tail -30 $OUT/merge_ab.txt; exit 1; }
import os, sys, json
sys.path.insert(0, ".")
import numpy as np
import torch
torch.cuda.set_device(0)
import bench, combblas_amd as cb
A = cb.rmat(22, 16, dtype=np.float64)
for v in ("1", "0", "1"):
    os.environ["CBH_MERGE2"] = v
    import importlib
    r = bench.merge_measurement(A, 1 / 16, 3)
    print(v, json.dumps(r), flush=True)
PY
cat $OUT/merge_ab.txt | cut -c1-400
