#!/bin/bash
# SQ counters of the C4 dot-form kernels (one TC step at scale 24).  gpurun -- bash tools/gpu_tcpmc.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-tcpmc}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --kernel-include-regex 'dot_' --output-format csv -d $OUT/pmc -o run -- \
  python3 $GRAFT_REPO_ROOT/bench_tc.py --no-cpu-baseline --steps 1 --warmup 0 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
python3 - $OUT/pmc/run_counter_collection.csv <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    v = c.get("SQ_INSTS_VALU", 0); s = c.get("SQ_INSTS_SALU", 0); l = c.get("SQ_INSTS_LDS", 0)
    w = c.get("SQ_WAIT_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1))
    bc = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1))
    print(f"{k:60s} VALU {v:.3e} SALU {s:.3e} LDS {l:.3e} wait {w:.2f} ldsconf {bc:.2f} busy {c.get('SQ_BUSY_CYCLES',0):.3e} wavecyc {c.get('SQ_WAVE_CYCLES',0):.3e}")
PY
