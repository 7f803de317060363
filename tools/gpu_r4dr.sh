# session run r4dr: dense split ratio re-tuned after the absolute window snap (dense 300 -> 280 ms)
set -o pipefail
OUT=gpurun_out/r4dr; mkdir -p $OUT; export TMPDIR=/tmp
for v in base dr8 dr9 dr6 base dr8 dr9 dr6; do
  if [ $v = base ]; then unset CBH_LIB; else export CBH_LIB=$v; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -20 $OUT/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/ab_$v.json')); k=d['config']['kernel_ms']; print('$v', d['value'], d['check']['ok'], 'dense', k['num_dense'], 'hash', k['num_large'], 'sym', k['sym_large'])"
done
echo "== $(date +%T) done"
