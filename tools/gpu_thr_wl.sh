#!/bin/bash
# Phase-threshold sweep ("leaf,shade") on one workload's bench line (paired schedule)
export TMPDIR=/tmp
WL=${WL:-C5}; st=${STEPS:-32}
for th in ${THS:-16,32 8,32 32,32 16,16 16,48 24,24}; do
  MCPT_PHASE_THRESHOLDS=$th timeout -k 10 300 python bench.py --no-cpu --workload $WL --steps $st --warmup 4 --schedule paired > gpurun_out/thr.json 2> gpurun_out/thr_err.log || { echo "bench failed"; tail gpurun_out/thr_err.log; exit 1; }
  python3 -c "import json;j=json.loads(open('gpurun_out/thr.json').read().strip().splitlines()[-1]);print('$WL th=$th', j['value'], j['roofline']['avg_launch_ms'])"
done
