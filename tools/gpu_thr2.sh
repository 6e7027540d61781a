#!/bin/bash
# phase-threshold sweep of the paired schedule on bench workloads
export TMPDIR=/tmp
for wl in ${WLS:-C2 C4}; do
  for t in ${THR:-12,32 8,32 16,32 12,24 12,40}; do
    MCPT_PHASE_THRESHOLDS=$t timeout -k 10 300 python bench.py --no-cpu --workload $wl --steps ${STEPS:-32} --warmup 2 --schedule ${SCH:-paired} > gpurun_out/t2_${wl}_$t.json 2> gpurun_out/t2_${wl}_$t.err || { echo "bench $wl $t failed"; tail gpurun_out/t2_${wl}_$t.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/t2_${wl}_$t.json'));r=j['roofline'];print('$wl $t', j['value'], 'launch ms', r['avg_launch_ms'])"
  done
done
