#!/bin/bash
# frames-per-block sweep of the default bench (C2, 64 frames per call)
export TMPDIR=/tmp
for f in ${FPLS:-8 16 32 64}; do
  timeout -k 10 300 python bench.py --no-cpu --workload ${WL:-C2} --steps 64 --warmup 4 --frames-per-launch $f --schedule ${SCH:-paired} > gpurun_out/fpl_$f.json 2> gpurun_out/fpl_$f.err || { echo "bench $f failed"; tail gpurun_out/fpl_$f.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/fpl_$f.json'));r=j['roofline'];print('fpl $f', j['value'], 'launch ms', r['avg_launch_ms'])"
done
