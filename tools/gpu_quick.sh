#!/bin/bash
# one GPU call: full GPU suite, then bench lines for the given workloads
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/q_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/q_pytest.log | head; tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -1 gpurun_out/q_pytest.log
for wl in ${WLS:-C2}; do
  timeout -k 10 300 python bench.py --no-cpu --workload $wl --steps ${STEPS:-64} --warmup 4 > gpurun_out/q_$wl.json 2> gpurun_out/q_$wl.err || { echo "bench $wl failed"; tail gpurun_out/q_$wl.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/q_$wl.json'));r=j['roofline'];print('$wl', j['value'], 'Msamples/s; seg/s', j['active_Msegments_per_s'], 'launch ms', r['avg_launch_ms'])"
done
