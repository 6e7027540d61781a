#!/bin/bash
# parity suites (incl. the paired schedule), then bench lines with auto schedule
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/sched_pytest.log 2>&1 || { echo "parity failed"; grep -E "FAILED|Error|assert" gpurun_out/sched_pytest.log | head -20; tail -30 gpurun_out/sched_pytest.log; exit 1; }
tail -1 gpurun_out/sched_pytest.log
for wl in ${WLS:-C2 C3 C4}; do
  for sc in ${SCHEDS:-auto single paired}; do
    timeout -k 10 300 python bench.py --no-cpu --workload $wl --steps ${STEPS:-32} --warmup 2 --schedule $sc > gpurun_out/sch_${wl}_$sc.json 2> gpurun_out/sch_${wl}_$sc.err || { echo "bench $wl $sc failed"; tail gpurun_out/sch_${wl}_$sc.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/sch_${wl}_$sc.json'));r=j['roofline'];print('$wl $sc ->', j['config']['schedule'], j['value'], 'launch ms', r['avg_launch_ms'])"
  done
done
