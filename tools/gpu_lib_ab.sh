#!/bin/bash
# Bench lines of the working library vs lib/libmcpt_hip_$ALT.so per workload,
# interleaved; render parity suites on the alternative first
export TMPDIR=/tmp
L=$PWD/montecarlopathtracing_amd/lib
ALT=$L/libmcpt_hip_${ALT:-alt}.so
MCPT_LIB_OVERRIDE=$ALT timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/libab_pytest.log 2>&1 || { echo "parity failed"; grep -E "FAILED|Error|assert" gpurun_out/libab_pytest.log | head -20; tail -30 gpurun_out/libab_pytest.log; exit 1; }
tail -1 gpurun_out/libab_pytest.log
for wl in ${WLS:-C2 C3 C4 C5}; do
  st=64; [ "$wl" = "C4" ] && st=16
  for v in base alt base alt; do
    so=$L/libmcpt_hip.so; [ "$v" = "alt" ] && so=$ALT
    MCPT_LIB_OVERRIDE=$so timeout -k 10 300 python bench.py --no-cpu --workload $wl --steps $st --warmup 4 > gpurun_out/libab.json 2> gpurun_out/libab_err.log || { echo "bench failed"; tail gpurun_out/libab_err.log; exit 1; }
    python3 -c "import json;j=json.loads(open('gpurun_out/libab.json').read().strip().splitlines()[-1]);r=j['roofline'];print('$wl $v', j['value'], r['avg_launch_ms'], r['kernel_node_fetches_per_seg'], r['kernel_tri_tests_per_seg'], j['config']['schedule'])"
  done
done
