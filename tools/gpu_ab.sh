#!/bin/bash
# A/B of the working library against libmcpt_hip_prev.so: parity suites on the
# working one, then interleaved quick_perf runs per scene
export TMPDIR=/tmp
L=$PWD/montecarlopathtracing_amd/lib
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/ab_pytest.log 2>&1 || { echo "parity failed"; grep -E "FAILED|Error|assert" gpurun_out/ab_pytest.log | head -20; tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
fi
for sc in ${SCENES:-cbox_diffuse mis}; do
  for v in prev base prev base; do
    so=$L/libmcpt_hip_$v.so; [ "$v" = "base" ] && so=$L/libmcpt_hip.so
    echo "== $sc $v: $(MCPT_LIB_OVERRIDE=$so QP_REPS=${REPS:-11} timeout -k 10 120 python tools/quick_perf.py ${FRAMES:-32} 1024 $sc 2>&1 | grep -E 'stats=0|SIMT' | sed 's/mode=0 stats=0 //' | tr '\n' ' ')" || exit 1
  done
done
