#!/bin/bash
# one GPU call: parity of window-stack variants, then quick_perf per variant (C2 + optional scene)
#   VARIANTS="w4k0 w5k16" [PARITY="w6k8"] [SCENE=cbox_diffuse] bash tools/sweep_variants.sh
export TMPDIR=/tmp
L=$PWD/montecarlopathtracing_amd/lib
for v in $PARITY; do
  MCPT_LIB_OVERRIDE=$L/libmcpt_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "render or near or exact_equals or handoff" > gpurun_out/par_$v.log 2>&1 || { echo "parity $v failed"; tail -30 gpurun_out/par_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/par_$v.log)"
done
for v in $VARIANTS; do
  so=$L/libmcpt_hip_$v.so; [ "$v" = "base" ] && so=$L/libmcpt_hip.so
  echo "== $v"
  MCPT_LIB_OVERRIDE=$so timeout -k 10 120 python tools/quick_perf.py 16 1024 ${SCENE:-cbox_diffuse} 2>&1 | grep -v amdgpu.ids || exit 1
done
