#!/bin/bash
for w in ${WAVES:-3 5 6}; do
  echo "== waves/SIMD target $w"
  MCPT_LIB_OVERRIDE=$PWD/montecarlopathtracing_amd/lib/libmcpt_hip_w$w.so timeout -k 10 120 python tools/quick_perf.py 16 1024 2>&1 | grep -v amdgpu.ids || exit 1
done
