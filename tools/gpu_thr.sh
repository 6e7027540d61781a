#!/bin/bash
# phase-threshold sweep ("leaf,shade") of the working library vs prev at its default
export TMPDIR=/tmp
L=$PWD/montecarlopathtracing_amd/lib
for sc in ${SCENES:-cbox_diffuse}; do
  echo "== $sc prev: $(MCPT_LIB_OVERRIDE=$L/libmcpt_hip_prev.so QP_REPS=11 timeout -k 10 120 python tools/quick_perf.py 32 1024 $sc 2>&1 | grep -E 'stats=0' | sed 's/mode=0 stats=0 //')" || exit 1
  for t in ${THR:-2,32 4,32 8,32 4,24 4,40}; do
    echo "== $sc base $t: $(MCPT_PHASE_THRESHOLDS=$t QP_REPS=11 timeout -k 10 120 python tools/quick_perf.py 32 1024 $sc 2>&1 | grep -E 'stats=0' | sed 's/mode=0 stats=0 //')" || exit 1
  done
done
