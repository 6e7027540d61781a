#!/bin/bash
# tuning sweep of one env knob over quick_perf (C2):  VAR=MCPT_QUEUE_CHUNK VALS="1 16 64" bash tools/sweep_env.sh [scene]
for v in $VALS; do
  echo "== $VAR=$v"
  env $VAR=$v timeout -k 10 120 python tools/quick_perf.py 16 1024 ${1:-cbox_diffuse} 2>&1 | grep -v amdgpu.ids || exit 1
done
