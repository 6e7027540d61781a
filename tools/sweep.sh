#!/bin/bash
# threshold sweep for the fused kernel's phase gating
for T in "1,1" "8,16" "16,32" "24,40" "32,48" "16,48" "8,32" "32,32"; do
  echo "== MCPT_PHASE_THRESHOLDS=$T"
  MCPT_PHASE_THRESHOLDS=$T timeout -k 10 120 python tools/quick_perf.py 16 1024 2>&1 | grep -v amdgpu.ids || exit 1
done
