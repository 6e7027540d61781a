#!/bin/bash
# bench.py lines of the working library vs libmcpt_hip_prev.so (and env variants)
export TMPDIR=/tmp
L=$PWD/montecarlopathtracing_amd/lib
for wl in ${WLS:-C3 C4 C5}; do
  for v in ${VARS:-prev base base8}; do
    # v = lib[:leaf,shade]  (lib: prev or base)
    lib=${v%%:*}; so=$L/libmcpt_hip_$lib.so; env=""
    [ "$lib" = "base" ] && so=$L/libmcpt_hip.so
    [ "$v" != "$lib" ] && env="MCPT_PHASE_THRESHOLDS=${v#*:}"
    env="$env ${ENVX:-}"
    env MCPT_LIB_OVERRIDE=$so $env timeout -k 10 300 python bench.py --no-cpu --workload $wl --steps ${STEPS:-16} --warmup 2 ${BARGS:-} > gpurun_out/ab_${wl}_${v/:/_}.json 2> gpurun_out/ab_${wl}_${v/:/_}.err || { echo "bench $wl $v failed"; tail gpurun_out/ab_${wl}_${v/:/_}.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/ab_${wl}_${v/:/_}.json'));r=j['roofline'];print('$wl $v', j['value'], 'launch ms', r['avg_launch_ms'])"
  done
done
