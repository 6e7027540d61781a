#!/bin/bash
# one GPU call: bench.py lines for each workload x library variant
#   WLS="C5 C4" VARIANTS="base w4k16m0" STEPS=8 bash tools/sweep_bench.sh
export TMPDIR=/tmp
L=$PWD/montecarlopathtracing_amd/lib
for wl in $WLS; do
  for v in $VARIANTS; do
    so=$L/libmcpt_hip_$v.so; [ "$v" = "base" ] && so=$L/libmcpt_hip.so
    MCPT_LIB_OVERRIDE=$so timeout -k 10 300 python bench.py --no-cpu --workload $wl --steps ${STEPS:-16} --warmup 2 > gpurun_out/sb_${wl}_$v.json 2> gpurun_out/sb_${wl}_$v.err || { echo "bench $wl $v failed"; tail gpurun_out/sb_${wl}_$v.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/sb_${wl}_$v.json'));r=j['roofline'];print('$wl $v', j['value'], 'Msamples/s; seg/s', j['active_Msegments_per_s'], 'launch ms', r['avg_launch_ms'])"
  done
done
