#!/bin/bash
# One GPU call: the default bench line, then rocprofv3 kernel-trace/stats of the
# same command, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (MI355X_MICROARCH.md HBM section).  Outputs under gpurun_out/prof_<tag>/;
# tools/summarize_profiles.py <tag> copies them into profiles/.
#   bash tools/profile_round.sh r01 [workload]
TAG=${1:-r01}
WL=${2:-C2}
R=$PWD
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
STEPS=${STEPS:-64}
timeout -k 10 400 python bench.py --workload $WL --steps $STEPS > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cat $O/bench.json
# the profiled runs use the schedule the bench line's tuning picked (no tuning launches in the traces)
SCHED=$(python3 -c "import json,sys;print(json.loads(open('$O/bench.json').read().strip().splitlines()[-1])['config']['schedule'])")
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- \
  python3 $R/bench.py --no-cpu --workload $WL --steps $STEPS --warmup $STEPS --schedule $SCHED > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -- \
    python3 $R/bench.py --no-cpu --workload $WL --steps $STEPS --warmup $STEPS --schedule $SCHED > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail $O/pmc_$c.log; exit 1; }
done
echo profile done
