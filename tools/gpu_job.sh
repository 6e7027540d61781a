#!/bin/bash
# One gpurun call = a list of steps, run in order; the first failure ends the
# call (no GPU work after a fault, an abort or a time limit).  Each step:
#   "pytest <files/args>"    python -m pytest -m gpu on them (per-test 300 s limit)
#   "profile <tag> <args>"   tools/profile.py run (bench line + rocprofv3 passes)
#   "sweep <args>"           tools/sweep.py        "ab <args>"   tools/ab.py
#   "bench <args>"           bench.py              "smoke"       __graft_entry__.smoke()
#   "run <command>"          any other command (600 s limit)
# Logs: gpurun_out/job_<k>_<kind>.log
#   gpurun -- bash tools/gpu_job.sh "pytest tests/test_gpu_parity.py" "bench --steps 20 --warmup 5"
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for step in "$@"; do
  k=$((k + 1))
  kind=${step%% *}
  rest=${step#"$kind"}
  log=gpurun_out/job_${k}_${kind}.log
  case $kind in
    pytest)  cmd="timeout -k 10 1100 python -u -m pytest $rest -x -q --timeout 300 --timeout-method thread -m gpu" ;;
    profile) cmd="timeout -k 10 1100 python3 -u tools/profile.py run $rest" ;;
    sweep)   cmd="timeout -k 10 900 python -u tools/sweep.py $rest" ;;
    ab)      cmd="timeout -k 10 900 python -u tools/ab.py $rest" ;;
    bench)   cmd="timeout -k 10 600 python -u bench.py $rest" ;;
    smoke)   cmd="timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
    run)     cmd="timeout -k 10 600 $rest" ;;
    *) echo "unknown step kind: $kind"; exit 2 ;;
  esac
  echo "=== step $k: $step"
  eval "$cmd" > "$log" 2>&1
  rc=$?
  tail -n 25 "$log"
  if [ $rc -ne 0 ]; then echo "=== step $k failed rc=$rc"; exit $rc; fi
done
echo "=== all $k steps ok"
