#!/bin/bash
# round-end rehearsal: whole GPU suite, smoke(), then the C2 profile set (bench line + rocprofv3)
export TMPDIR=/tmp
[ -n "$SKIPTEST" ] || timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/final_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/final_pytest.log | head -20; tail -30 gpurun_out/final_pytest.log; exit 1; }
[ -n "$SKIPTEST" ] || tail -1 gpurun_out/final_pytest.log
[ -n "$SKIPTEST" ] || timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final_smoke.log; exit 1; }
[ -n "$SKIPTEST" ] || tail -2 gpurun_out/final_smoke.log
for wl in ${WLS:-C2}; do
  tag=${TAGP:-r01}; [ "$wl" != "C2" ] && tag=${tag}$(echo $wl | tr C c)
  bash tools/profile_round.sh $tag $wl || exit 1
done
