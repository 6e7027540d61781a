#!/bin/bash
# one GPU call: the whole GPU suite, quick perf, then the EPO goldens
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/all_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/all_pytest.log | head -20; tail -40 gpurun_out/all_pytest.log; exit 1; }
tail -3 gpurun_out/all_pytest.log
timeout -k 10 200 python tools/quick_perf.py 16 1024 > gpurun_out/check_perf.log 2>&1 || { echo "perf failed"; cat gpurun_out/check_perf.log; exit 1; }
cat gpurun_out/check_perf.log
if [ "$1" = "gold" ]; then
timeout -k 10 200 python tools/make_goldens.py bvh gpurun_out/golden > gpurun_out/gold.log 2>&1 || { echo "goldens failed"; tail gpurun_out/gold.log; exit 1; }
ls -la gpurun_out/golden
fi
