#!/bin/bash
# one GPU call: parity tests on the diningroom proxy, then the C4 bench line
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k dining > gpurun_out/c4_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/c4_pytest.log; exit 1; }
tail -3 gpurun_out/c4_pytest.log
timeout -k 10 300 python bench.py --workload C4 --steps 16 --warmup 2 > gpurun_out/c4_bench.json 2> gpurun_out/c4_bench.err || { echo "bench failed"; tail gpurun_out/c4_bench.err; exit 1; }
cat gpurun_out/c4_bench.json
