#!/bin/bash
# one GPU call: the BVH-pass GPU tests + build timings
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "treelet or bvh" > gpurun_out/tl_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/tl_pytest.log; exit 1; }
tail -3 gpurun_out/tl_pytest.log
timeout -k 10 300 python tools/bench_build.py C2 C3 C5 > gpurun_out/tl_build.json 2> gpurun_out/tl_build.err || { echo "build bench failed"; tail gpurun_out/tl_build.err; exit 1; }
cat gpurun_out/tl_build.json
