#!/bin/bash
# one GPU call: BVH-pass / metric GPU tests, then the EPO goldens from the reference kernel
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/bvh_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/bvh_pytest.log; exit 1; }
tail -3 gpurun_out/bvh_pytest.log
timeout -k 10 200 python tools/make_goldens.py bvh gpurun_out/golden > gpurun_out/gold.log 2>&1 || { echo "goldens failed"; tail gpurun_out/gold.log; exit 1; }
ls -la gpurun_out/golden
