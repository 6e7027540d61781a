timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/bench_build.py C2 C3 C5 > gpurun_out/build.json 2> gpurun_out/build.err || { tail gpurun_out/build.err; exit 1; }
cat gpurun_out/build.json
