timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
QP_REPS=3 timeout -k 10 200 python tools/quick_perf.py 64 1024 || exit 1
QP_REPS=3 timeout -k 10 200 python tools/quick_perf.py 64 2048 || exit 1
timeout -k 10 600 python bench.py --workload C3 --no-cpu > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 900 python bench.py --workload C5 --no-cpu --steps 16 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
