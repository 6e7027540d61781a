#!/bin/bash
# one GPU call: bench rehearsal tests, then an instruction-mix PMC pass on the C2 bench (k_render)
R=$PWD
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/bench_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/bench_pytest.log; exit 1; }
tail -3 gpurun_out/bench_pytest.log
cd /tmp
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
  tag=$(echo $set | cut -c1-20 | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_$tag -- python3 $R/bench.py --no-cpu --steps 16 --warmup 1 > $R/gpurun_out/pmc_$tag.log 2>&1 || { echo "pmc failed $set"; tail $R/gpurun_out/pmc_$tag.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
res = collections.defaultdict(list)
for f in glob.glob('/root/repo/gpurun_out/pmc_*/*/*_counter_collection.csv') + glob.glob('/root/repo/gpurun_out/pmc_*/*_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_render<0, false>' in r['Kernel_Name']:
            res[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(res.items()):
    print(k, ['%.4g' % x for x in v])
PY
