#!/bin/bash
# one GPU call: parity tests + quick perf (+ optional VALU-utilisation PMC pass)
R=$PWD
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/check_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/check_pytest.log; exit 1; }
tail -2 gpurun_out/check_pytest.log
timeout -k 10 200 python tools/quick_perf.py 16 1024 > gpurun_out/check_perf.log 2>&1 || { echo "perf failed"; cat gpurun_out/check_perf.log; exit 1; }
cat gpurun_out/check_perf.log
if [ "$1" = "pmc" ]; then
  cd /tmp
  timeout -k 10 200 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/check_pmc -- python3 $R/bench.py --no-cpu --steps 16 --warmup 1 > $R/gpurun_out/check_pmc.log 2>&1 || exit 1
  python3 - <<'PY'
import csv, glob, collections
res = collections.defaultdict(list)
for f in glob.glob('/root/repo/gpurun_out/check_pmc/*/*_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_render<0, false>' in r['Kernel_Name']:
            res[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(res.items()):
    print(k, ['%.4g' % x for x in v])
if res:
    print('VALU lane util %.3f' % (res['SQ_THREAD_CYCLES_VALU'][-1] / (64 * res['SQ_INSTS_VALU'][-1])))
PY
fi
