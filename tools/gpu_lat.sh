#!/bin/bash
# L1 / L2 request rates and latencies of k_render (C2 bench)
R=$PWD
export TMPDIR=/tmp
cd /tmp
for set in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_BUSY_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum TCP_TOTAL_READ_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"; do
  tag=$(echo $set | cut -c1-24 | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/lat_$tag -- python3 $R/bench.py --no-cpu --steps 8 --warmup 1 > $R/gpurun_out/lat_$tag.log 2>&1 || { echo "pmc failed: $set"; tail -5 $R/gpurun_out/lat_$tag.log; }
done
python3 - <<'PY'
import csv, glob, collections
res = collections.defaultdict(list)
for f in glob.glob('/root/repo/gpurun_out/lat_*/*/*_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_render<0, false, false' in r['Kernel_Name']:
            res[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(res.items()):
    print('%-36s %s' % (k, ' '.join('%.4g' % x for x in v)))
PY
