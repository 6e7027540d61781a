#!/bin/bash
# which vector-memory unit binds k_render: TA / TD / TCP busy vs GPU active cycles
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/avail.txt 2>&1 || true
grep -oE "\b(TA|TD|TCP|GRBM)_[A-Z0-9_]+" $R/gpurun_out/avail.txt | sort -u > $R/gpurun_out/avail_names.txt || true
wc -l $R/gpurun_out/avail_names.txt
for set in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  tag=$(echo $set | cut -c1-24 | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/ta_$tag -- python3 $R/bench.py --no-cpu --steps 8 --warmup 1 > $R/gpurun_out/ta_$tag.log 2>&1 || { echo "pmc failed: $set"; tail -5 $R/gpurun_out/ta_$tag.log; }
done
python3 - <<'PY'
import csv, glob, collections
res = collections.defaultdict(list)
for f in glob.glob('/root/repo/gpurun_out/ta_*/*/*_counter_collection.csv') + glob.glob('/root/repo/gpurun_out/ta_*/*_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_render<0, false' in r['Kernel_Name']:
            res[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(res.items()):
    print('%-40s %.4g (n=%d)' % (k, sum(v) / len(v), len(v)))
PY
