R=$PWD; O=$R/gpurun_out/probe; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for lib in cur prev; do
  if [ $lib = prev ]; then export MCPT_LIB_OVERRIDE=$R/montecarlopathtracing_amd/lib/libmcpt_hip_prev.so; fi
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/${lib}_$c -- python3 $R/bench.py --no-cpu --steps 32 --warmup 0 > $O/${lib}_$c.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('/root/repo/gpurun_out/probe/*/*/*_counter_collection.csv')):
    rows = [r for r in csv.DictReader(open(f)) if 'k_render' in r['Kernel_Name']]
    print(f.split('/')[-3], [(r['Kernel_Name'][5:22], r['Counter_Value']) for r in rows])
PY
