export QP_REPS=5 MCPT_PHASE_THRESHOLDS=4,32
for fpl in 16 8; do for c in 2 4 8 16 32; do
  echo "== fpl $fpl chunk $c"
  QP_FPL=$fpl MCPT_QUEUE_CHUNK=$c timeout -k 10 120 python tools/quick_perf.py 64 1024 2>&1 | grep "stats=0" || exit 1
done; done
for t in 2,32 4,24 4,40 8,32; do
  echo "== fpl 16 chunk 8 th $t"
  QP_FPL=16 MCPT_QUEUE_CHUNK=8 MCPT_PHASE_THRESHOLDS=$t timeout -k 10 120 python tools/quick_perf.py 64 1024 2>&1 | grep "stats=0" || exit 1
done
