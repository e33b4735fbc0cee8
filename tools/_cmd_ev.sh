# one event pair per chunk for the fused bounces vs 2 per bounce (the empty ones recorded after the last bounce)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_ev.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in ev2 ev18; do
    if [ $v = ev2 ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ev_${v}$i.json 2>/dev/null || exit 1
  done
done
