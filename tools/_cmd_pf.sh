# k_vol_sched next-lookup prefetch: volpath parity + config-4 A/B (same box) + prefetch hit count
set -o pipefail
MH_LIB=gpurun_exp/lib_lookups.so timeout -k 10 200 python bench.py --config 4 --steps 1 --warmup 0 --no-cpu > gpurun_out/pf_hits.json 2> gpurun_out/pf_hits.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_aux.py -k "volpath or config4" -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_pf.log 2>&1 || exit 1
for i in 1 2; do
  for v in pf nopf; do
    if [ $v = pf ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/pf_c4_${v}$i.json 2>/dev/null || exit 1
  done
done
