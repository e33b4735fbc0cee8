# full GPU suite + bench lines + A/Bs (round 4 HEAD)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4.json 2> gpurun_out/bench_r4.err || exit 1
for i in 1 2; do
  for v in noslp segold def; do
    if [ $v = def ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_${v}$i.json 2>/dev/null || exit 1
  done
done
unset MH_LIB
for v in def noslp segold; do
  if [ $v = def ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
  timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_$v.txt 2>&1 || exit 1
  timeout -k 10 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4_$v.json 2>/dev/null || exit 1
done
unset MH_LIB
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c5_r4.json 2> gpurun_out/bench_c5_r4.err || exit 1
for c in 1 3; do timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_c${c}_r4.json 2> gpurun_out/bench_c${c}_r4.err || exit 1; done
