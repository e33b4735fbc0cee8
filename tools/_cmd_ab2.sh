# same-box A/B: previous commit's library vs HEAD (host quotients + fast lane-map division) vs HEAD with compiler divisions
set -o pipefail
for i in 1 2; do
  for v in prev cur nofd; do
    if [ $v = cur ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab2_${v}$i.json 2>/dev/null || exit 1
  done
done
unset MH_LIB
MH_PRIMC=1 timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_primc.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_base.txt 2>&1 || exit 1

timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "deterministic" -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_det.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu --deterministic > gpurun_out/pvp_det2.json 2>&1 || exit 1
