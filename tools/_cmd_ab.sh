# round 4 A/B (stream engine) + the prbvolpath traffic breakdown
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "large_mesh" -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_def.txt 2>&1 || exit 1
MH_LIB=gpurun_exp/lib_sorted.so timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_sorted.txt 2>&1 || exit 1
MH_LIB=gpurun_exp/lib_w5.so timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_w5.txt 2>&1 || exit 1
MH_BVH4Q=1 timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_q.txt 2>&1 || exit 1
bash tools/profile_pvb_traffic.sh gpurun_out/pvb_traffic
