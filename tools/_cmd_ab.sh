# full GPU suite + bench lines + stream-engine A/B (round 4 HEAD)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4.json 2> gpurun_out/bench_r4.err || exit 1
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c5_r4.json 2> gpurun_out/bench_c5_r4.err || exit 1
timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_def.txt 2>&1 || exit 1
MH_PRIMC=1 timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_primc.txt 2>&1 || exit 1
MH_BVH4Q=1 timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_q.txt 2>&1 || exit 1
