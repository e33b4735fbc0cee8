# full GPU suite + bench lines (round 4: host-side quotients, fast lane-map division)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4b.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4b_$i.json 2> gpurun_out/bench_r4b_$i.err || exit 1; done
timeout -k 10 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4_r4b.json 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_r4b.txt 2>&1 || exit 1
for d in "" --deterministic; do timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu $d > gpurun_out/pvp_r4b$d.json 2>&1 || exit 1; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r4b -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r4b.log 2>&1 || exit 1
