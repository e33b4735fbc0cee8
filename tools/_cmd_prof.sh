# round-4 profiles: bench PMC (r4_pmc.json), large-mesh traversal rooflines, 2-rank gloo rehearsal of the packed step
set -o pipefail
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/bench_r4_$i.json 2> gpurun_out/bench_r4_$i.err || exit 1; done
timeout -k 10 300 python bench.py --config 4 --no-cpu > gpurun_out/bench_c4_r4.json 2> gpurun_out/bench_c4_r4.err || exit 1
bash tools/profile_r2.sh gpurun_out/prof_r4 > gpurun_out/prof_r4.log 2>&1 || exit 1
bash tools/profile_mesh.sh gpurun_out/prof_mesh_1m 1000000 > gpurun_out/prof_mesh_1m.log 2>&1 || exit 1
bash tools/profile_mesh.sh gpurun_out/prof_mesh_4m 4000000 > gpurun_out/prof_mesh_4m.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_n2_gloo_r4.json 2> gpurun_out/bench_n2_gloo_r4.err || exit 1
bash tools/profile_volsched.sh gpurun_out/prof_vs > gpurun_out/prof_vs.log 2>&1 || exit 1
for d in "" --deterministic; do timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu $d > gpurun_out/pvp_det$d.json 2>&1 || exit 1; done
