set -o pipefail
bash tools/profile_r2.sh gpurun_out/prof_r2 > gpurun_out/prof_r2.txt 2>&1 || { tail -30 gpurun_out/prof_r2.txt; tail -30 gpurun_out/prof_r2/log.txt; exit 1; }
cat gpurun_out/prof_r2.txt
mkdir -p profiles && cp gpurun_out/prof_r2/pmc.json profiles/r2_pmc.json
timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b10.log 2>&1 || { cat gpurun_out/b10.log; exit 1; }
tail -1 gpurun_out/b10.log
