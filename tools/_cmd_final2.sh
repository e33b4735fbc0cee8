# round-4 final lines: bench (with its CPU leg) x2, configs 1 / 3 / 4 / 5, and the PMC passes bench.py reads (profiles/r4_pmc.json)
set -o pipefail
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/final_c2_$i.json 2> gpurun_out/final_c2_$i.err || exit 1; done
for c in 1 3 4; do timeout -k 10 300 python bench.py --config $c > gpurun_out/final_c$c.json 2> gpurun_out/final_c$c.err || exit 1; done
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 > gpurun_out/final_c5.json 2> gpurun_out/final_c5.err || exit 1
bash tools/profile_r2.sh gpurun_out/prof_r4f > gpurun_out/prof_r4f.log 2>&1 || exit 1
