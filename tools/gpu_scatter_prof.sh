set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/profile_sq_script.sh gpurun_out/sq_bmp tools/bench_bitmap.py --reps 1 > gpurun_out/sq_bmp.txt 2>&1 || { tail -20 gpurun_out/sq_bmp.txt; tail -20 gpurun_out/sq_bmp/log.txt; exit 1; }
grep -E "scatter|bounce_prb" gpurun_out/sq_bmp.txt
MH_PRB_LDS_TEX=0 timeout -k 10 100 python tools/bench_bitmap.py > gpurun_out/bmp_glob.log 2>&1 || exit 1
tail -1 gpurun_out/bmp_glob.log
timeout -k 10 100 python tools/bench_bitmap.py > gpurun_out/bmp_lds.log 2>&1 || exit 1
tail -1 gpurun_out/bmp_lds.log
