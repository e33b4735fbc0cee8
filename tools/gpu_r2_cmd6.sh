set -o pipefail
bash tools/gpu_ab.sh base gpurun_exp/lib_t2.so gpurun_exp/lib_s2.so || exit 1
bash tools/profile_gpu.sh gpurun_out/prof_r2a > gpurun_out/prof_r2a.txt 2>&1 || { tail -20 gpurun_out/prof_r2a.txt; exit 1; }
tail -20 gpurun_out/prof_r2a.txt
