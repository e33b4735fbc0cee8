# W splat (k_splat_px<1>) with its sample loop unrolled by 2 vs 1: rocprof kernel stats of the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_su1 -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_su1.log 2>&1 || exit 1
MH_LIB=$GRAFT_REPO_ROOT/gpurun_exp/lib_su2.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_su2 -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_su2.log 2>&1 || exit 1
