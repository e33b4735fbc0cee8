# splat diagnostic: rocprof kernel stats of the bench with / without the footprint atomics
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_splat_def -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_splat_def.log 2>&1 || exit 1
MH_LIB=$GRAFT_REPO_ROOT/gpurun_exp/lib_noat.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_splat_noat -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_splat_noat.log 2>&1 || exit 1
