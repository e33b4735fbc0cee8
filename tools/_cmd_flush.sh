# config 3 texel scatter: cost of the per-workgroup flush (MH_EXP_NO_FLUSH diagnostic: wrong gradients) and 1 / 2 workgroups per CU
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fl_def -o trace -- python3 $R/bench.py --config 3 --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/prof_fl_def.log 2>&1 || exit 1
MH_LIB=$R/gpurun_exp/lib_noflush.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fl_no -o trace -- python3 $R/bench.py --config 3 --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/prof_fl_no.log 2>&1 || exit 1
