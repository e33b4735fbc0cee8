set -o pipefail
export MH_LIB=gpurun_exp/lib_cnt.so
timeout -k 10 120 python tools/exp_counts.py 64 > gpurun_out/cnt.log 2>&1 || { cat gpurun_out/cnt.log; exit 1; }
cat gpurun_out/cnt.log
unset MH_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1 || true
grep -i "VALU\|SQ_INST_CYCLES\|SQ_BUSY\|GRBM_GUI" $GRAFT_REPO_ROOT/gpurun_out/counters.txt | head -80
