cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1; echo rc=$?
