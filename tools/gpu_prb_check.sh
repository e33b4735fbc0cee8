# PRB parity subset + bench step kernel stats of the in-tree library
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "prb or bitmap or config3 or multirank or smoke or linearity" > gpurun_out/prb_tests.log 2>&1 || { tail -30 gpurun_out/prb_tests.log; exit 1; }
tail -1 gpurun_out/prb_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pc -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/pc.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/pc.log
python3 -c "
import csv
for r in csv.reader(open('$R/gpurun_out/pc/run_kernel_stats.csv')):
    if r[0]!='Name' and float(r[4])>1: print('   ', r[0][:45], r[1], r[3])"
