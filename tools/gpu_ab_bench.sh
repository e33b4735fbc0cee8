# A/B of the bench step: in-tree library vs MH_LIB=$1 (profiles of both)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_a -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/ab_a.log 2>&1 || exit 1
MH_LIB=$R/$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_b -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/ab_b.log 2>&1 || exit 1
for x in a b; do python3 -c "
import csv, json
l=open('$R/gpurun_out/ab_$x.log').read().strip().splitlines()[-1]
print('$x', json.loads(l)['ms_per_step'])
for r in csv.reader(open('$R/gpurun_out/ab_$x/run_kernel_stats.csv')):
    if r[0]!='Name' and float(r[4])>1: print('   ', r[0][:45], r[1], r[3])"; done
