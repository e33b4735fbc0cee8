set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MH_LIB=$R/gpurun_exp/lib_noflush.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg_prof3 -o run --output-format csv -- python3 $R/tools/bench_configs.py > $R/gpurun_out/cfg3.log 2>&1 || exit 1
grep "3(b)" $R/gpurun_out/cfg3.log
python3 -c "
import csv
for r in csv.reader(open('$R/gpurun_out/cfg_prof3/run_kernel_stats.csv')):
    if 'bitmap' in r[0]: print(r[0][:50], r[1:4])"
