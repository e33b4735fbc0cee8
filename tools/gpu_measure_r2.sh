# Round-2 measurement refresh (GPU box): the default bench line (with the CPU
# baseline), the rocprofv3 kernel stats of the same command, per-config timings
# (configs 2 / 3(a) / 3(b) / 4 / prbvolpath) and the config-5 slab.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/meas
timeout -k 10 300 python bench.py > gpurun_out/meas/bench_line.txt 2> gpurun_out/meas/bench_err.txt || { tail -20 gpurun_out/meas/bench_err.txt; exit 1; }
tail -1 gpurun_out/meas/bench_line.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/meas/bstats -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/gpurun_out/meas/bench_rocprof_line.txt 2>&1 || exit 1
cd $R
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/meas/configs.txt 2>&1 || { tail -20 gpurun_out/meas/configs.txt; exit 1; }
timeout -k 10 300 python tools/bench_config5.py > gpurun_out/meas/config5.txt 2>&1 || { tail -20 gpurun_out/meas/config5.txt; exit 1; }
tail -12 gpurun_out/meas/configs.txt; tail -4 gpurun_out/meas/config5.txt
