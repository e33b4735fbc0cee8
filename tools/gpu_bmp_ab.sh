set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bitmap" > gpurun_out/bmp_tests.log 2>&1 || { tail -30 gpurun_out/bmp_tests.log; exit 1; }
tail -1 gpurun_out/bmp_tests.log
timeout -k 10 200 python tools/bench_configs.py > gpurun_out/cfg_a.log 2>&1 || exit 1
grep "3(b)" gpurun_out/cfg_a.log
MH_LIB=gpurun_exp/lib_bmw5.so timeout -k 10 200 python tools/bench_configs.py > gpurun_out/cfg_b.log 2>&1 || exit 1
grep "3(b)" gpurun_out/cfg_b.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cfg_prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py > /dev/null 2>&1 || exit 1
grep -E "bitmap_scatter|true>\(|true, true" $GRAFT_REPO_ROOT/gpurun_out/cfg_prof2/run_kernel_stats.csv | cut -c1-60,300-400 | head
