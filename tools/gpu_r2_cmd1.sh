set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_multirank.py "tests/test_gpu_parity.py" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -5 gpurun_out/t1.log
timeout -k 10 300 python tools/bench_config5.py > gpurun_out/c5.log 2>&1 || { cat gpurun_out/c5.log; exit 1; }
cat gpurun_out/c5.log
