set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t7.log 2>&1 || { tail -40 gpurun_out/t7.log; exit 1; }
tail -2 gpurun_out/t7.log
bash tools/gpu_ab.sh base gpurun_exp/lib_w4.so
