set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t0.log 2>&1 || { tail -30 gpurun_out/t0.log; exit 1; }
tail -2 gpurun_out/t0.log
timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b0.log 2>&1 || exit 1
cat gpurun_out/b0.log
