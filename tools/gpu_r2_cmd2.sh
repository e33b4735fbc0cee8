set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1 || { tail -60 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b2.log 2>&1 || { cat gpurun_out/b2.log; exit 1; }
cat gpurun_out/b2.log
timeout -k 10 300 python tools/bench_config5.py > gpurun_out/c5.log 2>&1 || { cat gpurun_out/c5.log; exit 1; }
cat gpurun_out/c5.log
