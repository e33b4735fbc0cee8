# bitmap PRB: parity tests (fused wavefront + replay) and config timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread -k "bitmap or smooth_normals_prb" > gpurun_out/bmp_tests.log 2>&1 || { tail -40 gpurun_out/bmp_tests.log; exit 1; }
tail -3 gpurun_out/bmp_tests.log
timeout -k 10 200 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log
