# deterministic replay / prbvolpath tests + full GPU suite + bench
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_parity.py -k "deterministic" -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest_det2.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4c.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4c_$i.json 2> gpurun_out/bench_r4c_$i.err || exit 1; done
timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu --deterministic > gpurun_out/pvp_det3.json 2>&1 || exit 1
