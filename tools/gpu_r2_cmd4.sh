set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t4.log 2>&1 || { tail -40 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
for v in "" gpurun_exp/lib_w4.so gpurun_exp/lib_nodef.so; do
  echo "== MH_LIB=$v"
  MH_LIB=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b4.log 2>&1 || { cat gpurun_out/b4.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b4.log').read().strip().split('\n')[-1]);print(d['value'],d['ms_per_step'],d['fwd_kernel_ms'],d['bwd_kernel_ms'],d['roofline']['kernel_avg_us'])"
done
