# A/B: synchronous wrapper calls (sync=1, default) vs MH_ASYNC_CALLS=1 (sync=0) (bench step, no CPU leg)
for v in 0 1 0 1; do
  MH_ASYNC_CALLS=$((1-v)) timeout -k 10 200 python bench.py --no-cpu > gpurun_out/s$v.log 2>&1 || { tail -20 gpurun_out/s$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s$v.log').read().strip().splitlines()[-1]); print('sync=$v', d['ms_per_step'], d['fwd_kernel_ms'], d['bwd_kernel_ms'], d['roofline']['kernel_avg_us'], d['roofline'].get('clock_ghz'))"
done
