# -m gpu suite, then three default-config bench lines (no CPU leg)
set -o pipefail
bash tools/gpu_tests.sh || exit 1
for i in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b$i.log 2>&1 || { tail -20 gpurun_out/b$i.log; exit 1; }; python3 -c "
import json; d=json.loads(open('gpurun_out/b$i.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['fwd_kernel_ms'], d['bwd_kernel_ms'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])"; done
