# A/B bench of library variants: bash tools/gpu_ab.sh <lib.so | ""> ...   ("" = in-tree library)
set -o pipefail
for v in "$@"; do
  [ "$v" = base ] && v=""
  MH_LIB=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().split('\n')[-1]);print(sys.argv[1], d['value'],d['ms_per_step'],d['fwd_kernel_ms'],d['bwd_kernel_ms'],d['roofline']['kernel_avg_us'])" "${v:-base}"
done
