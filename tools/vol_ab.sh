# A/B of library variants on the config-4 volpath bench: bash tools/vol_ab.sh <lib.so | base> ...
# (env of the caller applies to every run, e.g. MH_TRAVERSAL=lane)
set -o pipefail
for v in "$@"; do
  lib=$v; [ "$v" = base ] && lib=""
  MH_LIB=$lib timeout -k 10 200 python tools/bench_volpath.py --no-cpu --steps 3 > gpurun_out/vab.log 2>&1 || { cat gpurun_out/vab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/vab.log').read().strip().split('\n')[-1]);print(sys.argv[1], d['value'], d['ms_per_render'], d['kernel_ms'])" "$v"
done
