# bench runtime knobs at HEAD: blocks per CU of the wavefront kernels, chunk size
set -o pipefail
run() { timeout -k 10 150 env "$@" python bench.py --steps 20 --warmup 5 --no-cpu 2>/dev/null | tail -1; }
for k in "MH_X=0" "MH_WF_BPC=16" "MH_WF_BPC=24" "MH_WF_BPC=45" "MH_WF_CHUNK=16777216" "MH_X=1"; do
  echo "$k $(run $k | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')" >> gpurun_out/sweep_bench.txt || exit 1
done
