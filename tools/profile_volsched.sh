#!/bin/bash
# k_vol_sched roofline (config 4 volpath; run on the GPU box via gpurun):
#   lookups   bench.py --config 4 (its line carries the device-counted grid lookups)
#   profile   tools/profile_r2.sh --config 4 on the release build (durations, SQ, calibrated traffic)
# then tools/volsched_roofline.py.  usage: tools/profile_volsched.sh <outdir>
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/prof_vs}
mkdir -p "$OUT"
timeout -k 10 200 python3 "$ROOT/bench.py" --config 4 --steps 1 --warmup 0 --no-cpu \
    > "$OUT/lookups.json" 2> "$OUT/lookups.err" || exit 1
bash "$ROOT/tools/profile_r2.sh" "$OUT" --config 4 > "$OUT/profile.log" 2>&1 || exit 1
python3 "$ROOT/tools/volsched_roofline.py" "$OUT" | tee "$OUT/roofline.txt"
