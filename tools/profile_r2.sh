#!/bin/bash
# Round-2 profile of one bench step (run on the GPU box via gpurun):
#   trace        rocprofv3 --kernel-trace --stats (durations)
#   sq           SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES / SQ_WAIT_ANY /
#                SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY + GRBM_GUI_ACTIVE (clock)
#   fetch, write FETCH_SIZE, WRITE_SIZE (separate passes)
#   calib_*      the same FETCH / WRITE passes over tools/calib_fetch (known bytes)
# then tools/make_pmc.py -> <outdir>/pmc.json.  usage: tools/profile_r2.sh <outdir> [bench args]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/prof_r2}; shift
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --steps 2 --warmup 1 $*"
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$ROOT/bench.py" $ARGS >> "$OUT/log.txt" 2>&1; }
crun() { timeout -k 10 120 rocprofv3 "$@" --output-format csv -d "$OUT" -- "$ROOT/tools/calib_fetch" >> "$OUT/log.txt" 2>&1; }
run --kernel-trace --stats -o trace || exit 1
run --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -o sq || exit 1
run --kernel-trace --pmc FETCH_SIZE -o fetch || exit 1
run --kernel-trace --pmc WRITE_SIZE -o write || exit 1
crun --kernel-trace --pmc FETCH_SIZE -o calib_fetch || exit 1
crun --kernel-trace --pmc WRITE_SIZE -o calib_write || exit 1
python3 "$ROOT/tools/make_pmc.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
