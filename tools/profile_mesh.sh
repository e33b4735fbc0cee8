#!/bin/bash
# Large-mesh traversal profile (run on the GPU box via gpurun): the unfused
# stream engine (k_wf_trace / k_wf_shadow over the BVH4 of a PLY blob),
# tools/bench_mesh.py at one triangle count, passes:
#   trace          rocprofv3 --kernel-trace --stats (durations)
#   sq             SQ wave-cycle split + VALU issue + GRBM_GUI_ACTIVE (clock)
#   fetch, write   FETCH_SIZE, WRITE_SIZE (separate passes)
#   tcc            TCC_HIT_sum / TCC_MISS_sum (L2 hit rate)
#   calib_*        FETCH / WRITE over tools/calib_fetch (known bytes)
# then tools/make_pmc.py -> <outdir>/pmc.json.  usage: tools/profile_mesh.sh <outdir> <tris>
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/prof_mesh}; TRIS=${2:-1000000}
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="--tris $TRIS --steps 1 --warmup 0"
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$ROOT/tools/bench_mesh.py" $ARGS >> "$OUT/log.txt" 2>&1; }
crun() { timeout -k 10 120 rocprofv3 "$@" --output-format csv -d "$OUT" -- "$ROOT/tools/calib_fetch" >> "$OUT/log.txt" 2>&1; }
timeout -k 10 300 python3 "$ROOT/tools/bench_mesh.py" --tris $TRIS --steps 3 > "$OUT/bench.txt" 2>> "$OUT/log.txt" || exit 1
run --kernel-trace --stats -o trace || exit 1
run --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -o sq || exit 1
run --kernel-trace --pmc FETCH_SIZE -o fetch || exit 1
run --kernel-trace --pmc WRITE_SIZE -o write || exit 1
run --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -o tcc || exit 1
crun --kernel-trace --pmc FETCH_SIZE -o calib_fetch || exit 1
crun --kernel-trace --pmc WRITE_SIZE -o calib_write || exit 1
python3 "$ROOT/tools/make_pmc.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
