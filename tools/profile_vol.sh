#!/bin/bash
# Config-4 profile (run on the GPU box via gpurun): tools/bench_volpath.py
# (256^2 @ 64 spp, 256^3 fBm medium) with volpath (k_vol_sched<VolMachine>) or
# prbvolpath (k_vol_sched<PvMachine> forward + k_prbvol_backward), passes:
#   trace          rocprofv3 --kernel-trace --stats (durations)
#   sq             SQ wave-cycle split + VALU issue + GRBM_GUI_ACTIVE (clock)
#   fetch, write   FETCH_SIZE, WRITE_SIZE (separate passes)
#   tcc            TCC_HIT_sum / TCC_MISS_sum (L2 hit rate)
#   calib_*        FETCH / WRITE over tools/calib_fetch (known bytes)
# then tools/make_pmc.py -> <outdir>/pmc.json.  usage: tools/profile_vol.sh <outdir> [volpath|prbvolpath]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/prof_vol}; INTEG=${2:-volpath}
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --steps 1 --integrator $INTEG"
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$ROOT/tools/bench_volpath.py" $ARGS >> "$OUT/log.txt" 2>&1; }
crun() { timeout -k 10 120 rocprofv3 "$@" --output-format csv -d "$OUT" -- "$ROOT/tools/calib_fetch" >> "$OUT/log.txt" 2>&1; }
timeout -k 10 300 python3 "$ROOT/tools/bench_volpath.py" --no-cpu --steps 3 --integrator $INTEG > "$OUT/bench.txt" 2>> "$OUT/log.txt" || exit 1
run --kernel-trace --stats -o trace || exit 1
run --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -o sq || exit 1
run --kernel-trace --pmc FETCH_SIZE -o fetch || exit 1
run --kernel-trace --pmc WRITE_SIZE -o write || exit 1
run --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -o tcc || exit 1
crun --kernel-trace --pmc FETCH_SIZE -o calib_fetch || exit 1
crun --kernel-trace --pmc WRITE_SIZE -o calib_write || exit 1
python3 "$ROOT/tools/make_pmc.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
