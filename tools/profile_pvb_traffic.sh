#!/bin/bash
# prbvolpath backward traffic by source (run on the GPU box):
# config 4 (tools/bench_volpath.py --integrator prbvolpath) on the default
# library and on diagnostic builds that take one source out
#   nomain  MainLog entries kept at entry 0 (-DMH_EXP_PVB_MAIN_FIXED)
#   nonee   NeeLog entries kept at entry 0 (-DMH_EXP_PVB_NEE_FIXED)
#   noatom  no grid-gradient corner atomics (-DMH_EXP_NO_SIGMA_ATOMIC)
# (tools/build_variant.sh builds them into gpurun_exp/), a timing run and a
# FETCH_SIZE and a WRITE_SIZE pass each; tools/pvb_traffic.py summarises.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/pvb_traffic}
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
for v in base nomain nonee noatom; do
  if [ $v = base ]; then unset MH_LIB; else export MH_LIB=$ROOT/gpurun_exp/lib_pvb_$v.so; fi
  timeout -k 10 300 python3 "$ROOT/tools/bench_volpath.py" --no-cpu --steps 3 --integrator prbvolpath > "$OUT/bench_$v.txt" 2>> "$OUT/log.txt" || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT" -o ${v}_$c -- python3 "$ROOT/tools/bench_volpath.py" --no-cpu --steps 1 --integrator prbvolpath >> "$OUT/log.txt" 2>&1 || exit 1
  done
done
python3 "$ROOT/tools/pvb_traffic.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
