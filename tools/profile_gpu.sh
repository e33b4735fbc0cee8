#!/bin/bash
# rocprofv3 passes over one bench step (run on the GPU box via gpurun).
# usage: tools/profile_gpu.sh <outdir> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/prof}; shift
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --steps 1 --warmup 1 $*"
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$ROOT/bench.py" $ARGS >> "$OUT/log.txt" 2>&1; }
run --kernel-trace --stats -o trace || exit 1
run --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -o pmc_a || exit 1
run --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -o pmc_b || exit 1
run --kernel-trace --pmc FETCH_SIZE -o pmc_c || exit 1
run --kernel-trace --pmc WRITE_SIZE -o pmc_d || exit 1
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
