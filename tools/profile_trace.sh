#!/bin/bash
# Stream-engine traversal counters (run on the GPU box via gpurun): the
# unfused k_wf_trace / k_wf_shadow of tools/bench_mesh.py at one triangle
# count, under the environment given (A/B of node formats), passes:
#   trace  rocprofv3 --kernel-trace --stats
#   sq     wave cycles / waits / VALU + VMEM instruction counts and the VMEM
#          level (SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM = cycles a VMEM load is in flight)
#   ta     TA busy / stalled by the L1, TD busy, L1->L2 read latency, L1 accesses
#   tlb    UTCL1 translation hits / misses, L2 hit / miss
# then tools/trace_pmc.py <outdir>.  usage: tools/profile_trace.sh <outdir> <tris> [VAR=value ...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/prof_trace}; TRIS=${2:-1000000}; shift 2
for kv in "$@"; do export "$kv"; done
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="--tris $TRIS --steps 1 --warmup 0"
run() { timeout -k 10 240 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$ROOT/tools/bench_mesh.py" $ARGS >> "$OUT/log.txt" 2>&1; }
timeout -k 10 300 python3 "$ROOT/tools/bench_mesh.py" --tris $TRIS --steps 3 > "$OUT/bench.txt" 2>> "$OUT/log.txt" || exit 1
run --kernel-trace --stats -o trace || exit 1
run --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -o sq || exit 1
run --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum -o ta || exit 1
run --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum -o tlb || exit 1
python3 "$ROOT/tools/trace_pmc.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
