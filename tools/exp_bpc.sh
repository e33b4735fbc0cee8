#!/bin/bash
# bench step time vs wavefront workgroups per CU (MH_WF_BPC); GPU box.
# usage: tools/exp_bpc.sh [--full] bpc...
MODE=--fwd-only
if [ "$1" = "--full" ]; then MODE=""; shift; fi
for b in "$@"; do
  echo "bpc=$b $(MH_WF_BPC=$b timeout -k 10 120 python bench.py --no-cpu $MODE --steps 3 --warmup 1 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_us": [0-9.]*' | tr '\n' ' ')"
done
