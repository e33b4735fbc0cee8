#!/bin/bash
# A/B timing of library variants on the bench step (GPU box).
# usage: tools/ab_fwd.sh [--full] name...   (name "cur" = the in-tree library,
# otherwise gpurun_exp/lib_<name>.so from tools/build_variant.sh)
MODE=--fwd-only
if [ "$1" = "--full" ]; then MODE=""; shift; fi
for v in "$@"; do
  if [ "$v" = cur ]; then L=""; else L=gpurun_exp/lib_$v.so; fi
  echo "$v $(MH_LIB=$L timeout -k 10 120 python bench.py --no-cpu $MODE --steps 3 --warmup 1 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_us": [0-9.]*' | tr '\n' ' ')"
done
