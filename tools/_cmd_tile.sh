# tiled film splat: GPU suite + bench A/B vs the row splat (same box) + rocprof splat times
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_tile.log 2>&1 || exit 1
for i in 1 2; do
  for v in tile notile; do
    if [ $v = tile ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/tile_${v}$i.json 2>/dev/null || exit 1
  done
done
unset MH_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_tile -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_tile.log 2>&1 || exit 1
