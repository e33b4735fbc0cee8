set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/b2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p2 -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/p2.log 2>&1 || exit 1
