# round-2 (session 4) check: full -m gpu suite, prbvolpath timing + kernel stats, bench marker trace (roctx)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python tools/bench_volpath.py --integrator prbvolpath --no-cpu > gpurun_out/pvp.log 2>&1 || { tail -20 gpurun_out/pvp.log; exit 1; }
tail -1 gpurun_out/pvp.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pvp_prof -o run --output-format csv -- python3 $R/tools/bench_volpath.py --integrator prbvolpath --no-cpu --steps 1 > $R/gpurun_out/pvp_prof.log 2>&1 || { tail -20 $R/gpurun_out/pvp_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $R/gpurun_out/mk_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 2 --warmup 1 > $R/gpurun_out/mk_prof.log 2>&1 || { tail -20 $R/gpurun_out/mk_prof.log; exit 1; }
find $R/gpurun_out/pvp_prof $R/gpurun_out/mk_prof -name "*.csv" | head -20
