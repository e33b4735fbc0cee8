# round-2 data collection: bench line (with CPU baseline), PMC profile of the bench step,
# per-config timings, config 4 / 5 / prbvolpath, kernel stats of the configs run
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash tools/profile_r2.sh gpurun_out/prof_r2 > gpurun_out/prof_r2.txt 2>&1 || { tail -30 gpurun_out/prof_r2.txt; tail -30 gpurun_out/prof_r2/log.txt; exit 1; }
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
timeout -k 10 300 python tools/bench_volpath.py > gpurun_out/vol.log 2>&1 || { tail -20 gpurun_out/vol.log; exit 1; }
timeout -k 10 300 python tools/bench_volpath.py --integrator prbvolpath > gpurun_out/pvp.log 2>&1 || { tail -20 gpurun_out/pvp.log; exit 1; }
timeout -k 10 400 python tools/bench_config5.py > gpurun_out/c5.log 2>&1 || { tail -20 gpurun_out/c5.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg_prof -o run --output-format csv -- python3 $R/tools/bench_configs.py > $R/gpurun_out/cfg_prof.log 2>&1 || { tail -20 $R/gpurun_out/cfg_prof.log; exit 1; }
cat $R/gpurun_out/configs.log $R/gpurun_out/vol.log $R/gpurun_out/pvp.log $R/gpurun_out/c5.log | grep -v amdgpu.ids
