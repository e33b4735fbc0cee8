set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "volpath or config4 or invalid or furnace or absorber or sun or medium" > gpurun_out/vol_tests.log 2>&1 || { tail -30 gpurun_out/vol_tests.log; exit 1; }
tail -1 gpurun_out/vol_tests.log
timeout -k 10 200 python tools/bench_volpath.py --no-cpu > gpurun_out/vol.log 2>&1 || exit 1
tail -1 gpurun_out/vol.log
bash tools/profile_cmd.sh gpurun_out/vol_pc2 tools/bench_volpath.py --no-cpu --steps 1 > gpurun_out/vol_pc2.txt 2>&1 || exit 1
grep vol_sched gpurun_out/vol_pc2.txt
