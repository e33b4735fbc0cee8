set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu --steps 2 > gpurun_out/pvp_base.log 2>&1 || exit 1
tail -1 gpurun_out/pvp_base.log
MH_LIB=gpurun_exp/lib_noatom.so timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu --steps 2 > gpurun_out/pvp_noatom.log 2>&1 || exit 1
tail -1 gpurun_out/pvp_noatom.log
