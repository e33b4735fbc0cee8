# volpath vs prbvolpath primal on config 4: phase statistics (MH_EXP_VSCNT) + device-counted grid lookups (MH_EXP_LOOKUPS)
set -o pipefail
export MH_LIB=gpurun_exp/lib_vsdiag.so MH_VW_DEBUG=1
timeout -k 10 200 python tools/bench_volpath.py --no-cpu --steps 1 > gpurun_out/vsdiag_volpath.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu --steps 1 > gpurun_out/vsdiag_prbvolpath.txt 2>&1 || exit 1
unset MH_LIB MH_VW_DEBUG
timeout -k 10 200 python tools/bench_volpath.py --integrator prbvolpath --no-cpu > gpurun_out/pvp_rays.json 2>&1 || exit 1
