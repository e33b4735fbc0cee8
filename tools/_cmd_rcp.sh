# bound: k_vol_sched with approximate bbox reciprocals vs exact (config 4, same box)
set -o pipefail
for i in 1 2; do
  for v in def fastrcp; do
    if [ $v = def ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/rcp_${v}$i.json 2>/dev/null || exit 1
  done
done
