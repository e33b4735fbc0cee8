# stream-engine occupancy A/B: 6 (default) / 7 / 8 waves per SIMD, 1M / 4M meshes, same box
set -o pipefail
for i in 1 2; do
  for v in def w7 w8; do
    if [ $v = def ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
    timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/w_${v}$i.txt 2>&1 || exit 1
  done
done
