# stream-engine stack / occupancy sweep on the large meshes (round 4)
set -o pipefail
for v in def w6; do for sc in 64 12 16 20; do
  if [ $v = def ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
  MH_STREAM_STACK=$sc timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/mesh_${v}_sc$sc.txt 2>&1 || exit 1
done; done
