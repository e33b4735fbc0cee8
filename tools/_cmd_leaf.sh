# BVH leaf size x SAH C_t sweep for the stream engine (1M / 4M-triangle meshes)
set -o pipefail
for L in 4 6 8 12; do for C in 1 2 4; do
  MH_BVH_LEAF=$L MH_BVH_CT=$C timeout -k 10 200 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 > gpurun_out/leaf_${L}_${C}.txt 2>&1 || exit 1
done; done
