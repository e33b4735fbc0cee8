# -m gpu suite on the in-tree library, then bench A/B: in-tree vs gpurun_exp/lib_$1.so
set -o pipefail
bash tools/gpu_tests.sh || exit 1
bash tools/ab_fwd.sh --full cur $1 cur $1
