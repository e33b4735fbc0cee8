# run selected GPU tests: bash tools/gpu_quick.sh "<pytest -k expr>" [files...]
set -o pipefail
mkdir -p gpurun_out
K="$1"; shift
FILES="${@:-tests}"
timeout -k 10 500 python -u -m pytest $FILES -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" > gpurun_out/quick.log 2>&1 || { tail -50 gpurun_out/quick.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" gpurun_out/quick.log | tail -40; tail -2 gpurun_out/quick.log
