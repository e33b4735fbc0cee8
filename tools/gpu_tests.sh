# -m gpu suite (optionally a -k filter as $1), stop at the first failure
set -o pipefail
mkdir -p gpurun_out
K=${1:+-k "$1"}
eval timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread $K > gpurun_out/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/tests.log | head -40; tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
