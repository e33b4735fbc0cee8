# round-4 HEAD: smoke, full GPU suite, bench lines (configs 2 and 4)
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4d.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py > gpurun_out/bench_r4d_$i.json 2> gpurun_out/bench_r4d_$i.err || exit 1; done
timeout -k 10 200 python bench.py --config 4 --no-cpu > gpurun_out/bench_c4_r4d.json 2>/dev/null || exit 1
