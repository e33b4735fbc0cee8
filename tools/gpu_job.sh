#!/bin/bash
# The recurring GPU jobs, run on the box through gpurun from the repo root:
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/gpu_job.sh <job> [args]
# Every step has its own time limit and the steps stop at the first failure.
#
#   suite                         smoke() + the whole -m gpu suite
#   final <tag>                   bench.py (with its CPU leg) x2, configs 1 / 3 / 4 / 5,
#                                 and the PMC passes bench.py reads (tools/profile_r2.sh)
#   ab <runs> <bench args> -- <variant>...
#                                 same-box A/B of library variants: each variant is
#                                 `cur` (the in-tree library) or the name of a build
#                                 made here by `tools/build_variant.sh <name> <flags>`;
#                                 the flags of every variant are printed from
#                                 gpurun_exp/<name>.flags, so an A/B is reproducible
#                                 from the repo (the libraries themselves are not tracked)
#   rocprof <out> [bench args]    rocprofv3 --kernel-trace --stats of bench.py
#   vol [args]                    tools/bench_volpath.py (config 4) with the given args
#   mesh [args]                   tools/bench_mesh.py --tris 1000000,4000000 (large-mesh path)
#   gloo2                         bench.py --gpus 2 --backend gloo: the launcher starts 2 ranks on the one GPU
# Outputs go to gpurun_out/job_<job>_*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
job=$1; shift
case "$job" in
suite)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/job_suite_smoke.log 2>&1 || exit 1
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/job_suite.log 2>&1 || exit 1
    ;;
final)
    tag=${1:-final}
    for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/job_${tag}_c2_$i.json 2> gpurun_out/job_${tag}_c2_$i.err || exit 1; done
    for c in 1 3 4; do timeout -k 10 300 python bench.py --config $c > gpurun_out/job_${tag}_c$c.json 2> gpurun_out/job_${tag}_c$c.err || exit 1; done
    timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 > gpurun_out/job_${tag}_c5.json 2> gpurun_out/job_${tag}_c5.err || exit 1
    # the PMC passes and the kernel trace with one stream per call: the line's
    # rooflines come from its one-stream roofline pass (MH_WF_STREAMS=1), and a
    # two-stream launch's duration is shared with the other chunk's launches
    MH_WF_STREAMS=1 bash tools/profile_r2.sh gpurun_out/job_${tag}_prof > gpurun_out/job_${tag}_prof.log 2>&1 || exit 1
    ;;
ab)
    runs=$1; shift
    args=()
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
    shift
    for v in "$@"; do
        if [ "$v" = cur ]; then echo "variant cur: in-tree library"; else echo "variant $v: $(cat gpurun_exp/$v.flags 2>/dev/null)"; fi
    done > gpurun_out/job_ab_variants.txt
    for i in $(seq 1 "$runs"); do
        for v in "$@"; do
            if [ "$v" = cur ]; then unset MH_LIB; else export MH_LIB=gpurun_exp/lib_$v.so; fi
            timeout -k 10 200 python bench.py "${args[@]}" --no-cpu > gpurun_out/job_ab_${v}_$i.json 2>/dev/null || exit 1
        done
    done
    unset MH_LIB
    python3 - <<'EOF' >> gpurun_out/job_ab_variants.txt
import glob, json, re, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/job_ab_*_*.json")):
    m = re.match(r"gpurun_out/job_ab_(.+)_(\d+)\.json", f)
    try:
        r[m.group(1)].append(json.load(open(f))["value"])
    except Exception:
        pass
for k, v in r.items():
    print(k, v)
EOF
    ;;
rocprof)
    out=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$out" -o trace -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/$out.log" 2>&1 || exit 1
    ;;
vol)
    timeout -k 10 300 python tools/bench_volpath.py --no-cpu "$@" > gpurun_out/job_vol.json 2> gpurun_out/job_vol.err || exit 1
    ;;
gloo2)
    timeout -k 10 400 python bench.py --gpus 2 --backend gloo --no-cpu --steps 3 --warmup 1 > gpurun_out/job_gloo2.json 2> gpurun_out/job_gloo2.err || exit 1
    ;;
mesh)
    timeout -k 10 300 python tools/bench_mesh.py --tris 1000000,4000000 --steps 3 "$@" > gpurun_out/job_mesh.txt 2>&1 || exit 1
    ;;
*)
    echo "unknown job: $job" >&2
    exit 2
    ;;
esac
