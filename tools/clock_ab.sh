# Shader clock of the bounce kernels with synchronous vs asynchronous wrapper
# calls (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration), bench step, no CPU leg
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/clk
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  MH_ASYNC_CALLS=$m timeout -k 10 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $R/gpurun_out/clk/m$m -o run -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/clk/m$m.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for m in ("0", "1"):
    f = glob.glob(f"gpurun_out/clk/m{m}/run_counter_collection.csv")[0]
    acc = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE": continue
        k = r["Kernel_Name"]
        if "k_wf_bounce" not in k: continue
        key = k.split("(")[0].replace("void mh::", "")
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = acc[key]; a[0] += float(r["Counter_Value"]); a[1] += dur; a[2] += 1
    for k, (g, d, n) in sorted(acc.items()):
        print(f"async={m} {k:40s} calls {n:4d} avg_us {d / n / 1e3:8.1f} clock_GHz {g / 8 / d:.3f}")
PY
