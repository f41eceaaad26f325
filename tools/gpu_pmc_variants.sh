# SQ counters of the tracer kernel per variant (final scene, 1080p 64 spp): VALU/SALU/SMEM/LDS
# instruction counts, busy and wait cycles. VARIANTS_PMC="2 3 4" by default.
set -o pipefail
mkdir -p gpurun_out/pmcv
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
cd /tmp
for v in ${VARIANTS_PMC:-2 3 4}; do
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $ROOT/gpurun_out/pmcv/v${v}_a -o run -- python3 $ROOT/tools/render_once.py --spp 64 --variant $v > $ROOT/gpurun_out/pmcv/v${v}_a.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $ROOT/gpurun_out/pmcv/v${v}_b -o run -- python3 $ROOT/tools/render_once.py --spp 64 --variant $v > $ROOT/gpurun_out/pmcv/v${v}_b.log 2>&1 || exit 1
done
cd $ROOT
VARIANTS_PMC="${VARIANTS_PMC:-2 3 4}" python3 - <<'PY'
import csv, collections, os
for v in os.environ["VARIANTS_PMC"].split():
    agg = collections.defaultdict(float)
    for part in "ab":
        for r in csv.DictReader(open(f"gpurun_out/pmcv/v{v}_{part}/run_counter_collection.csv")):
            if r["Kernel_Name"].startswith("vcrt_trace"):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    busy = agg["SQ_ACTIVE_INST_VALU"] / max(agg["SQ_BUSY_CYCLES"], 1)
    print("variant", v, "valu/busy %.2f" % busy, {k: "%.4g" % x for k, x in sorted(agg.items())})
PY
echo all_done
