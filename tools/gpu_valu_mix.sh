# VALU instruction mix and LDS conflicts of one C4 frame (three --pmc passes of 8 SQ counters).
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
P=$ROOT/gpurun_out/mix
rm -rf $P && mkdir -p $P
RO=${RO:-"--spp 256"}
cd /tmp
i=0
for pass in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
            "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $P/p$i -o run -- python3 $ROOT/tools/render_once.py $RO > $P/p$i.log 2>&1 || { tail -5 $P/p$i.log; exit 1; }
done
python3 - <<PY
import csv, collections
agg = collections.defaultdict(float); n = collections.Counter()
for i in (1, 2, 3):
    for r in csv.DictReader(open("$P/p%d/run_counter_collection.csv" % i)):
        if not r["Kernel_Name"].startswith("vcrt_trace"): continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
v = agg["SQ_INSTS_VALU"] / n["SQ_INSTS_VALU"]
for k in sorted(agg):
    x = agg[k] / n[k]
    print("%-28s %14.4g  %5.1f%% of VALU" % (k, x, 100 * x / v))
PY
