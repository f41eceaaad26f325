# Instruction counters of one frame, the ab_objs/prev tree against the current tree (and the
# code objects in $OBJS), RO = tools/render_once.py arguments (default: 1080p 256 spp).
# Output: gpurun_out/pmcab/<tag>_<pass>/ (rocprofv3 csv); summarise with tools/pmc_ab_summary.py.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
P=$ROOT/gpurun_out/pmcab
rm -rf $P && mkdir -p $P
RO=${RO:-"--spp 256"}
PASS1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PASS2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
cd /tmp
one() {  # tag, script, extra args
  local tag=$1 script=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $PASS1 --output-format csv -d $P/${tag}_1 -o run -- python3 $script $RO "$@" > $P/${tag}_1.log 2>&1 || { tail -5 $P/${tag}_1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $PASS2 --output-format csv -d $P/${tag}_2 -o run -- python3 $script $RO "$@" > $P/${tag}_2.log 2>&1 || { tail -5 $P/${tag}_2.log; exit 1; }
}
one prev $ROOT/ab_objs/prev/tools/render_once.py
one new $ROOT/tools/render_once.py
i=0
for o in $OBJS; do i=$((i+1)); one obj$i $ROOT/tools/render_once.py --code-object $ROOT/$o; done
echo pmc_done
