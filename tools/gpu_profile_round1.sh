set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo pytest_exit=$? >> gpurun_out/pytest_gpu.log
for v in 1 2; do for b in 0 2 4; do
  timeout -k 10 120 python tools/render_once.py --spp 64 --variant $v --blocks-per-cu $b --frames 2 > gpurun_out/sweep_v${v}_b${b}.json 2>&1 || exit 1
done; done
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_kt -o run -- python $GRAFT_REPO_ROOT/tools/render_once.py --spp 256 --frames 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_kt.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_pmc1 -o run -- python tools/render_once.py --spp 64 > gpurun_out/prof_pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/prof_pmc2 -o run -- python tools/render_once.py --spp 64 > gpurun_out/prof_pmc2.log 2>&1 || exit 1
echo all_done
