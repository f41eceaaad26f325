# Round profiles: tests, bench, rocprofv3 kernel trace of the bench command, PMC passes at the
# bench config (HBM bytes, VALU busy). Collect with: python tools/collect_profile.py <tag>
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
RO="$ROOT/tools/render_once.py --spp 1024"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof/kt -o bench -- python3 $ROOT/bench.py --no-cpu-baseline > $ROOT/gpurun_out/prof/kt_bench.json 2> $ROOT/gpurun_out/prof/kt_bench.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/prof/pmc_fetch -o run -- python3 $RO > $ROOT/gpurun_out/prof/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/prof/pmc_write -o run -- python3 $RO > $ROOT/gpurun_out/prof/pmc_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $ROOT/gpurun_out/prof/pmc_sq1 -o run -- python3 $RO > $ROOT/gpurun_out/prof/pmc_sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F32 --output-format csv -d $ROOT/gpurun_out/prof/pmc_sq2 -o run -- python3 $RO > $ROOT/gpurun_out/prof/pmc_sq2.log 2>&1 || exit 1
echo all_done
