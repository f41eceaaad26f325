# Round profiles (run on the GPU box from the repo root; collect with
#   python tools/collect_profile.py <tag>):
#   bench lines of the BASELINE configs c4 (headline), c3, c2, c5;
#   rocprofv3 --kernel-trace --stats of the c4 bench command itself;
#   PMC passes (one counter block per run) of one c4 frame (tools/render_once.py), and of one
#   c2 and one c5 frame (SQ instruction mix, HBM bytes).
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
P=$ROOT/gpurun_out/prof
rm -rf $P && mkdir -p $P
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $P/bench_c4.json 2> $P/bench_c4.err || exit 1
timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $P/bench_c3.json 2> $P/bench_c3.err || exit 1
timeout -k 10 200 python bench.py --config c2 --steps 50 --warmup 5 > $P/bench_c2.json 2> $P/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 > $P/bench_c5.json 2> $P/bench_c5.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o bench -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $P/kt_bench.json 2> $P/kt_bench.err || exit 1
for cfg in c4 c2 c5; do
  case $cfg in
    c4) RO="--spp 1024";;
    c2) RO="--scene three --width 800 --height 450 --spp 64 --depth 8";;
    c5) RO="--scene stress4096 --width 3840 --height 2160 --spp 4096 --depth 50";;
  esac
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/${cfg}_fetch -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${cfg}_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/${cfg}_write -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${cfg}_write.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/${cfg}_sq1 -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${cfg}_sq1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F32 --output-format csv -d $P/${cfg}_sq2 -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${cfg}_sq2.log 2>&1 || exit 1
done
echo all_done
