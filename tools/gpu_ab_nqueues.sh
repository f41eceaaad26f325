# Work queues per device: 8 (one per XCD) against 16 and 32 (ab_objs/q*.hsaco,
# EXTRA=-DVCRT_QUEUES=N tools/mkab.sh qN) on C2, C3, C4 8-way shards and the stress scene.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
C2="--scene three --width 800 --height 450 --spp 64 --depth 8"
timeout -k 10 150 python tools/ab.py ab_objs/q8.hsaco ab_objs/q16.hsaco ab_objs/q32.hsaco --rounds 3 --frames 6 $C2 > gpurun_out/abn_c2.json 2>&1 || { cat gpurun_out/abn_c2.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/q8.hsaco ab_objs/q16.hsaco ab_objs/q32.hsaco --rounds 2 --spp 256 > gpurun_out/abn_c3.json 2>&1 || { cat gpurun_out/abn_c3.json; exit 1; }
timeout -k 10 250 python tools/ab.py ab_objs/q8.hsaco ab_objs/q16.hsaco ab_objs/q32.hsaco --rounds 2 --scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50 > gpurun_out/abn_c5.json 2>&1 || { cat gpurun_out/abn_c5.json; exit 1; }
for rep in 1 2; do
  for q in 8 16 32; do
    timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 --code-object ab_objs/q$q.hsaco > gpurun_out/abn_n8_q${q}_$rep.json 2>/dev/null || exit 1
    echo "q$q"; tail -1 gpurun_out/abn_n8_q${q}_$rep.json
  done
done
