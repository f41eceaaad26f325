# Each wave's first block of its queue without an atomic (ab_objs/sf.hsaco, -DVCRT_STATIC_FIRST)
# against the shipped fetch (ab_objs/cur.hsaco); ab.py checks that the bits are equal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
C2="--scene three --width 800 --height 450 --spp 64 --depth 8"
timeout -k 10 150 python tools/ab.py ab_objs/cur.hsaco ab_objs/sf.hsaco --rounds 3 --frames 6 $C2 > gpurun_out/absf_c2.json 2>&1 || { cat gpurun_out/absf_c2.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/cur.hsaco ab_objs/sf.hsaco --rounds 2 --spp 256 > gpurun_out/absf_c3.json 2>&1 || { cat gpurun_out/absf_c3.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/cur.hsaco ab_objs/sf.hsaco --rounds 2 --spp 1024 > gpurun_out/absf_c4.json 2>&1 || { cat gpurun_out/absf_c4.json; exit 1; }
for rep in 1 2; do
  for q in cur sf; do
    timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 --code-object ab_objs/$q.hsaco > gpurun_out/absf_n8_${q}_$rep.json 2>/dev/null || exit 1
    echo "$q"; tail -1 gpurun_out/absf_n8_${q}_$rep.json
  done
done
