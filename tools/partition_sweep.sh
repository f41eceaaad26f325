# N-way shard partition sweep (GPU box): per-rank kernel ms of the C4 shards rendered in turn
# for several (chunk, tail, tail chunk) settings, interleaved over $REPS repetitions.
#   bash tools/partition_sweep.sh "16:0:0 32:256:4 ..."   (0 = the rule)
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
for r in $(seq 1 ${REPS:-2}); do
  for p in $1; do
    IFS=: read k t kt <<< "$p"
    timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds ${WORLDS:-8} --chunk $k \
      --tail $t --tail-chunk $kt > $OUT/psweep.json 2> $OUT/psweep.err || { tail $OUT/psweep.err; exit 1; }
    python - $OUT/psweep.json $p <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
for key in sorted(x for x in r if x.startswith("world")):
    w = r[key]
    print(f"{sys.argv[2]:>10} {key}: K {w['chunk']} tail {w['tail']} max {w['max_ms']:.2f} "
          f"mean {w['sum_ms'] / len(w['per_rank_ms']):.2f} full {r['full_ms']:.2f}", flush=True)
PY
  done
done
