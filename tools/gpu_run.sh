# The one GPU driver (run on the GPU box from the repo root, e.g.
#   gpurun -- 'bash tools/gpu_run.sh test ab profile'):
# every mode below runs in order; a failing step ends the call (nothing more touches the GPU).
#
#   test        pytest -m gpu (one process, per-test timeout) and smoke()
#   bench       bench.py lines of the BASELINE configs in $CFGS (default c4 c3 c2 c5)
#   ab          A/B timing, interleaved single-process renders (tools/ab.py): the current tree
#               against the tree in $PREV (an earlier commit built by tools/mkab_tree.sh; any ABI)
#               and the code objects / env settings in $OBJS (tools/ab.py syntax: OBJ@VAR=V,...),
#               on $AB_CFGS (default c4; also c2, c3, stress) for $ROUNDS rounds; digests must agree
#   sweep       the N-way shards of C4 rendered one after another (tools/shard_sweep.py), max and
#               per-rank kernel ms for N in $WORLDS (default 2,4,8), $SWEEP_REPS times
#   profile     the round's profile set for tools/collect_profile.py $TAG: bench lines (c4 c3 c2
#               c5), rocprofv3 --kernel-trace --stats of each bench command, and PMC passes (one
#               counter block per run: FETCH_SIZE, WRITE_SIZE, two SQ sets) of one frame of each
#   pmcab       instruction counters of one frame ($PMC_CFG, default c4) for the prev tree ($PREV),
#               the current tree and the code objects in $OBJS: two PMC passes each, summarised by
#               tools/pmc_ab_summary.py (VALU per wave-segment, issue, lane utilisation)
#   trafficab   FETCH_SIZE / WRITE_SIZE (KB units) of one frame of $PMC_CFG, $PREV and current tree
#   phases      stats build (VCRT_DEBUG_STATS=1): s_memtime per phase of the flat scan ($RO args)
#   wavetimes   diagnostics build $WT_OBJ (VCRT_DEBUG_STATS=2): wave lifetimes ($WT_ARGS)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out

cfg_args() {  # tools/ab.py / render_once.py arguments of a config
  case $1 in
    c2) echo "--scene three --width 800 --height 450 --spp 64 --depth 8";;
    c3) echo "--spp 256";;
    c4) echo "--spp 1024";;
    c5) echo "--scene stress4096 --width 3840 --height 2160 --spp 4096 --depth 50";;
    stress) echo "--scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50";;
  esac
}

bench_steps() {
  case $1 in c5) echo "--steps 2 --warmup 1";; c2) echo "--steps 50 --warmup 5";;
             *) echo "--steps 10 --warmup 3";; esac
}

mode_test() {
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; return 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { cat $OUT/smoke.log; return 1; }
  tail -1 $OUT/smoke.log
}

mode_bench() {
  for c in ${CFGS:-c4 c3 c2 c5}; do
    timeout -k 10 300 python bench.py --config $c $(bench_steps $c) > $OUT/bench_$c.json \
      2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; return 1; }
    python -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
}

ab_run() {  # tag, command...
  local tag=$1; shift
  timeout -k 10 200 "$@" > $OUT/abt.json 2>&1 || { cat $OUT/abt.json; return 1; }
  echo "$tag $(grep -o '"msamples_per_s": [0-9.]*' $OUT/abt.json | head -1) $(grep -o '"kernel_ms": [0-9.]*' $OUT/abt.json | head -1) $(grep -o '"sha": "[0-9a-f]*"' $OUT/abt.json | head -1)"
}

mode_ab() {
  for i in $(seq 1 ${ROUNDS:-2}); do
    for c in ${AB_CFGS:-c4}; do
      local a="$(cfg_args $c) --frames ${AB_FRAMES:-2}"
      [ $c = c2 ] && a="$(cfg_args $c) --frames 20"
      if [ -n "$PREV" ]; then
        ab_run "prev $c" env VCRT_PKG_ROOT=$PREV python tools/ab.py default --rounds 1 $a || return 1
      fi
      ab_run "new $c" python tools/ab.py default --rounds 1 $a || return 1
      for o in $OBJS; do ab_run "$o $c" python tools/ab.py $o --rounds 1 $a || return 1; done
    done
  done
  echo ab_done
}

sweep_one() {  # tag, env prefix (or "none"), shard_sweep arguments...
  local tag=$1 env=$2
  shift 2
  ( [ "$env" != none ] && export $env
    timeout -k 10 300 python tools/shard_sweep.py --spp 1024 --worlds ${WORLDS:-2,4,8} "$@" \
      > $OUT/sweep_$tag.json 2> $OUT/sweep_$tag.err ) || { tail -20 $OUT/sweep_$tag.err; return 1; }
  python - "$OUT/sweep_$tag.json" "$tag" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
for key in sorted(x for x in r if x.startswith("world")):
    w = r[key]
    print(f"{sys.argv[2]} full {r['full_ms']:.2f} ms {key}: max {w['max_ms']:.2f} "
          f"sum {w['sum_ms']:.1f} estimate {w['ideal_efficiency']:.3f}")
PY
}

mode_sweep() {  # $PREV: also the prev tree; $SWEEP_ENVS: env settings (A=1,B=2 ...); $SWEEP_OBJS
  for i in $(seq 1 ${SWEEP_REPS:-1}); do
    if [ -n "$PREV" ]; then sweep_one prev_$i VCRT_PKG_ROOT=$ROOT/$PREV || return 1; fi
    sweep_one new_$i none || return 1
    local j=0
    for e in $SWEEP_ENVS; do
      j=$((j+1)); sweep_one env${j}_$i "$(echo $e | tr , ' ')" || return 1
    done
    for o in $SWEEP_OBJS; do  # code objects of the current tree
      sweep_one $(basename $o .hsaco)_$i none --code-object $ROOT/$o || return 1
    done
  done
}

mode_profile() {
  local P=$OUT/prof
  rm -rf $P && mkdir -p $P
  for c in c4 c3 c2 c5; do
    timeout -k 10 300 python bench.py --config $c $(bench_steps $c) > $P/bench_$c.json \
      2> $P/bench_$c.err || { tail $P/bench_$c.err; return 1; }
  done
  for c in c4 c3 c2 c5; do
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt_$c \
      -o bench -- python3 $ROOT/bench.py --config $c $(bench_steps $c) --no-cpu-baseline \
      > $P/kt_$c.json 2> $P/kt_$c.err) || { tail $P/kt_$c.err; return 1; }
  done
  for c in c4 c3 c2 c5; do
    local RO="$(cfg_args $c) --frames 2"  # the second frame: steady state (collect_profile.py)
    (cd /tmp &&
     timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/${c}_fetch -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${c}_fetch.log 2>&1 &&
     timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/${c}_write -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${c}_write.log 2>&1 &&
     timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/${c}_sq1 -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${c}_sq1.log 2>&1 &&
     timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F32 --output-format csv -d $P/${c}_sq2 -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${c}_sq2.log 2>&1) \
      || { echo "pmc $c failed"; return 1; }
  done
  echo profile_done
}

mode_pmcab() {
  local P=$OUT/pmcab RO=$(cfg_args ${PMC_CFG:-c4})
  rm -rf $P && mkdir -p $P
  local S1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  local S2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
  pmc_one() {  # tag, env prefix / extra render_once args...
    local tag=$1 env=$2; shift 2
    for pass in 1 2; do
      local C=$S1; [ $pass = 2 ] && C=$S2
      (cd /tmp && export $env && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv \
        -d $P/${tag}_$pass -o run -- python3 $ROOT/tools/render_once.py $RO "$@" \
        > $P/${tag}_$pass.log 2>&1) || { tail -5 $P/${tag}_$pass.log; return 1; }
    done
  }
  if [ -n "$PREV" ]; then pmc_one prev VCRT_PKG_ROOT=$ROOT/$PREV || return 1; fi
  pmc_one new VCRT_OBJ=none || return 1
  local i=0
  for o in $OBJS; do  # a code object, or args:A,B (render_once arguments with the current one)
    i=$((i+1))
    case $o in
      args:*) pmc_one obj$i VCRT_OBJ=args $(echo ${o#args:} | tr , ' ') || return 1;;
      *) pmc_one obj$i VCRT_OBJ=$o --code-object $ROOT/$o || return 1;;
    esac
  done
  python tools/pmc_ab_summary.py $P
}

mode_trafficab() {  # FETCH_SIZE / WRITE_SIZE of one frame ($PMC_CFG) for $PREV and the current tree
  local P=$OUT/traffic RO=$(cfg_args ${PMC_CFG:-c3})
  rm -rf $P && mkdir -p $P
  for t in prev new; do
    [ $t = prev ] && [ -z "$PREV" ] && continue
    local env=VCRT_OBJ=none; [ $t = prev ] && env=VCRT_PKG_ROOT=$ROOT/$PREV
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export $env && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv \
        -d $P/${t}_$c -o run -- python3 $ROOT/tools/render_once.py $RO > $P/${t}_$c.log 2>&1) \
        || { tail -5 $P/${t}_$c.log; return 1; }
    done
  done
  python - $P <<'PY'
import collections, csv, os, sys
P = sys.argv[1]
for t in ("prev", "new"):
    out = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(P, f"{t}_{c}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg, n = collections.defaultdict(float), collections.Counter()
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            if k.startswith("vcrt_trace") and row["Counter_Name"] == c:
                agg[k] += float(row["Counter_Value"])
                n[k] += 1
        out[c] = {k: agg[k] / n[k] for k in agg}  # KB per dispatch
    if out:
        fe, wr = out.get("FETCH_SIZE", {}), out.get("WRITE_SIZE", {})
        for k in sorted(set(fe) | set(wr)):
            print(f"{t} {k}: FETCH_SIZE {fe.get(k, 0) / 1024:.1f} MB, WRITE_SIZE "
                  f"{wr.get(k, 0) / 1024:.1f} MB, traffic (2 FETCH + WRITE) "
                  f"{(2 * fe.get(k, 0) + wr.get(k, 0)) / 1024 ** 2:.3f} GB")
PY
}

mode_phases() {
  VCRT_DEBUG_STATS=1 timeout -k 10 200 python tools/render_once.py ${RO:---spp 64} \
    --variant ${PV:-5} > $OUT/phases.json || return 1
  python tools/phases_report.py $OUT/phases.json
}

mode_valuattr() {  # region counts (stats build) and the product's SQ_INSTS_VALU, same frames ($RO)
  local P=$OUT/valuattr RO=${RO:---spp 64 --frames 2}
  rm -rf $P && mkdir -p $P
  VCRT_DEBUG_STATS=1 timeout -k 10 200 python tools/render_once.py $RO > $P/stats.json || return 1
  timeout -k 10 200 python tools/render_once.py $RO > $P/product.json || return 1
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv \
     -d $P/pmc -o run -- python3 $ROOT/tools/render_once.py $RO > $P/pmc.log 2>&1) \
    || { tail -20 $P/pmc.log; return 1; }
  find $P/pmc -name '*counter_collection.csv' | head -1 | xargs -I{} cp {} $P/counters.csv
  python - $P/counters.csv <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "vcrt_trace" in r["Kernel_Name"]]
per = collections.defaultdict(dict)
for r in rows:
    per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for d in sorted(per):
    print("dispatch", d, per[d])
PY
}

mode_wavetimes() {
  VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ${WT_OBJ:-ab_objs/wt.hsaco} \
    ${WT_ARGS:---spp 1024 --worlds 8} || return 1
}

for m in "$@"; do
  echo "== $m"
  mode_$m || { echo "mode $m failed"; exit 1; }
done
echo all_done
