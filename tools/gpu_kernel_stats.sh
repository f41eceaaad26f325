# rocprofv3 --kernel-trace --stats of the bench command for configs c3, c2, c5 (c4: gpu_profile.sh);
# summaries to gpurun_out/kstats/<cfg>/ (copy the *_kernel_stats.csv into profiles/).
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
P=$ROOT/gpurun_out/kstats
rm -rf $P && mkdir -p $P
cd /tmp
for cfg in c3 c2 c5; do
  case $cfg in c5) ST="--steps 2 --warmup 1";; c2) ST="--steps 50 --warmup 5";; *) ST="--steps 10 --warmup 3";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$cfg -o bench -- python3 $ROOT/bench.py --config $cfg $ST --no-cpu-baseline > $P/$cfg.json 2> $P/$cfg.err || exit 1
  echo "$cfg done"
done
