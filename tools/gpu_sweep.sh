# usage: bash tools/gpu_sweep.sh <tag> [render_once args...]; one JSON line per variant
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
out=gpurun_out/sweep_$tag.jsonl
: > $out
run() {  # name, env, args
    local name=$1; shift
    local line
    line=$(timeout -k 10 180 env "$@" 2>/dev/null | tail -1) || { echo "FAILED $name" >> $out; return 1; }
    echo "{\"name\": \"$name\", \"r\": $line}" >> $out
}
