set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_phases.sh > gpurun_out/phases.txt 2>&1 || { cat gpurun_out/phases.txt; exit 1; }
cat gpurun_out/phases.txt
for c in c2 c3; do timeout -k 10 120 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2>gpurun_out/bench_$c.err || exit 1; done
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2>gpurun_out/bench_c5.err || exit 1
cat gpurun_out/bench_c*.json | cut -c1-300
