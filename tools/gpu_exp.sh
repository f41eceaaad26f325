set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; exit 1; }
timeout -k 10 300 python tools/shard_sweep.py --spp 1024 > gpurun_out/shard_sweep.json 2> gpurun_out/shard_sweep.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo all_done
