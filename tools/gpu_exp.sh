set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export VCRT_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --spp 64 --chunk 16 --validate > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 3 --steps 1 --warmup 1 --spp 32 --chunk 16 --validate > gpurun_out/bench_n3.json 2> gpurun_out/bench_n3.err || exit 1
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --spp 64 --chunk 16 --validate --no-cpu-baseline > gpurun_out/bench_n1v.json 2> gpurun_out/bench_n1v.err || exit 1
echo all_done
