set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 120 ./vulkancomputeraytracing_amd/bin/vcrt_render --width 1920 --height 1080 --spp 64 --depth 10 --frames 2 --out gpurun_out/final_1080p_64spp.ppm > gpurun_out/cli.log 2>&1 || exit 1
timeout -k 10 120 ./vulkancomputeraytracing_amd/bin/vcrt_render --width 800 --height 450 --spp 64 --depth 8 --scene three --out gpurun_out/three_800x450_64spp.ppm >> gpurun_out/cli.log 2>&1 || exit 1
echo all_done
