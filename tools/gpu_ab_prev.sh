# A/B across ABI changes: the build in exp/prev (an earlier commit) against the code objects in
# exp/ab/ loaded by the current tree, alternating processes, final scene 1080p 256 spp.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2; do
  VCRT_PKG_ROOT=exp/prev timeout -k 10 120 python tools/ab.py default --rounds 1 ${ABARGS} > gpurun_out/abp_prev_$i.json 2>&1 || exit 1
  echo "prev $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abp_prev_$i.json) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abp_prev_$i.json)"
  for o in exp/ab/*.hsaco; do
    timeout -k 10 120 python tools/ab.py $o --rounds 1 ${ABARGS} > gpurun_out/abp_cur.json 2>&1 || exit 1
    echo "$o $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abp_cur.json) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abp_cur.json)"
  done
done
timeout -k 10 60 python tools/render_once.py --spp 16 > gpurun_out/ro.json 2>&1 && grep -o '"lds_bytes": [0-9]*\|"grid_blocks": [0-9]*' gpurun_out/ro.json
