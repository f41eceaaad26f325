# A/B of the current tree against the build in exp/prev (an earlier commit, any ABI): parity
# tests of the current tree, then alternating single-tree timing runs of tools/ab.py on the
# final scene (1080p 256 spp) and the stress scene (4K 32 spp depth 50). The digests must match.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
S="--scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50"
for i in 1 2; do
  VCRT_PKG_ROOT=exp/prev timeout -k 10 120 python tools/ab.py default --rounds 1 > gpurun_out/abd_prev_$i.json 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py default --rounds 1 > gpurun_out/abd_new_$i.json 2>&1 || exit 1
done
VCRT_PKG_ROOT=exp/prev timeout -k 10 120 python tools/ab.py default --rounds 1 $S > gpurun_out/abd_prev_s.json 2>&1 || exit 1
timeout -k 10 120 python tools/ab.py default --rounds 1 $S > gpurun_out/abd_new_s.json 2>&1 || exit 1
for f in gpurun_out/abd_*.json; do echo "$f $(grep -o '"msamples_per_s": [0-9.]*' $f) $(grep -o '"sha": "[0-9a-f]*"' $f)"; done
