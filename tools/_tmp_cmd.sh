set -o pipefail
A="--scene three --width 800 --height 450 --spp 64 --depth 8 --frames 40 --rounds 1"
for i in 1 2 3 4 5; do
  for t in p9d p9c cur; do
    if [ $t = cur ]; then R=$PWD; else R=$PWD/ab_objs/$t; fi
    VCRT_PKG_ROOT=$R timeout -k 10 120 python tools/ab.py default $A > gpurun_out/c2ab.json || exit 1
    echo "$t $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c2ab.json | head -1) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/c2ab.json | head -1)"
  done
done
