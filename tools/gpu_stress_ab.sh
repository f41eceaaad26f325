set -o pipefail
S="--scene stress4096 --width 3840 --height 2160 --spp 256 --depth 50 --frames 2"
for i in 1 2; do
  VCRT_PKG_ROOT=ab_objs/prev timeout -k 10 120 python tools/ab.py default --rounds 1 $S > gpurun_out/a1.json 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py default ab_objs/uninode.hsaco --rounds 1 $S > gpurun_out/a2.json 2>&1 || exit 1
  echo "prev $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/a1.json | head -1)"
  grep -o '"msamples_per_s": [0-9.]*\|"sha": "[0-9a-f]*"' gpurun_out/a2.json | paste - - 
done
