set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do for v in 8 12 0 63; do
  VCRT_ACCUM_RING=$v timeout -k 10 120 python tools/ab.py default --rounds 1 --spp 1024 --frames 2 > gpurun_out/abr.json 2>&1 || { cat gpurun_out/abr.json; exit 1; }
  echo "ring=$v $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abr.json | head -1) $(grep -o '"ring_entries": [0-9]*' gpurun_out/abr.json | head -1) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abr.json | head -1)"
done; done
