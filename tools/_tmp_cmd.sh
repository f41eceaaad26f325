set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "flat or boxes or stress or cost_order" > gpurun_out/nf_test.log 2>&1 || { tail -30 gpurun_out/nf_test.log; exit 1; }
tail -1 gpurun_out/nf_test.log
timeout -k 10 300 python tools/ab.py default ab_objs/pre.hsaco --spp 1024 --rounds 3 --frames 2 > gpurun_out/c4nf.json &&
timeout -k 10 300 python tools/ab.py default ab_objs/pre.hsaco --scene stress4096 --width 3840 --height 2160 --spp 256 --depth 50 --rounds 3 --frames 2 > gpurun_out/c5nf.json
