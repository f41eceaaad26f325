set -o pipefail
timeout -k 10 300 python tools/_tmp_ab_boxes.py 2000 && timeout -k 10 300 python tools/_tmp_ab_boxes.py 1000
