set -o pipefail
timeout -k 10 600 python tools/tail_probe.py 8 2 2048 2048 4096 20
