set -o pipefail
for c in 64 32 16; do echo "== chunk $c"; ZRT_CHUNK=$c timeout -k 10 300 python tools/tail_probe.py 8 2 2048 2048 1024 20 short || exit 1; done
bash tools/ab.sh ab22 1 default default@32 default@16 -- --steps 3 --warmup 1
