set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t3.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/t3.log
bash tools/ab.sh ab3 1 ww4 ww5 ww6 -- --steps 3 --warmup 1
bash tools/ab.sh ab3b 1 default -- --steps 3 --warmup 1 --traversal binary
