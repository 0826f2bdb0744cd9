set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t4.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t4.log
bash tools/ab.sh ab4 1 ww4 ww5 ww6 ww7 -- --steps 3 --warmup 1
