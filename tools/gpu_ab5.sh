set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t5.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t5.log
bash tools/ab.sh ab5 1 base p30 p70 s2 s8 w5 w7 -- --steps 3 --warmup 1
