set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t2.log
bash tools/ab.sh ab2 2 w5 w6 w7 w8 -- --steps 3 --warmup 1
