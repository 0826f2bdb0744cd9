set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab17_tests.log 2>&1; tail -3 gpurun_out/ab17_tests.log
bash tools/ab.sh ab17 2 head default -- --steps 3 --warmup 1
