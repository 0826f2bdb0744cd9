set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab11_tests.log 2>&1; tail -3 gpurun_out/ab11_tests.log
bash tools/ab.sh ab11 1 default q1 q4 q16 s2 w5 w7 default@32 -- --steps 3 --warmup 1
