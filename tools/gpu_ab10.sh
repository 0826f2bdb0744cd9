set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab10_tests.log 2>&1; tail -3 gpurun_out/ab10_tests.log
bash tools/ab.sh ab10 1 default default@16 s1 s2 s4 s8 s64 u4s8 w5 s4w5 -- --steps 3 --warmup 1
