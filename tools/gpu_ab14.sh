set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab14_tests.log 2>&1; tail -3 gpurun_out/ab14_tests.log
bash tools/ab.sh ab14 1 head default pf0 pfw5 pfw4 -- --steps 3 --warmup 1
