set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/ab20_tests.log 2>&1; tail -3 gpurun_out/ab20_tests.log
bash tools/ab.sh ab20 2 head default -- --steps 3 --warmup 1 && \
timeout -k 10 300 python tools/tail_probe.py 8 && timeout -k 10 300 python tools/tail_probe.py 2 3 1024 1024 256 20
