set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab7_tests.log 2>&1 && tail -2 gpurun_out/ab7_tests.log && \
bash tools/ab.sh ab7 1 g1 default il5 il7 default@32 default@16 -- --steps 3 --warmup 1
