set -o pipefail
ZRT_LIB=build/variants/slanes/libzrt.so timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "not schedule and not c5" > gpurun_out/slanes_tests.log 2>&1; tail -3 gpurun_out/slanes_tests.log
bash tools/ab.sh ab21 2 head slanes -- --steps 3 --warmup 1
