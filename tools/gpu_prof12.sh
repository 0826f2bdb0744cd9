set -o pipefail
ZRT_LIB=build/variants/prof/libzrt.so timeout -k 10 300 python tools/prof_sections.py > gpurun_out/sections12.txt 2>&1 && cat gpurun_out/sections12.txt && \
bash tools/gpu_sq.sh sq12
