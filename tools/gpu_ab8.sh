set -o pipefail
ZRT_LIB=build/variants/prof/libzrt.so timeout -k 10 300 python tools/prof_sections.py > gpurun_out/sections8.txt 2>&1 && cat gpurun_out/sections8.txt && \
bash tools/ab.sh ab8 1 default r1 r2 r8 -- --steps 3 --warmup 1 && \
bash tools/gpu_sq.sh sq8
