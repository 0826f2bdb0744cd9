# GPU box: interleaved A/B of kernel variants (tools/variants.sh builds them).
# usage (via gpurun): bash tools/gpu_ab.sh <tag> <rounds> <variant>[@chunk]... [-- bench args]
# e.g.  bash tools/gpu_ab.sh ab21 2 head default -- --steps 3 --warmup 1
set -o pipefail
bash tools/ab.sh "$@"
