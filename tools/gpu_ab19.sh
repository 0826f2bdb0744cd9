set -o pipefail
bash tools/ab.sh ab19 2 head sort3 -- --steps 3 --warmup 1
