set -o pipefail
bash tools/ab.sh ab15 2 head noslp noslp7 noslp8 noslp5 -- --steps 3 --warmup 1
