set -o pipefail
bash tools/ab.sh ab6 1 head g1 g4 g16 g4r8 -- --steps 3 --warmup 1
