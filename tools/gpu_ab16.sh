set -o pipefail
bash tools/ab.sh ab16 2 head trk trk7 trk5 -- --steps 3 --warmup 1
