set -o pipefail
bash tools/ab.sh ab9 1 default default@32 default@16 default@8 default@4 default@1 r2 -- --steps 3 --warmup 1
