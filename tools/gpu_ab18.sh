set -o pipefail
bash tools/ab.sh ab18 1 head xrng xsin xunit xinv xall -- --steps 3 --warmup 1
