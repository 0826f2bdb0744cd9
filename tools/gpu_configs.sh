# Bench lines for BASELINE.json configs C4 (default), C2 and C3 on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-configs}; mkdir -p $O
timeout -k 10 400 python $R/bench.py > $O/c4.json 2> $O/c4.err && tail -1 $O/c4.json && \
timeout -k 10 400 python $R/bench.py --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 > $O/c2.json 2> $O/c2.err && tail -1 $O/c2.json && \
timeout -k 10 400 python $R/bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 > $O/c3.json 2> $O/c3.err && tail -1 $O/c3.json
