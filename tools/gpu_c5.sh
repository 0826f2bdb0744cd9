# GPU tests (incl. scene 6 parity) + the C5-substitute bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-c5}; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/tests.log 2>&1; tail -3 $O/tests.log
timeout -k 10 900 python $R/bench.py --scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 > $O/c5.json 2> $O/c5.err && tail -1 $O/c5.json
