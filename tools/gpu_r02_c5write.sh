set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r02c5w; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "c5 or loops or stack" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --scene 6 --width 4096 --height 4096 --spp 4096 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); r=d['roofline']; print('C5', d['value'], r['bound'], r['frac'], r.get('write_budget'))"
