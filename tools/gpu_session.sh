#!/bin/bash
# GPU box: one measurement session - the GPU test suite, the driver's default
# bench line (C4), then optional extra steps named on the command line:
#   pmc:<cfg>   rocprofv3 --pmc passes of config <cfg> (tools/gpu_pmc.sh)
#   bench:<cfg> one bench line of config <cfg>
#   rehearse    the N-rank path on one GPU over gloo (tools/gpu_rehearse_dist.sh)
#   adv         the adversarial exactness tests alone, reported without stopping the session
# PYTEST_K: a -k expression for the main test run (e.g. "not near_miss")
# <cfg>: c2 | c3 | c4 | c5 (BASELINE.json configs)
# usage: bash tools/gpu_session.sh <tag> [--no-tests] [step...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cfg_args() {
  case $1 in
    c2) echo "--scene 1 --width 1000 --height 1000 --spp 1000 --depth 30" ;;
    c3) echo "--scene 3 --width 1024 --height 1024 --spp 256 --depth 20" ;;
    c4) echo "" ;;
    c5) echo "--scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 1 --warmup 0" ;;
  esac
}
if [ "$1" == "--no-tests" ]; then shift; else
  (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1); rc=$?
  tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
(cd $R && timeout -k 10 600 python bench.py > $O/c4.json 2> $O/c4.err) || { echo "bench failed"; tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r.get('bound'), r.get('frac'), r.get('reason'))"
for step in "$@"; do
  kind=${step%%:*}; c=${step#*:}
  case $kind in
    pmc) bash $R/tools/gpu_pmc.sh $TAG/pmc_$c $(cfg_args $c) || exit 1 ;;
    bench) (cd $R && timeout -k 10 900 python bench.py $(cfg_args $c) > $O/$c.json 2> $O/$c.err) || { echo "bench $c failed"; tail -5 $O/$c.err; exit 1; }
           python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['frame_sha1'][:12])" ;;
    rehearse) bash $R/tools/gpu_rehearse_dist.sh $TAG/dist || exit 1 ;;
    adv) (cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "near_miss or transformed or far_spheres" > $O/adv.log 2>&1); rc=$?
         tail -15 $O/adv.log; [ $rc -le 1 ] || exit $rc ;;
  esac
done
echo session-done
