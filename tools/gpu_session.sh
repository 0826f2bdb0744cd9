#!/bin/bash
# GPU box: one measurement session - the GPU test suite, the driver's default
# bench line (C4), then the steps named on the command line, in order:
#   pmc:<cfg>                 rocprofv3 --pmc passes of config <cfg> (tools/gpu_pmc.sh)
#   bench:<cfg>               one bench line of config <cfg>
#   multi:<cfg>:<devices>     bench.py's one-process path (zrt_multi_*) over a device
#                             list, e.g. multi:c4:0,0 (two ranks rehearsed on GPU 0)
#   rehearse:<c3|4k>[:<n,..>] the N-rank torch.distributed path on one GPU over gloo (rank
#                             counts, default 2,3; e.g. rehearse:4k:2,8)
#   ab:<cfg>:<rounds>:<v,..>  interleaved A/B of build variants (abvar/<v>, tools/variants.sh;
#                             "default" = the shipped library)
#   envab:<cfg>:<rounds>:<E1|E2..>  interleaved A/B of environment settings (tools/gpu_env_ab.sh)
#   smoke                     __graft_entry__.smoke()
#   adv                       the adversarial exactness tests alone, reported without stopping
# PYTEST_K: a -k expression for the main test run (e.g. "not near_miss")
# <cfg>: c2 | c3 | c3g (C3 with the grazing-triangle guard) | c4 | c5 | c5q (C5 at 1024 spp) | 4k
#        (BASELINE.json configs)
# usage: bash tools/gpu_session.sh <tag> [--no-tests] [--no-bench] [step...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cfg_args() {
  case $1 in
    c2) echo "--scene 1 --width 1000 --height 1000 --spp 1000 --depth 30" ;;
    c3) echo "--scene 3 --width 1024 --height 1024 --spp 256 --depth 20" ;;
    c3g) echo "--scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --guard" ;;
    c4) echo "" ;;
    c5) echo "--scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 1 --warmup 0" ;;
    c5q) echo "--scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1" ;;
    4k) echo "--scene 2 --width 4096 --height 4096 --spp 64 --depth 20" ;;
    *) echo "unknown config $1" >&2; exit 1 ;;
  esac
}
if [ "$1" == "--no-tests" ]; then shift; else
  (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1); rc=$?
  tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$1" == "--no-bench" ]; then shift; else
  (cd $R && timeout -k 10 600 python bench.py > $O/c4.json 2> $O/c4.err) || { echo "bench failed"; tail -5 $O/c4.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r.get('bound'), r.get('frac'), r.get('reason'))"
fi
for step in "$@"; do
  IFS=: read -r kind c a3 a4 <<< "$step"
  case $kind in
    pmc) bash $R/tools/gpu_pmc.sh $TAG/pmc_$c $(cfg_args $c) || exit 1 ;;
    bench) (cd $R && timeout -k 10 900 python bench.py $(cfg_args $c) --no-cpu-baseline > $O/$c.json 2> $O/$c.err) || { echo "bench $c failed"; tail -5 $O/$c.err; exit 1; }
           python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['frame_sha1'][:12], d['roofline'].get('bound'), d['roofline'].get('frac'))" ;;
    multi) f=$O/multi_${c}_${a3//,/_}.json
           (cd $R && timeout -k 10 900 python bench.py $(cfg_args $c) --devices $a3 > $f 2> ${f%.json}.err) || { echo "multi $c $a3 failed"; tail -5 ${f%.json}.err; exit 1; }
           python -c "import json; d=json.load(open('$f')); print('multi $c $a3', d['value'], d['ms_per_step'], d['frame_equal_to_n1'], d['per_rank_ms'])" ;;
    rehearse) bash $R/tools/gpu_rehearse_dist.sh $TAG/dist_$c $c "${a3//,/ }" || exit 1 ;;
    ab) bash $R/tools/ab.sh $TAG/ab_$c $a3 ${a4//,/ } -- --no-reference-check $(cfg_args $c) || exit 1 ;;
    envab) IFS='|' read -ra ENVS <<< "$a4"
           bash $R/tools/gpu_env_ab.sh $TAG/envab_$c $a3 "${ENVS[@]}" -- --no-reference-check $(cfg_args $c) || exit 1 ;;
    smoke) (cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1) || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
           tail -1 $O/smoke.txt ;;
    adv) (cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "near_miss or transformed or far_spheres" > $O/adv.log 2>&1); rc=$?
         tail -15 $O/adv.log; [ $rc -le 1 ] || exit $rc ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo session-done
