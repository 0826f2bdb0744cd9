# GPU box: full GPU test suite, the profiled bench (tools/gpu_profile.sh) and the C2/C3 lines.
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 900 python -m pytest $R/tests -m gpu -x -q > $R/gpurun_out/$TAG/tests.log 2>&1; rc=$?; tail -2 $R/gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_profile.sh $TAG/prof > $R/gpurun_out/$TAG/profile.log 2>&1 || { tail -5 $R/gpurun_out/$TAG/profile.log; exit 1; }
cd $R && bash tools/gpu_configs.sh $TAG/configs > /dev/null && echo configs-done
