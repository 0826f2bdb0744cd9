set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r03c
(cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/r03c/tests.log 2>&1); rc=$?; tail -3 $R/gpurun_out/r03c/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh ab_sph 2 head=default nosph=nosph r02=r02 -- --steps 3 --warmup 1 || exit 1
bash tools/gpu_ab2.sh ab_pool_c3 2 lock=default pool=default:ZRT_POOL=1 wf=default:ZRT_WF=1 r02=r02 -- --steps 5 --warmup 1 --scene 3 --width 1024 --height 1024 --spp 256 || exit 1
bash tools/gpu_ab2.sh ab_pool_c5 1 wf=default pool=default:ZRT_POOL=1 r02=r02 -- --steps 2 --warmup 1 --scene 6 --width 4096 --height 4096 --spp 64 || exit 1
