# GPU box: WRITE_SIZE of the render kernel for the shipped library and A/B
# variants (tools/variants.sh builds them), one rocprofv3 --pmc pass each.
# usage: bash tools/gpu_pmc_write_ab.sh <tag> <variant>...   ("default" = zraytrace_amd/libzrt.so)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  if [ "$v" == "default" ]; then L=$R/zraytrace_amd/libzrt.so; else L=$R/build/variants/$v/libzrt.so; fi
  ZRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { echo "variant $v failed"; exit 1; }
done
echo pmcw-done
