# Rehearse bench.py's N>1 path on a one-GPU box: ranks share GPU 0 over gloo.
# usage: bash tools/gpu_rehearse_dist.sh <out tag> [c3|4k] ["rank counts", default "2 3"]
#   c3 (default): config C3 (scene 3, 1024x1024 @ 256 spp, depth 20)
#   4k: north_star's "tiled 4K" case - the bunny scene (C4's) at 4096x4096 @ 64 spp, depth 20
# Every line carries frame_sha1 and frame_equal_to_n1 against the committed
# one-GPU hash (profiles/frame_hashes.json) and per-rank kernel / gather milliseconds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-dist}; mkdir -p $O
export MASTER_ADDR=127.0.0.1
case ${2:-c3} in
  4k) A="--scene 2 --width 4096 --height 4096 --spp 64 --depth 20 --no-cpu-baseline --no-reference-check" ;;
  *)  A="--scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-cpu-baseline" ;;
esac
# (gloo prints its connection lines to stdout too: the bench line is the last '{' line)
show() { python -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print(d['n_gpus'], d['value'], d['frame_sha1'][:12], d['frame_equal_to_n1'], d['per_rank_ms'])"; }
timeout -k 10 300 python $R/bench.py $A > $O/n1.json 2> $O/n1.err && show $O/n1.json || exit 1
port=29517
for n in ${3:-2 3}; do  # rank counts (e.g. "2 3 8": the driver's N = 8 partition, all ranks on GPU 0)
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port \
    $R/bench.py --gpus $n --steps 2 --warmup 1 --dist-backend gloo --device 0 $A > $O/n$n.json 2> $O/n$n.err && show $O/n$n.json || exit 1
  port=$((port + 1))
done
