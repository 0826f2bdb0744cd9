# Rehearse bench.py's N>1 path on a one-GPU box: ranks share GPU 0 over gloo.
# Compare frame_sha1 across the 1-, 2- and 3-rank lines: the frame must be identical.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-dist}; mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python $R/bench.py --width 1024 --height 1024 --spp 64 --no-cpu-baseline > $O/n1.json 2> $O/n1.err && tail -1 $O/n1.json && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  $R/bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --device 0 --width 1024 --height 1024 --spp 64 > $O/n2.json 2> $O/n2.err && tail -1 $O/n2.json && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29518 \
  $R/bench.py --gpus 3 --steps 2 --warmup 1 --dist-backend gloo --device 0 --width 1024 --height 1024 --spp 64 > $O/n3.json 2> $O/n3.err && tail -1 $O/n3.json
