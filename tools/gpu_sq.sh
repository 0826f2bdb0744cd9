set -o pipefail
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && O=$R/gpurun_out/${1:-sq}
mkdir -p $O
A="--width 1024 --height 1024 --spp 256 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $O/p1 -o run -- python $R/bench.py $A > $O/p1.json 2> $O/p1.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- python $R/bench.py $A > $O/p2.json 2> $O/p2.err
echo rc=$?
