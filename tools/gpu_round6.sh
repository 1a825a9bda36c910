# Round 6's GPU calls, by step (profiles/INDEX.md names the files each made):
#   bash tools/gpu_round6.sh a   the group allocator and the per-communicator copy streams: their GPU tests (Python and
#                                C++); then the placement A/B on bench.py's own allocation orders (pair / scan / tree x
#                                plain / rotating / group, pair also same_slot), interleaved 3x in one process under a
#                                rocprofv3 kernel trace (tools/placement_ab.py, tools/placement_ab_trace.py)
#                                then the N > 1 shard kernel on its receive layout, packed vs 4 KiB-skewed shards
#                                (tools/shard_layout_ab.py)
#   bash tools/gpu_round6.sh b   the placement A/B on another box (TAG=r06b)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
TAG=${TAG:-r06a}
case "$1" in
a)
    timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_parity.py tests/test_gpu_comm.py tests/test_gpu_timeout.py -k "alloc or allreduce_host or time" \
        > gpurun_out/${TAG}_tests.log 2>&1 &&
    timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
        tests/test_cpp_communicator.py -m gpu >> gpurun_out/${TAG}_tests.log 2>&1 &&
    bash tools/gpu_round6.sh ab &&
    bash tools/gpu_round6.sh shard
    ;;
shard)
    timeout -k 10 300 python -u tools/shard_layout_ab.py --reps 3 > gpurun_out/${TAG}_shard_layout.jsonl \
        2> gpurun_out/${TAG}_shard_layout.err
    ;;
b)
    bash tools/gpu_round6.sh ab
    ;;
ab)
    cd /tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 3 > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl
    ;;
*)
    echo "unknown step $1" >&2
    exit 2
    ;;
esac
