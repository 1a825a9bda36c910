# Round 6's GPU calls, by step (profiles/INDEX.md names the files each made):
#   bash tools/gpu_round6.sh a   the group allocator and the per-communicator copy streams: their GPU tests (Python and
#                                C++); then the placement A/B on bench.py's own allocation orders (pair / scan / tree x
#                                plain / rotating / group, pair also same_slot), interleaved 3x in one process under a
#                                rocprofv3 kernel trace (tools/placement_ab.py, tools/placement_ab_trace.py)
#                                then the N > 1 shard kernel on its receive layout, packed vs 4 KiB-skewed shards
#                                (tools/shard_layout_ab.py)
#   bash tools/gpu_round6.sh b   placement, round two (TAG=r06b): the allocator's placements beside explicit slot lists,
#                                mode order rotated per rep, under a kernel trace
#   bash tools/gpu_round6.sh c   placement, round three (TAG=r06c): per-set slot shifts (s:...@K), pair and scan
#   bash tools/gpu_round6.sh d   the skewed shard receive: its GPU suites, then the shard kernel in fmi_comm_allreduce
#                                with 8 LOCAL ranks, skew on / off (TAG=r06d)
#   bash tools/gpu_round6.sh f   carved groups: their GPU tests, placement round four (group vs rotating vs the same
#                                slots as separate allocations), the default line (TAG=r06f)
#   bash tools/gpu_round6.sh g   the pair's buckets: plain, carved group, per-set carve, one 8 GiB carve; then the
#                                shard kernel's output carved into the staging range: its tests and the layout A/B
#                                (TAG=r06g)
#   bash tools/gpu_round6.sh p   bench.py --force-dist at world 1 over RCCL, diagnostics and C5 at 1 GiB (TAG=r06p)
#   bash tools/gpu_round6.sh q   the N > 1 line at full size, 8 PROC ranks on one GPU (TAG=r06q)
#   bash tools/gpu_round6.sh r   the N > 1 line at N = 2 and 4, PROC ranks on one GPU (TAG=r06r)
#   bash tools/gpu_round6.sh s   soaks: the P-way and communicator random sweeps at fresh seeds
#   bash tools/gpu_round6.sh h   the device copy by placement (TAG=r06h)
#   bash tools/gpu_round6.sh t   the N > 1 line's GPU tests (TAG=r06t)
#   bash tools/gpu_round6.sh l   the LOCAL exchange ordered on the streams: its suites, then C5's co-resident block
#                                async / synchronised (TAG=r06l)
#   bash tools/gpu_round6.sh i   the fused kernels' launch knobs re-checked on carved groups (TAG=r06i)
#   bash tools/gpu_round6.sh cold  C2 as the first work of a fresh box, twice, then after a 60 s pause (TAG=r06k)
#   bash tools/gpu_round6.sh two the default line twice, separate processes (TAG=r06v)
#   bash tools/gpu_round6.sh z   the round-end sequence: GPU suite, smoke(), default line, C2 profile (TAG=r06z...)
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
    # placement, round two: the allocator's own placements beside explicit slot lists made by identical allocation
    # calls (s:...), the mode order rotated by one per rep (so no mode always follows the same one), under a trace
    cd /tmp
    timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 3 --rotate-order \
        --modes-pair plain,rotating,group,s:0.5,s:5.0,s:5.6,s:0.0 \
        --modes-scan plain,rotating,group,s:0.1.2.3.4.5.6.7.8.9.10.11.12.13.14.15,s:0.1.2.3.4.5.6.7.0.1.2.3.4.5.6.7,s:0.2.4.6.8.10.12.14.1.3.5.7.9.11.13.15 \
        --modes-tree plain,rotating,group,s:0.1.2.3.4.5.6.7.8,s:1.2.3.4.5.6.7.8.0,s:8.9.10.11.12.13.14.15.0 \
        > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl
    ;;
ab)
    cd /tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 3 > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl
    ;;
c)
    # placement, round three: is it the slot of each stream, or how consecutive launches' slots differ? Explicit
    # lists with a per-set shift (s:...@K): the bench's rotating layouts rebuilt exactly, and the group's with the
    # sets alternating halves; order rotated per rep, 4 reps
    cd /tmp
    timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 4 --rotate-order --kernels pair,scan \
        --modes-pair plain,rotating,group,s:0.1@2,s:0.0@2,s:0.0@0 \
        --modes-scan rotating,group,s:0.1.2.3.4.5.6.7.0.1.2.3.4.5.6.7@8,s:0.1.2.3.4.5.6.7.0.1.2.3.4.5.6.7@0,s:0.1.2.3.4.5.6.7.8.9.10.11.12.13.14.15@8,s:0.1.2.3.4.5.6.7.8.9.10.11.12.13.14.15@0 \
        > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl
    ;;
d)
    # the skewed shard receive in the product (FMI_TUNE_COMM_SHARD_SKEW): its parity tests (LOCAL, PROC, the full-size
    # C4 and C5 allreduces, the communicator sweep at its default seeds), then the shard kernel inside fmi_comm_allreduce
    # with 8 LOCAL ranks, skew on / off interleaved (tools/shard_skew_comm.py)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_comm.py tests/test_gpu_proc.py tests/test_gpu_comm_random_sweep.py \
        > gpurun_out/${TAG}_tests.log 2>&1 &&
    timeout -k 10 400 python -u tools/shard_skew_comm.py --ranks 8 --reps 4 > gpurun_out/${TAG}_shard_skew_comm.jsonl \
        2> gpurun_out/${TAG}_shard_skew_comm.err
    ;;
f)
    # the carved groups (fmi_dev_alloc_group: one allocation per group, bucket j at j x (bucket + 4 KiB)): their GPU
    # tests; then placement, round four: the carved group against rotating slots and the same slots as separate
    # allocations (s:...), order rotated per rep, 4 reps, under a trace; then the default line
    timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_parity.py -k "alloc" > gpurun_out/${TAG}_tests.log 2>&1 &&
    timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
        tests/test_cpp_communicator.py -m gpu >> gpurun_out/${TAG}_tests.log 2>&1 &&
    cd /tmp &&
    timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 4 --rotate-order \
        --modes-pair plain,group,rotating \
        --modes-scan rotating,group,s:0.1.2.3.4.5.6.7.8.9.10.11.12.13.14.15 \
        --modes-tree rotating,group,s:0.1.2.3.4.5.6.7.8,plain \
        > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl &&
    timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
    ;;
g)
    # the pair kernel's buckets: plain separate allocations, the carved group, each set carved at stride bucket + 0,
    # and all 16 sets carved from one 8 GiB allocation at + 0 / + 4 KiB; order rotated per rep, 4 reps, under a trace
    cd /tmp &&
    timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 4 --rotate-order --kernels pair \
        --modes-pair plain,group,c:0,call:0,call:4 \
        > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl &&
    timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_comm.py -k "skewed or c4_8peer or c5_host" tests/test_gpu_proc.py > gpurun_out/${TAG}_tests.log 2>&1 &&
    timeout -k 10 300 python -u tools/shard_layout_ab.py --reps 3 > gpurun_out/${TAG}_shard_layout.jsonl \
        2> gpurun_out/${TAG}_shard_layout.err
    ;;
p)
    # the N > 1 code path at world size 1 over RCCL with the full exchange (--force-dist, diagnostics on: the
    # exchange variants run the grouped all-to-all, i.e. RCCL's grouped ncclSend / ncclRecv with the skewed shard
    # receive), C5 at 1 GiB
    timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
        --master-port 29633 bench.py --force-dist --steps 20 --warmup 5 --c5-mib 1024 \
        > gpurun_out/${TAG}_force_dist.json 2> gpurun_out/${TAG}_force_dist.err
    ;;
q)
    # the N > 1 line rehearsed at full size with 8 ranks as processes on the one GPU (PROC transport over gloo):
    # 256 MiB buckets, C4 at 1 GiB per peer, C5 at 1 GiB per rank, diagnostics on
    FMI_PROC_TIMEOUT_S=300 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
        --master-addr 127.0.0.1 --master-port 29644 bench.py --gpus 8 --transport proc --steps 20 --warmup 3 \
        --diag-deadline 600 > gpurun_out/${TAG}_bench_proc8_rehearsal.json 2> gpurun_out/${TAG}_bench_proc8_rehearsal.err
    ;;
s)
    # soaks on the final library (placement changed: plain allocations by default, carved groups, skewed shards):
    # the P-way sweep and the communicator sweep at fresh seeds, every case bit-exact against the oracle
    FMI_SWEEP_SEEDS=70000:70400 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider tests/test_gpu_random_sweep.py > gpurun_out/r06_random_sweep_soak_70000_70400.log 2>&1 &&
    FMI_SWEEP_SEEDS=80000:80600 timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider tests/test_gpu_comm_random_sweep.py > gpurun_out/r06_comm_sweep_soak_80000_80600.log 2>&1
    ;;
h)
    # the device copy (the P = 1 allreduce, 1 in : 1 out) by placement: plain, carved group (dst in slot 1), carved
    # at + 0; 4 reps rotated, under a trace
    cd /tmp &&
    timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_placement_trace -o run -- \
        python3 $R/tools/placement_ab.py --reps 4 --rotate-order --kernels copy --steps 40 \
        > $R/gpurun_out/${TAG}_placement_ab.jsonl 2> $R/gpurun_out/${TAG}_placement_ab.err &&
    cd $R &&
    python3 tools/placement_ab_trace.py gpurun_out/${TAG}_placement_ab.jsonl gpurun_out/${TAG}_placement_trace \
        > gpurun_out/${TAG}_placement_ab_trace.jsonl
    ;;
t)
    # the N > 1 line's GPU tests after a change to its one-GPU anchor (local_equivalent on carved groups)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_bench_dist.py > gpurun_out/${TAG}_bench_dist_tests.log 2>&1
    ;;
l)
    # history (commit 8631a58, removed after this run: slower): the LOCAL transport's exchange ordered on the streams
    # by events (its FMI_TUNE_COMM_LOCAL_ASYNC key and tools/local_async_ab.py are gone): the communicator, PROC,
    # timeout and host suites on it; then C5's co-resident block, async / host-synchronised, interleaved 3x
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        tests/test_gpu_comm.py tests/test_gpu_timeout.py tests/test_gpu_comm_random_sweep.py tests/test_gpu_fmi_python.py \
        > gpurun_out/${TAG}_tests.log 2>&1 &&
    timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
        tests/test_cpp_communicator.py -m gpu >> gpurun_out/${TAG}_tests.log 2>&1 &&
    timeout -k 10 600 python -u tools/local_async_ab.py --reps 3 > gpurun_out/${TAG}_local_async_ab.jsonl \
        2> gpurun_out/${TAG}_local_async_ab.err
    ;;
i)
    # the fused kernels' in-flight cap x access policy re-checked on carved groups, two interleaved rounds
    timeout -k 10 400 python -u tools/fused_retune.py --rounds 2 --budgets 0,32,64,128 --policies 2,0 \
        > gpurun_out/${TAG}_fused_retune.jsonl 2> gpurun_out/${TAG}_fused_retune.err
    ;;
cold)
    # is C2 slower as the first work of a fresh box (the driver's bench runs so)? The line twice, back to back, as
    # the first GPU work of the call, then once more after a 60 s idle pause
    timeout -k 10 300 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/${TAG}_cold1.json 2> gpurun_out/${TAG}_cold1.err &&
    timeout -k 10 300 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/${TAG}_cold2.json 2> gpurun_out/${TAG}_cold2.err &&
    sleep 60 &&
    timeout -k 10 300 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/${TAG}_cold3.json 2> gpurun_out/${TAG}_cold3.err
    ;;
r)
    # the N > 1 line rehearsed at the scaling curve's other sizes, N = 2 and 4 PROC ranks on the one GPU, full size
    FMI_PROC_TIMEOUT_S=300 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
        --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --transport proc --steps 20 --warmup 3 \
        --diag-deadline 400 > gpurun_out/${TAG}_bench_proc2_rehearsal.json 2> gpurun_out/${TAG}_bench_proc2_rehearsal.err &&
    FMI_PROC_TIMEOUT_S=300 timeout -k 10 800 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
        --master-addr 127.0.0.1 --master-port 29666 bench.py --gpus 4 --transport proc --steps 20 --warmup 3 \
        --diag-deadline 500 > gpurun_out/${TAG}_bench_proc4_rehearsal.json 2> gpurun_out/${TAG}_bench_proc4_rehearsal.err
    ;;
two)
    # the default line twice in a row (separate processes)
    timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench1.json 2> gpurun_out/${TAG}_bench1.err &&
    timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err
    ;;
z)
    # the round-end sequence on the current library and bench: the whole GPU suite, smoke(), the default line, then
    # the C2 profile (kernel trace + stats, separate FETCH_SIZE / WRITE_SIZE passes, an unprofiled line; then
    # tools/pmc_summarize.py --tag $TAG_c2 --merge here)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/${TAG}_full_gpu.log 2>&1 &&
    timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 &&
    timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
    bash tools/c2_profile.sh
    ;;
*)
    echo "unknown step $1" >&2
    exit 2
    ;;
esac
