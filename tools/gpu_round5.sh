# Round 5's GPU calls, by step (profiles/INDEX.md names the files each made):
#   bash tools/gpu_round5.sh a   C5's co-resident DMA ceiling by issue shape (tools/microbench_pcie_peers.hip: own vs
#                                shared streams, SDMA vs kernel copies, 1 / 2 / 8 peers), the host-combine crossover
#                                (tools/host_crossover.py), the counters this rocprofv3 offers, and the fused 8-way
#                                allreduce at 256 / 512 / 1024 MiB per peer under a kernel trace (tools/tree8_shapes.py)
#   bash tools/gpu_round5.sh b   the same three tree shapes under seven separate --pmc passes (read / write request
#                                levels and DRAM credit stalls, translation, TA / SQ stalls, FETCH_SIZE, WRITE_SIZE)
#   bash tools/gpu_round5.sh c   the pooled fmi_host_reduce_pair staging and the shared per-device copy streams of
#                                fmi_comm_allreduce_host: the whole GPU suite, C5's p1_copy + local_peers blocks, and the
#                                host-combine crossover to 512 MiB (profiles/r05_c_*, r05_c5_blocks.json)
#   bash tools/gpu_round5.sh d   the tree shapes by placement (inputs carved from one allocation at stride bucket + K
#                                KiB) and with the bucket launched in slices (profiles/r05_tree8_skew.jsonl, _slices)
#   bash tools/gpu_round5.sh e   C5's local_peers block (8 LOCAL ranks x 1 GiB) at 8 / 16 / 32 / 64 MiB pipeline chunks
#                                per rank (profiles/r05_c5_chunks.jsonl)
#   bash tools/gpu_round5.sh f   placement sweep: pair (C2), tree8 (32 / 512 MiB), scan8 (C3), copy, each with its
#                                buckets carved from one allocation at stride bucket + K KiB (profiles/r05_skew_sweep.jsonl)
#   bash tools/gpu_round5.sh g   the slotted fmi_dev_alloc: the whole GPU suite, separate allocations with slots off /
#                                on twice (profiles/r05_alloc_slots_ab.jsonl), the default bench line (r05_g_*)
#   bash tools/gpu_round5.sh h   the pair kernel, slots off / on x 4 (r05_pair_slots_ab.jsonl); C5's co-resident block
#                                with the 3-slot host pipeline at 32 / 64 MiB chunks, tapered or not, twice
#                                (r05_c5_chunks_depth3.jsonl)
#   bash tools/gpu_round5.sh i   FMI_TUNE_FUSED_INFLIGHT_KIB x FMI_TUNE_FUSED_POLICY on slotted buckets: tree8 1 GiB /
#                                32 MiB, scan8 64 MiB, two interleaved rounds (r05_fused_retune.jsonl); then the 8-peer
#                                shared-stream DMA with and without a concurrent HBM copy loop (r05_pcie_busy.jsonl)
#   bash tools/gpu_round5.sh j   host pipeline 3 vs 2 chunk slots (build/ab_d2; remove it from .gpurunignore to rerun), 3 x
#                                interleaved processes (r05_depth_ab.jsonl)
#   bash tools/gpu_round5.sh k   8-in / 1-out tree shape, U = 1 / 2 / 4 lane groups per thread x a cap of 2 / 4 / 8 / no
#                                workgroups per CU, slotted buckets, 1 GiB and 32 MiB per peer (tools/microbench_tree_u.hip)
#   bash tools/gpu_round5.sh l   C5 local_peers at GPU_MAX_HW_QUEUES 4 / 8 / 16, twice (r05_c5_hwq.jsonl)
#   bash tools/gpu_round5.sh m   C5 local_peers under rocprofv3 --kernel-trace --memory-copy-trace (r05_c5_trace*)
#   bash tools/gpu_round5.sh n   co-resident ranks' chunk-major first loads + small first chunks vs the build before
#                                (build/ab_prev), 3 x interleaved (r05_c5_start_ab.jsonl); then step m on the library
#   bash tools/gpu_round5.sh o   the pair kernel's sc1 tiles re-checked on slotted buckets (r05_ab_pair_sc1.jsonl)
#   bash tools/gpu_round5.sh p   bench.py --force-dist at world 1 over RCCL with C5 at 1 GiB (r05_force_dist_c5.json)
#   bash tools/gpu_round5.sh q   the N > 1 line at full size, 8 PROC ranks on one GPU (r05_bench_proc8_rehearsal.json)
#   bash tools/gpu_round5.sh z   the round-end sequence: GPU suite, smoke(), default line, C2 profile (r05z_*;
#                                then tools/pmc_summarize.py --tag r05z_c2 --merge)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
case "$1" in
a)
    timeout -k 10 240 build/mbpciepeers 3 0 > gpurun_out/r05_pcie_peers.jsonl 2> gpurun_out/r05_pcie_peers.err &&
    timeout -k 10 240 build/mbpciepeers 3 6 >> gpurun_out/r05_pcie_peers.jsonl 2>> gpurun_out/r05_pcie_peers.err &&
    timeout -k 10 200 python -u tools/host_crossover.py > gpurun_out/r05_host_crossover.jsonl 2> gpurun_out/r05_host_crossover.err &&
    timeout -k 10 120 rocprofv3 -L > gpurun_out/r05_rocprofv3_counters.txt 2>&1 &&
    timeout -k 10 200 python -u tools/tree8_shapes.py --mib 256,512,1024,512,256 > gpurun_out/r05_tree8_events.jsonl &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_tree8_trace -o run -- \
        python3 tools/tree8_shapes.py --mib 256,512,1024 > gpurun_out/r05_tree8_under_trace.jsonl 2> gpurun_out/r05_tree8_trace.err
    ;;
b)
    # one --pmc pass per counter group (MI355X_MICROARCH.md: separate passes, <= 4 TCC / 4 TCP / 2 TA / 2 GRBM / 8 SQ)
    R=$PWD
    cd /tmp
    k=0
    for pmc in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE" \
               "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE" \
               "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
               "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
               "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_BUSY_sum"; do
        k=$((k + 1))
        timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $R/gpurun_out/r05_tree8_pmc$k -o run -- \
            python3 $R/tools/tree8_shapes.py --mib 256,512,1024 > $R/gpurun_out/r05_tree8_pmc$k.jsonl 2> $R/gpurun_out/r05_tree8_pmc$k.err || exit 1
    done
    ;;
c)
    # the pooled host-combine staging and the shared per-device copy streams: their GPU tests, C5's blocks, the
    # crossover sweep to 512 MiB
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/r05_c_full_gpu.log 2>&1 &&
    timeout -k 10 300 python -u -c "
import json, bench, fmi_amd
fmi_amd.init(0)
bench.quiet_device()
print(json.dumps({'p1_copy': bench.c5_p1_copy(1024), 'local_peers': bench.c5_local_peers(8, 1024)}))
" > gpurun_out/r05_c5_blocks.json 2> gpurun_out/r05_c5_blocks.err &&
    timeout -k 10 300 python -u tools/host_crossover.py > gpurun_out/r05_host_crossover_512.jsonl 2> gpurun_out/r05_host_crossover_512.err
    ;;
d)
    # placement: the tree shapes with the 8 inputs + output carved from ONE allocation at stride bucket + K KiB
    # (K = -1: separate allocations), and the 1 GiB bucket launched as 4 slices of 256 MiB
    timeout -k 10 300 python -u tools/tree8_shapes.py --mib 256,512,1024 --skew-kib=-1,0,4,64,2052 \
        > gpurun_out/r05_tree8_skew.jsonl 2> gpurun_out/r05_tree8_skew.err &&
    timeout -k 10 200 python -u tools/tree8_shapes.py --mib 512,1024 --slices 1,2,4 \
        > gpurun_out/r05_tree8_slices.jsonl 2> gpurun_out/r05_tree8_slices.err
    ;;
e)
    # C5's co-resident block by pipeline chunk per rank (the shared copy streams' fill and drain shrink with it)
    timeout -k 10 400 python -u -c "
import json, bench, fmi_amd
fmi_amd.init(0)
for chunk in (8, 16, 32, 64, 16):
    bench.quiet_device()
    r = bench.c5_local_peers(8, 1024, chunk_mib=chunk)
    print(json.dumps({'chunk_mib': chunk, 'ms': r['ms'], 'pcie_GB_s': r['pcie_GB_s_both_directions'], 'ok': r['self_check']['ok']}), flush=True)
" > gpurun_out/r05_c5_chunks.jsonl 2> gpurun_out/r05_c5_chunks.err
    ;;
f)
    # placement sweep over every kernel shape of the line (tools/skew_sweep.py)
    timeout -k 10 600 python -u tools/skew_sweep.py --skew-kib=-1,0,1,2,4,8,16,32,2052 --tree-mib 32,512 \
        > gpurun_out/r05_skew_sweep.jsonl 2> gpurun_out/r05_skew_sweep.err
    ;;
g)
    # the slotted allocator: the whole GPU suite, the sweep's separate-allocation rows with slots off / on, the
    # default line
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/r05_g_full_gpu.log 2>&1 &&
    timeout -k 10 400 python -u tools/skew_sweep.py --skew-kib=-1 --alloc-slots 0,1,0,1 --tree-mib 32,128,512,1024 \
        > gpurun_out/r05_alloc_slots_ab.jsonl 2> gpurun_out/r05_alloc_slots_ab.err &&
    timeout -k 10 600 python bench.py > gpurun_out/r05_g_bench.json 2> gpurun_out/r05_g_bench.err
    ;;
h)
    # the pair kernel (C2) on separate allocations, slots off / on interleaved 4 times; then C5's co-resident block
    # with the 3-slot host pipeline at 32 / 64 MiB chunks, tapered and not, twice each
    timeout -k 10 300 python -u tools/skew_sweep.py --kernels pair --skew-kib=-1 --alloc-slots 0,1,0,1,0,1,0,1 \
        --launches 96 > gpurun_out/r05_pair_slots_ab.jsonl 2> gpurun_out/r05_pair_slots_ab.err &&
    timeout -k 10 500 python -u -c "
import json, bench, fmi_amd
fmi_amd.init(0)
for taper in (1, 0, 1, 0):  # as run: against fad2b1e's FMI_TUNE_HOST_TAPER (removed after: no gain)
    if hasattr(fmi_amd.Tune, 'HOST_TAPER'):
        fmi_amd.tune_set(fmi_amd.Tune.HOST_TAPER, taper)
    for chunk in (32, 64):
        bench.quiet_device()
        r = bench.c5_local_peers(8, 1024, chunk_mib=chunk)
        print(json.dumps({'chunk_mib': chunk, 'depth': 3, 'taper': taper, 'ms': r['ms'], 'pcie_GB_s': r['pcie_GB_s_both_directions'], 'ok': r['self_check']['ok']}), flush=True)
" > gpurun_out/r05_c5_chunks_depth3.jsonl 2> gpurun_out/r05_c5_chunks_depth3.err
    ;;
i)
    # the fused kernels' in-flight cap and access policy re-tuned on slotted buckets (tools/fused_retune.py)
    timeout -k 10 400 python -u tools/fused_retune.py --rounds 2 > gpurun_out/r05_fused_retune.jsonl \
        2> gpurun_out/r05_fused_retune.err &&
    timeout -k 10 200 build/mbpciepeers 3 0 1 > gpurun_out/r05_pcie_busy.jsonl 2> gpurun_out/r05_pcie_busy.err
    ;;
j)
    # the host pipeline depth of the library (2, or 3 for co-resident LOCAL ranks) vs always 2 (build/ab_d2, made by
    # round 5's `ab_depth2` Makefile target, removed with its compile-time hook in round 6: this step is history;
    # first run: the library at 3 for every communicator), separate processes, interleaved three times: C5's
    # p1_copy and local_peers blocks
    for k in 1 2 3; do
        for lib in fmi_amd/lib/libfmi_dev.so build/ab_d2/libfmi_dev.so; do
            FMI_DEV_LIB=$PWD/$lib timeout -k 10 200 python -u -c "
import json, os, bench, fmi_amd
fmi_amd.init(0)
bench.quiet_device()
p1 = bench.c5_p1_copy(1024)
bench.quiet_device()
lp = bench.c5_local_peers(8, 1024)
print(json.dumps({'lib': os.environ['FMI_DEV_LIB'].split('/repo/')[-1], 'p1_copy_ms': p1['ms'], 'p1_ok': p1['self_check']['ok'],
                  'local_peers_ms': lp['ms'], 'local_peers_GB_s': lp['pcie_GB_s_both_directions'], 'lp_ok': lp['self_check']['ok']}))
" >> gpurun_out/r05_depth_ab.jsonl 2>> gpurun_out/r05_depth_ab.err || exit 1
        done
    done
    ;;
k)
    # the 8-way tree's lane groups per thread (U) x workgroups-per-CU cap on slotted buckets (build/mbtreeu)
    timeout -k 10 300 build/mbtreeu 3 > gpurun_out/${OUT:-r05_tree_u}.jsonl 2> gpurun_out/${OUT:-r05_tree_u}.err
    ;;
l)
    # C5's co-resident block against the process's hardware-queue count (GPU_MAX_HW_QUEUES 4 / 8 / 16), twice
    for q in 4 8 16 4 8 16; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u -c "
import json, os, bench, fmi_amd
fmi_amd.init(0)
bench.quiet_device()
lp = bench.c5_local_peers(8, 1024)
print(json.dumps({'GPU_MAX_HW_QUEUES': int(os.environ['GPU_MAX_HW_QUEUES']), 'ms': lp['ms'], 'pcie_GB_s': lp['pcie_GB_s_both_directions'], 'ok': lp['self_check']['ok']}))
" >> gpurun_out/r05_c5_hwq.jsonl 2>> gpurun_out/r05_c5_hwq.err || exit 1
    done
    ;;
m)
    # C5's co-resident block under a kernel + memory-copy trace: where the 25 ms above the copy ceiling go
    R=$PWD
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r05_c5_trace \
        -o run -- python3 -c "
import sys, json
sys.path.insert(0, '$R')
import bench, fmi_amd
fmi_amd.init(0)
bench.quiet_device()
lp = bench.c5_local_peers(8, 1024, iters=1)
print(json.dumps({'ms': lp['ms'], 'ok': lp['self_check']['ok']}))
" > $R/gpurun_out/r05_c5_trace.json 2> $R/gpurun_out/r05_c5_trace.err
    ;;
n)
    # the library against the previous build (build/ab_prev: before the co-resident ranks' chunk-major first loads
    # and small first chunks), separate processes interleaved three times; then the library under the copy trace
    for k in 1 2 3; do
        for lib in fmi_amd/lib/libfmi_dev.so build/ab_prev/libfmi_dev.so; do
            FMI_DEV_LIB=$PWD/$lib timeout -k 10 200 python -u -c "
import json, os, bench, fmi_amd
fmi_amd.init(0)
bench.quiet_device()
p1 = bench.c5_p1_copy(1024)
bench.quiet_device()
lp = bench.c5_local_peers(8, 1024)
print(json.dumps({'lib': os.environ['FMI_DEV_LIB'].split('/repo/')[-1], 'p1_copy_ms': p1['ms'], 'p1_ok': p1['self_check']['ok'],
                  'local_peers_ms': lp['ms'], 'local_peers_GB_s': lp['pcie_GB_s_both_directions'], 'lp_ok': lp['self_check']['ok']}))
" >> gpurun_out/r05_c5_start_ab.jsonl 2>> gpurun_out/r05_c5_start_ab.err || exit 1
        done
    done
    rm -rf gpurun_out/r05_c5_trace && bash tools/gpu_round5.sh m
    ;;
o)
    # the pair kernel's sc1 tiles (FMI_TUNE_PAIR_SC1_OF_8 0 / 1 / 2 / 4) re-checked on slotted buckets: C2 (256 MiB,
    # 16 sets) and C3's i64 shape (64 MiB, 64 sets)
    timeout -k 10 300 python -u tools/ab_pair_sc1.py --rounds 5 --mib 256 --sets 16 --budgets 0,1,2,4 \
        > gpurun_out/r05_ab_pair_sc1.jsonl 2> gpurun_out/r05_ab_pair_sc1.err &&
    timeout -k 10 300 python -u tools/ab_pair_sc1.py --rounds 5 --mib 64 --sets 64 --dtype i64 --budgets 0,1,2,4 \
        >> gpurun_out/r05_ab_pair_sc1.jsonl 2>> gpurun_out/r05_ab_pair_sc1.err
    ;;
p)
    # the N > 1 code path at world size 1 over RCCL with the full exchange (--force-dist): C5's per-GPU pipeline with
    # the real RCCL calls per chunk, 1 GiB (the closest one-GPU form of C5 as BASELINE states it)
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --force-dist --steps 20 --warmup 5 --c5-mib 1024 --no-diagnostics \
        > gpurun_out/r05_force_dist_c5.json 2> gpurun_out/r05_force_dist_c5.err
    ;;
q)
    # the N > 1 line rehearsed at full size with 8 ranks as processes on the one GPU (PROC transport over gloo):
    # 256 MiB buckets, C4 at 1 GiB per peer, C5 at 1 GiB per rank, diagnostics on
    FMI_PROC_TIMEOUT_S=300 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
        --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 8 --transport proc --steps 20 --warmup 3 \
        --diag-deadline 600 > gpurun_out/r05_bench_proc8_rehearsal.json 2> gpurun_out/r05_bench_proc8_rehearsal.err
    ;;
z)
    # the round-end sequence on the final library and bench: the whole GPU suite, smoke(), the default line, then
    # the C2 profile (kernel trace + stats, separate FETCH_SIZE / WRITE_SIZE passes, an unprofiled line)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/${TAG:-r05z}_full_gpu.log 2>&1 &&
    timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG:-r05z}_smoke.log 2>&1 &&
    timeout -k 10 600 python bench.py > gpurun_out/${TAG:-r05z}_bench.json 2> gpurun_out/${TAG:-r05z}_bench.err &&
    bash tools/c2_profile.sh
    ;;
*)
    echo "usage: bash tools/gpu_round5.sh a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|z" >&2
    exit 2
    ;;
esac
