# C2 profiles for profiles/: kernel trace + stats of the default bench command, then separate --pmc FETCH_SIZE
# and --pmc WRITE_SIZE passes (MI355X_MICROARCH.md HBM recipe), then an unprofiled run for comparison.
# Every profiled pass runs with --no-c5 --no-cpu-baseline: C5's host_pair_reduce block launches the same
# pair_tile<OpSum, float> instantiation on 1 GiB page-locked HOST buckets (PCIe-bound, ~40 ms a launch) and the
# CPU baseline's c1_reference GPU leg launches it on 1 MiB staged buckets; rocprofv3's per-name --stats average
# would mix those with C2's 256 MiB HBM launches (tools/pmc_summarize.py keeps shapes apart anyway).
set -e
R=$PWD
mkdir -p gpurun_out/c2t gpurun_out/c2f gpurun_out/c2w
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c2t -o run -- python3 $R/bench.py --no-c5 --no-cpu-baseline > $R/gpurun_out/c2_bench_under_rocprof.txt 2> $R/gpurun_out/c2t.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/c2f -o run -- python3 $R/bench.py --no-cpu-baseline --no-c5 --steps 40 --warmup 5 > $R/gpurun_out/c2f.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/c2w -o run -- python3 $R/bench.py --no-cpu-baseline --no-c5 --steps 40 --warmup 5 > $R/gpurun_out/c2w.log 2>&1
cd $R
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/c2_bench_plain.json
