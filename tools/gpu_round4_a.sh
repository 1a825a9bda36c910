# Round 4, first GPU call (profiles/r04_a_*, r04_scan_lds*): the round's new GPU tests, the default bench line,
# and the LDS-staged scan experiment under rocprofv3. Its third step ran build/mbscanlds, built from
# tools/microbench_scan_lds.hip, which was deleted after the experiment failed its stop rule (the
# source is in git history at the commit that added profiles/r04_scan_lds.jsonl).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ref_binding.py tests/test_gpu_timeout.py tests/test_gpu_comm.py::test_c5_host_allreduce_full_size tests/test_gpu_bench_dist.py -rA > gpurun_out/r04_a_tests.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/r04_a_bench.json 2> gpurun_out/r04_a_bench.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r04_scanlds -o run -- /root/repo/build/mbscanlds 3 > /root/repo/gpurun_out/r04_scanlds.jsonl 2> /root/repo/gpurun_out/r04_scanlds.err
