# Round 4's GPU calls, by step (profiles/INDEX.md names the files each made):
#   bash tools/gpu_round4.sh a   the round's new GPU tests, the default bench line, and the LDS-staged scan
#                                experiment under rocprofv3 (profiles/r04_a_*, r04_scan_lds*). Its last step ran
#                                build/mbscanlds from tools/microbench_scan_lds.hip, deleted after the experiment
#                                failed its stop rule (`git show a77d10c^:tools/microbench_scan_lds.hip`).
#   bash tools/gpu_round4.sh b   the default bench line after the C2-size reference baseline's no-op mode was
#                                fixed, then the C2 profile of the round-4 library (tools/c2_profile.sh:
#                                kernel trace + stats, separate FETCH_SIZE / WRITE_SIZE passes, an unprofiled line)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
case "$1" in
a)
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ref_binding.py \
        tests/test_gpu_timeout.py tests/test_gpu_comm.py::test_c5_host_allreduce_full_size tests/test_gpu_bench_dist.py \
        -rA > gpurun_out/r04_a_tests.log 2>&1 &&
    timeout -k 10 600 python bench.py > gpurun_out/r04_a_bench.json 2> gpurun_out/r04_a_bench.err
    ;;
b)
    timeout -k 10 600 python bench.py > gpurun_out/r04_b_bench.json 2> gpurun_out/r04_b_bench.err &&
    bash tools/c2_profile.sh
    ;;
*)
    echo "usage: bash tools/gpu_round4.sh a|b" >&2
    exit 2
    ;;
esac
