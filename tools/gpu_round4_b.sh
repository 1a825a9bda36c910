# Round 4, second GPU call (profiles/r04_b_bench.json, r04_c2_*): the default bench line after the C2-size
# reference baseline's no-op mode was fixed, then the C2 profile (kernel trace + stats, separate FETCH_SIZE /
# WRITE_SIZE passes, an unprofiled line) of the round-4 library: tools/c2_profile.sh.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r04_b_bench.json 2> gpurun_out/r04_b_bench.err &&
bash tools/c2_profile.sh
