# Tail store-policy A/B of the pairwise kernel (tools/microbench_tailpol.hip): event timing, then the same
# binary under rocprofv3 --kernel-trace for per-launch medians.
# Usage (repo root, via gpurun; build/mbt built beforehand): bash tools/tailpol_run.sh
set -e -o pipefail
R=$PWD
mkdir -p gpurun_out/tp
timeout -k 10 240 build/mbt 7 > gpurun_out/tailpol_events.jsonl 2> gpurun_out/tailpol_events.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tp -o run -- $R/build/mbt 5 > $R/gpurun_out/tailpol_trace.log 2>&1
cd $R
python3 tools/trace_medians.py gpurun_out/tp pair_ > gpurun_out/tailpol_trace.jsonl
