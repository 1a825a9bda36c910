# Translation counters of the many-peer scan probe (tools/probe_scan_cliff.py --short), one rocprofv3 pass per
# counter group (MI355X_MICROARCH.md: no counter splitting). Usage (repo root, via gpurun): bash tools/scan_cliff_pmc.sh
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
n=0
for pmc in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  mkdir -p $R/gpurun_out/clpmc/p$n
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $R/gpurun_out/clpmc/p$n -o run -- python3 $R/tools/probe_scan_cliff.py --short > $R/gpurun_out/clpmc/p$n.log 2>&1
done
