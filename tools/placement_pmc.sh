# PMC passes over tools/microbench_placement.hip (scan8 placement study): per-dispatch TLB, DRAM credit
# stalls and read latency, each pass its own rocprofv3 run (MI355X_MICROARCH.md: no counter splitting).
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
n=0
for pmc in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" \
           "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  mkdir -p $R/gpurun_out/plpmc/p$n
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $R/gpurun_out/plpmc/p$n -o run -- $R/build/mbp2 6 > $R/gpurun_out/plpmc/p$n.log 2>&1
done
