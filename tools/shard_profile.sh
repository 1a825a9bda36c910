# PMC evidence for bench.py's N > 1 roofline.traffic: the fused shard kernel at the headline's shard shapes
# (tools/shard_kernels.py), kernel trace + separate --pmc FETCH_SIZE / WRITE_SIZE passes, merged into
# profiles/pmc_summary.json (MI355X_MICROARCH.md HBM recipe).
set -e
R=$PWD
mkdir -p gpurun_out/sht gpurun_out/shf gpurun_out/shw
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sht -o run -- python3 $R/tools/shard_kernels.py > $R/gpurun_out/sht.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/shf -o run -- python3 $R/tools/shard_kernels.py > $R/gpurun_out/shf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/shw -o run -- python3 $R/tools/shard_kernels.py > $R/gpurun_out/shw.log 2>&1
cd $R
python3 tools/pmc_summarize.py --trace gpurun_out/sht --fetch gpurun_out/shf --write gpurun_out/shw --tag ${TAG:-r02_shard} \
  --command "rocprofv3 -- python3 tools/shard_kernels.py (tools/shard_profile.sh)" --merge > gpurun_out/r02_shard_pmc.json
