set -e
R=$PWD
mkdir -p gpurun_out/c3t gpurun_out/c3f gpurun_out/c3w
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3t -o run -- python3 $R/tools/c3_kernels.py > $R/gpurun_out/c3t.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/c3f -o run -- python3 $R/tools/c3_kernels.py > $R/gpurun_out/c3f.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/c3w -o run -- python3 $R/tools/c3_kernels.py > $R/gpurun_out/c3w.log 2>&1
cd $R
find gpurun_out/c3t gpurun_out/c3f gpurun_out/c3w -name "*.csv" | head -20
