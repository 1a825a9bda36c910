# Full round-end check as the driver runs it: the CPU suite (pytest -m "not gpu", which the driver runs in the
# build container — run here too so a red contract test cannot slip past a GPU-only sequence), pytest -m gpu,
# smoke(), default bench.py line.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m "not gpu" -x -q --timeout 300 > gpurun_out/full_cpu.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
