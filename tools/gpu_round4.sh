# Round 4's GPU calls, by step (profiles/INDEX.md names the files each made):
#   bash tools/gpu_round4.sh a   the round's new GPU tests, the default bench line, and the LDS-staged scan
#                                experiment under rocprofv3 (profiles/r04_a_*, r04_scan_lds*). Its last step ran
#                                build/mbscanlds from tools/microbench_scan_lds.hip, deleted after the experiment
#                                failed its stop rule (`git show a77d10c^:tools/microbench_scan_lds.hip`).
#   bash tools/gpu_round4.sh b   the default bench line after the C2-size reference baseline's no-op mode was
#                                fixed, then the C2 profile of the round-4 library (tools/c2_profile.sh:
#                                kernel trace + stats, separate FETCH_SIZE / WRITE_SIZE passes, an unprofiled line)
#   bash tools/gpu_round4.sh e   the HIP path against the extended reference fixtures (f64 prod / min, i32 / i64 x
#                                4 ops), then the default bench line with the GPU-bound reference allreduce at 256 MiB
#                                (profiles/r04_ref_vectors_gpu.log, r04_e_bench.json)
#   bash tools/gpu_round4.sh f [tag]  fmi_host_reduce_pair on pageable 256 MiB pairs from 1, 2 and 4 threads at once (the
#                                reference binding's peers combine concurrently; profiles/r04_host_pair_threads*.jsonl)
#   bash tools/gpu_round4.sh c   C5's local_peers block (8 LOCAL ranks x 1 GiB) at GPU_MAX_HW_QUEUES = 4 / 8 / 16
#                                (profiles/r04_c5_local_peers_hwq.jsonl)
#   bash tools/gpu_round4.sh d   the DMA ceiling of that shape: 8 threads, each streaming 1 GiB H2D and 1 GiB D2H
#                                on two streams in 64 / 256 MiB pieces, no compute (profiles/r04_pcie_8streams.jsonl)
#   bash tools/gpu_round4.sh g   the round-end sequence on the final library: the whole GPU suite, smoke(), the default
#                                bench line, then the C2 profile (profiles/r04g_*)
#   bash tools/gpu_round4.sh h   the fused 8-way allreduce kernel against bucket size per peer (64 MiB .. 1 GiB),
#                                after a quiet second, events over back-to-back launches (profiles/r04_tree8_sizes.jsonl)
#   bash tools/gpu_round4.sh i   fmi_host_reduce_pair's staging chunk (FMI_TUNE_HOST_CHUNK 4..64 MiB) on pageable 256 MiB
#                                and 1 MiB pairs, 1 and 2 threads (profiles/r04_host_chunk_sweep.jsonl)
#   bash tools/gpu_round4.sh j   host memcpy bandwidth, pageable -> page-locked, 1..8 threads (numpy copyto, GIL
#                                released): could CPU-side staging beat the runtime's pageable copies? (r04_host_memcpy.jsonl)
#   bash tools/gpu_round4.sh k   the host-staged pageable pipeline (FMI_TUNE_HOST_COPY_THREADS 0 = the runtime's
#                                pageable copies, 2 / 4 / 8 threads) x staging chunk 4 / 16 / 64 MiB, on 256 MiB and
#                                1 MiB pairs, 1 and 2 callers (profiles/r04_host_staged_sweep.jsonl). Rejected and
#                                removed: it runs only against the library of commit ba6eddb
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
g)
    timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/r04g_full_gpu.log 2>&1 &&
    timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04g_smoke.log 2>&1 &&
    timeout -k 10 600 python bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err &&
    bash tools/c2_profile.sh
    ;;
h)
    timeout -k 10 300 python -u - > gpurun_out/r04_tree8_sizes.jsonl <<'PY'
import json, sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
import fmi_amd
from fmi_amd import Alg, Bucket, Event, Op
fmi_amd.init(0)
def run(mib, sets, launches=12, peers=8):
    n = mib * (1 << 20) // 4
    ins = [[Bucket(n, np.float32).fill_synthetic(11 + s, p) for p in range(peers)] for s in range(sets)]
    out = Bucket(n, np.float32)
    fmi_amd.sync()
    time.sleep(1.0)
    for k in range(2):
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins[k % sets])
    e0, e1 = Event(), Event()
    e0.record()
    for k in range(launches):
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins[k % sets])
    e1.record()
    e1.sync()
    ms = e0.elapsed_ms(e1) / launches
    per = []
    for k in range(min(sets * 2, 8)):
        a, b = Event(), Event()
        a.record(); fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins[k % sets]); b.record(); b.sync()
        per.append(round(a.elapsed_ms(b) * 1e3, 1))
    for b in [out] + [x for s in ins for x in s]:
        b.free()
    algo = (peers + 1) * n * 4
    return {"mib_per_peer": mib, "sets": sets, "us": round(ms * 1e3, 2), "frac": round(algo / (ms * 1e-3) / 8e12, 4), "single_launch_us": per}
for mib, sets in [(1024, 1), (512, 1), (256, 2), (128, 4), (64, 8), (1024, 1)]:
    print(json.dumps(run(mib, sets)), flush=True)
PY
    ;;
i | k)
    out=gpurun_out/r04_host_chunk_sweep.jsonl
    [ "$1" = k ] && out=gpurun_out/r04_host_staged_sweep.jsonl
    MODE=$1 timeout -k 10 400 python -u - > "$out" <<'PY'
import json, threading, time, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import fmi_amd
from fmi_amd import Op, Tune
fmi_amd.init(0)
def run(mib, threads, reps):
    n = (mib << 20) // 4
    pairs = [(np.random.default_rng(t).random(n, dtype=np.float32), np.random.default_rng(9 + t).random(n, dtype=np.float32)) for t in range(threads)]
    want = [a + b for a, b in pairs]
    bar = threading.Barrier(threads)
    times = [[0.0] * reps for _ in range(threads)]
    def body(t):
        a0, b = pairs[t]
        for r in range(reps):
            a = a0.copy()
            bar.wait()
            t0 = time.perf_counter()
            fmi_amd.host_reduce_pair(Op.SUM, a, b)
            times[t][r] = time.perf_counter() - t0
            if r == reps - 1 and not np.array_equal(a, want[t]):
                bad.append((mib, threads, t))
    bad = []
    th = [threading.Thread(target=body, args=(t,)) for t in range(threads)]
    [x.start() for x in th]; [x.join() for x in th]
    if bad:
        raise SystemExit(f"result mismatch: {bad}")
    per = sorted(max(times[t][r] for t in range(threads)) for r in range(1, reps))
    return round(per[len(per) // 2] * 1e3, 3)
if os.environ["MODE"] == "i":
    for chunk in (4, 8, 16, 32, 64):
        fmi_amd.tune_set(Tune.HOST_CHUNK, chunk << 20)
        row = {"chunk_mib": chunk, "pair_256MiB_1thread_ms": run(256, 1, 5), "pair_256MiB_2threads_ms": run(256, 2, 5),
               "pair_1MiB_1thread_ms": run(1, 1, 21)}
        print(json.dumps(row), flush=True)
else:
    for threads in (0, 2, 4, 8):
        fmi_amd.tune_set(Tune.HOST_COPY_THREADS, threads)
        for chunk in ((64,) if threads == 0 else (4, 16, 64)):
            fmi_amd.tune_set(Tune.HOST_STAGE_CHUNK if threads else Tune.HOST_CHUNK, chunk << 20)
            row = {"copy_threads": threads, "chunk_mib": chunk, "pair_256MiB_1caller_ms": run(256, 1, 5),
                   "pair_256MiB_2callers_ms": run(256, 2, 5), "pair_1MiB_1caller_ms": run(1, 1, 21)}
            print(json.dumps(row), flush=True)
PY
    ;;
j)
    timeout -k 10 300 python -u - > gpurun_out/r04_host_memcpy.jsonl <<'PY'
import json, threading, time, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import fmi_amd
from fmi_amd.device import PinnedArray
fmi_amd.init(0)
n = (512 << 20) // 4
src = np.random.default_rng(1).random(n, dtype=np.float32)
dst = PinnedArray(n, np.float32)
for threads in (1, 2, 4, 8):
    parts = np.array_split(np.arange(n), threads)
    bounds = [(int(p[0]), int(p[-1]) + 1) for p in parts]
    best = 1e9
    for rep in range(5):
        bar = threading.Barrier(threads + 1)
        def body(lo, hi):
            bar.wait()
            np.copyto(dst.array[lo:hi], src[lo:hi])
        th = [threading.Thread(target=body, args=b) for b in bounds]
        [x.start() for x in th]
        bar.wait()
        t0 = time.perf_counter()
        [x.join() for x in th]
        best = min(best, time.perf_counter() - t0)
    assert np.array_equal(dst.array, src)
    print(json.dumps({"threads": threads, "MiB": 512, "ms": round(best * 1e3, 2), "GB_s": round(n * 4 / best / 1e9, 1)}), flush=True)
back = np.empty_like(src)
for threads in (1, 2, 4, 8):  # and the other way: page-locked -> pageable (the host-staged path's copy-out)
    parts = np.array_split(np.arange(n), threads)
    bounds = [(int(p[0]), int(p[-1]) + 1) for p in parts]
    best = 1e9
    for rep in range(5):
        bar = threading.Barrier(threads + 1)
        def body(lo, hi):
            bar.wait()
            np.copyto(back[lo:hi], dst.array[lo:hi])
        th = [threading.Thread(target=body, args=b) for b in bounds]
        [x.start() for x in th]
        bar.wait()
        t0 = time.perf_counter()
        [x.join() for x in th]
        best = min(best, time.perf_counter() - t0)
    assert np.array_equal(back, src)
    print(json.dumps({"direction": "page-locked -> pageable", "threads": threads, "MiB": 512, "ms": round(best * 1e3, 2), "GB_s": round(n * 4 / best / 1e9, 1)}), flush=True)
dst.free()
PY
    ;;
f)
    timeout -k 10 300 python -u - > "gpurun_out/r04_host_pair_threads${2:+_$2}.jsonl" <<'PY'
import json, threading, time, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import fmi_amd
from fmi_amd import Op
fmi_amd.init(0)
n = (256 << 20) // 4
def run(threads, reps=4):
    pairs = [(np.random.default_rng(t).random(n, dtype=np.float32), np.random.default_rng(100 + t).random(n, dtype=np.float32)) for t in range(threads)]
    want = []
    for a, b in pairs:  # the result after `reps` in-place sums, in the same order
        w = a.copy()
        for _ in range(reps):
            w += b
        want.append(w)
    bar = threading.Barrier(threads)
    times = [[0.0] * reps for _ in range(threads)]
    def body(t):
        a, b = pairs[t]
        for r in range(reps):
            bar.wait()
            t0 = time.perf_counter()
            fmi_amd.host_reduce_pair(Op.SUM, a, b)
            times[t][r] = time.perf_counter() - t0
    th = [threading.Thread(target=body, args=(t,)) for t in range(threads)]
    [x.start() for x in th]; [x.join() for x in th]
    per = sorted(max(times[t][r] for t in range(threads)) for r in range(1, reps))
    exact = all(np.array_equal(pairs[t][0], want[t]) for t in range(threads))
    return {"threads": threads, "pageable_256MiB_pairs": threads, "ms": round(per[len(per) // 2] * 1e3, 2), "bit_exact": exact}
for k in (1, 2, 4):
    print(json.dumps(run(k)), flush=True)
PY
    ;;
e)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_ref_vectors.py -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/r04_ref_vectors_gpu.log 2>&1 &&
    timeout -k 10 600 python bench.py > gpurun_out/r04_e_bench.json 2> gpurun_out/r04_e_bench.err
    ;;
c)
    for q in 4 8 16; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u -c "
import json, bench, fmi_amd
fmi_amd.init(0)
r = bench.c5_local_peers(8, 1024)
print(json.dumps({'GPU_MAX_HW_QUEUES': $q, 'ms': r['ms'], 'host_buckets_GiB_s': r['host_buckets_GiB_s'],
                  'pcie_GB_s': r['pcie_GB_s_both_directions'], 'ok': r['self_check']['ok']}))
" >> gpurun_out/r04_c5_local_peers_hwq.jsonl || exit 1
    done
    ;;
d)
    timeout -k 10 300 python -u - > gpurun_out/r04_pcie_8streams.jsonl <<'PY'
import sys, os
sys.path.insert(0, os.getcwd())
import json, threading, time, ctypes
import numpy as np
import fmi_amd
from fmi_amd import Bucket, PinnedArray, _lib, Stream
fmi_amd.init(0)
MIB = 1 << 20
def run(peers, mib, chunk_mib, duplex=True):
    n = mib * MIB
    hs = [PinnedArray(n // 4, np.float32) for _ in range(peers)]
    ho = [PinnedArray(n // 4, np.float32) for _ in range(peers)]
    ds = [Bucket(n // 4, np.float32) for _ in range(peers)]
    st = [(Stream(), Stream()) for _ in range(peers)]
    bar = threading.Barrier(peers)
    t = [0.0] * peers
    def rank(r):
        bar.wait()
        t0 = time.perf_counter()
        c = chunk_mib * MIB
        for o in range(0, n, c):
            _lib.call("fmi_dev_h2d_async", ds[r].ptr + o, hs[r].ptr + o, c, st[r][0].handle)
            if duplex:
                _lib.call("fmi_dev_d2h_async", ho[r].ptr + o, ds[r].ptr + o, c, st[r][1].handle)
        _lib.call("fmi_stream_sync", st[r][0].handle)
        _lib.call("fmi_stream_sync", st[r][1].handle)
        t[r] = time.perf_counter() - t0
    for _ in range(2):
        th = [threading.Thread(target=rank, args=(r,)) for r in range(peers)]
        [x.start() for x in th]; [x.join() for x in th]
    ms = max(t) * 1e3
    for x in hs + ho: x.free()
    for x in ds: x.free()
    return {"peers": peers, "mib": mib, "chunk_mib": chunk_mib, "duplex": duplex, "ms": round(ms, 2),
            "GB_s_total": round((2 if duplex else 1) * peers * n / (ms * 1e-3) / 1e9, 1)}
for args in [(1, 1024, 64), (8, 1024, 64), (8, 1024, 64, False), (8, 1024, 256)]:
    print(json.dumps(run(*args)), flush=True)
PY
    ;;
*)
    echo "usage: bash tools/gpu_round4.sh a|b|c|d|e|f|g|h|i|j|k" >&2
    exit 2
    ;;
esac
