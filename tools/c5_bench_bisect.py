"""Bisect bench.py's N > 1 C5 figure (~39 ms at world size 1, against 23.5 ms for the same calls in
tools/c5_in_bench_probe.py on the same box): runs bench.py's own main() with CommAllreduce's methods wrapped
so that a 1 GiB host_bench is timed after every call bench.py makes, printed to stderr as JSON.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
        --master-port 29617 tools/c5_bench_bisect.py --force-dist --steps 20 --warmup 3 --no-diagnostics
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MIB = 1 << 20


def main():
    import bench
    from fmi_amd import collectives as col

    host = col.CommAllreduce.host_bench
    n5 = 1024 * MIB // 4
    seen = {}

    def wrap(name):
        orig = getattr(col.CommAllreduce, name)

        def f(self, *a, **k):
            r = orig(self, *a, **k)
            seen[name] = seen.get(name, 0) + 1
            ms = host(self, n5)["ms"]
            print(json.dumps({f"after_{name}_{seen[name]}": ms}), file=sys.stderr, flush=True)
            return r

        setattr(col.CommAllreduce, name, f)

    orig_init = col.CommAllreduce.__init__

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        print(json.dumps({"after_init": host(self, n5)["ms"]}), file=sys.stderr, flush=True)

    col.CommAllreduce.__init__ = init
    for name in ("bench", "self_check", "shard_kernel"):
        wrap(name)
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()


if __name__ == "__main__":
    main()
