"""Where C5's co-resident block spends its time (`bash tools/gpu_round5.sh m`): from rocprofv3's memory-copy trace,
the last fmi_comm_allreduce_host call of the 8 LOCAL ranks (8 GiB each way in chunk copies on the device's shared
copy streams). Reports the call's span, how long each direction's engine was busy
(union of its copies), the rate of one copy, the stretch before the first D2H (fill) and after the last H2D (drain),
and the idle gaps inside each direction. Prints one JSON object.

  python tools/c5_trace_summary.py gpurun_out/r05_c5_trace/run_memory_copy_trace.csv [copies per direction per call:
      8 ranks x chunks per bucket, 128 for 1 GiB in 64 MiB chunks; 144 with the co-resident c/8, c/4, c/2 start]
"""
import csv
import json
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main(path: str, per_dir: int) -> None:
    rows = [r for r in csv.DictReader(open(path))]
    copies = [(r["Direction"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    big = sorted((c for c in copies if c[2] - c[1] > 50_000), key=lambda c: c[1])  # chunk copies (>= 4 MiB)
    # the last call: its `per_dir` chunk copies of each direction (8 ranks x chunks per bucket)
    h2d_all = [c for c in big if c[0].endswith("HOST_TO_DEVICE")][-per_dir:]
    d2h_all = [c for c in big if c[0].endswith("DEVICE_TO_HOST")][-per_dir:]
    last = h2d_all + d2h_all
    h2d = [(a, b) for d, a, b in last if d.endswith("HOST_TO_DEVICE")]
    d2h = [(a, b) for d, a, b in last if d.endswith("DEVICE_TO_HOST")]
    t0 = min(a for _, a, _ in last)
    t1 = max(b for _, _, b in last)
    uh, ud = union(h2d), union(d2h)
    busy_h = sum(b - a for a, b in uh)
    busy_d = sum(b - a for a, b in ud)
    gaps_h = [b[0] - a[1] for a, b in zip(uh, uh[1:])]
    gaps_d = [b[0] - a[1] for a, b in zip(ud, ud[1:])]
    dur_h = sorted(b - a for a, b in h2d)
    dur_d = sorted(b - a for a, b in d2h)
    ms = 1e-6
    out = {
        "source": path, "copies_in_call": {"h2d": len(h2d), "d2h": len(d2h)},
        "call_span_ms": round((t1 - t0) * ms, 2),
        "h2d_busy_ms": round(busy_h * ms, 2), "d2h_busy_ms": round(busy_d * ms, 2),
        "h2d_copy_median_ms": round(dur_h[len(dur_h) // 2] * ms, 3), "d2h_copy_median_ms": round(dur_d[len(dur_d) // 2] * ms, 3),
        "h2d_GB_s_while_busy": round(8 * (1 << 30) / (busy_h * 1e-9) / 1e9, 1),
        "d2h_GB_s_while_busy": round(8 * (1 << 30) / (busy_d * 1e-9) / 1e9, 1),
        "fill_ms_before_first_d2h": round((min(a for a, _ in d2h) - t0) * ms, 2),
        "drain_ms_after_last_h2d": round((t1 - max(b for _, b in h2d)) * ms, 2),
        "h2d_idle_gaps_ms": round(sum(gaps_h) * ms, 2), "d2h_idle_gaps_ms": round(sum(gaps_d) * ms, 2),
        "h2d_largest_gaps_ms": [round(g * ms, 2) for g in sorted(gaps_h)[-3:]],
        "d2h_largest_gaps_ms": [round(g * ms, 2) for g in sorted(gaps_d)[-3:]],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 128)
