"""Per-launch durations of one kernel from a rocprofv3 kernel trace (run_kernel_trace.csv).

The bench's HIP-event `kernel_avg_ms` covers the timed launches only (K/S launches of S
sweeps); rocprofv3's --stats average also includes the shorter warm-up launch.  This prints
every launch so the two can be compared launch for launch.

    python tools/launch_stats.py gpurun_out/prof/run_kernel_trace.csv k_sweep_freespec
"""
import csv
import sys


def main(path, pattern):
    rows = list(csv.DictReader(open(path)))
    name_key = next(k for k in rows[0] if k.lower() in ("kernel_name", "name"))
    t0 = next(k for k in rows[0] if k.lower().startswith("start_timestamp"))
    t1 = next(k for k in rows[0] if k.lower().startswith("end_timestamp"))
    d = [(int(r[t1]) - int(r[t0])) / 1e6 for r in rows if pattern in r[name_key]]
    if not d:
        print(f"no launches of {pattern}")
        return
    print(f"{pattern}: {len(d)} launches, ms: " + " ".join(f"{x:.3f}" for x in d))
    tail = d[1:] if len(d) > 1 else d
    print(f"mean all {sum(d) / len(d):.3f} ms; mean excluding the first (warm-up) launch "
          f"{sum(tail) / len(tail):.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
