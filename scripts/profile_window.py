"""Per-dispatch view of a rocprofv3 kernel trace: the durations of one kernel's
dispatches in order, and their mean over a dispatch window -- by default
6..25, the 20 timed launches after bench.py's 5 warm-up launches (the
driver's `--warmup 5 --steps 20` protocol), which is the window the bench
line's `roofline.kernel_ms` averages.

  python scripts/profile_window.py <kernel_trace.csv> [name-substring] [first last] [bytes_per_launch]

Prints one JSON line: the window's mean / min / max (ms), the mean over all
dispatches, and GB/s + fraction of 8 TB/s when bytes_per_launch is given."""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "decim_stream_cf32"
    first, last = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (6, 25)
    nbytes = float(sys.argv[5]) if len(sys.argv) > 5 else 10.0 * (1 << 28)
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r.get("Kernel_Name", ""):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    ms = [d / 1e6 for _, d in rows]
    win = ms[first - 1:last]
    out = {"trace": path, "kernel_substring": name, "dispatches": len(ms), "window": [first, last],
           "window_mean_ms": round(sum(win) / len(win), 4) if win else None,
           "window_min_ms": round(min(win), 4) if win else None, "window_max_ms": round(max(win), 4) if win else None,
           "all_mean_ms": round(sum(ms) / len(ms), 4) if ms else None,
           "per_dispatch_ms": [round(v, 4) for v in ms]}
    if win:
        gbs = nbytes / (out["window_mean_ms"] * 1e-3) / 1e9
        out.update(window_gbs=round(gbs, 1), window_frac_of_8tbs=round(gbs / 8000.0, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
