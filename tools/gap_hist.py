"""Per-kernel duration and launch-to-launch gap histogram from a rocprofv3
kernel_trace.csv (the window / chain sequence of a timed step).
usage: python tools/gap_hist.py <run_kernel_trace.csv> [kernel substring]"""
import csv
import sys
from collections import Counter


def main(path, sub=None):
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if sub is None or sub in r["Kernel_Name"]]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
    # idle time between the end of one dispatch and the start of the next (any kernel)
    idle = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
    period = [(int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
    def hist(v, w):
        c = Counter(int(x // w) * w for x in v)
        return {f"{k:.1f}-{k + w:.1f}": n for k, n in sorted(c.items())}
    n = len(dur)
    print(f"{sub or 'all'}: {n} dispatches, duration avg {sum(dur) / max(n, 1):.2f} us, "
          f"start-to-start avg {sum(period) / max(len(period), 1):.2f} us")
    print("duration us:", hist(dur, 2.0))
    print("idle between dispatches us:", hist([x for x in idle if x < 100], 0.5))
    print("start-to-start us:", hist([x for x in period if x < 200], 2.0))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
