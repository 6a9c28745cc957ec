"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV, in
launch order, and the average over the last K launches (bench.py's timed
steps are the command's last launches of the hot kernel).

usage: python scripts/trace_timed.py KERNEL_TRACE_CSV KERNEL_SUBSTRING K [OUT.txt]
"""
import csv
import sys


def main():
    path, kern, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows[-k:], rows[-k + 1:])]
    lines = [f"{kern}: {len(d)} launches in the trace",
             f"last {k} (the timed steps): average {sum(d[-k:]) / k:.4f} ms, min {min(d[-k:]):.4f}, max {max(d[-k:]):.4f}; "
             f"gap between them {sum(gaps) / max(len(gaps), 1):.1f} us",
             f"all launches: average {sum(d) / len(d):.4f} ms",
             "durations in launch order (ms): " + " ".join(f"{x:.3f}" for x in d)]
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
