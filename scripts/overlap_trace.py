"""Reads a rocprofv3 --kernel-trace CSV of scripts/overlap_probe.py and reports
whether the stand-in kernels on stream B (torch reductions or auto_range) ran
while a hot-kernel launch (chroma_kernel) was running, or only after one.

usage: python scripts/overlap_trace.py KERNEL_TRACE_CSV [OUT.txt]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    hot = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                 if "chroma_kernel" in r["Kernel_Name"])
    side = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows
                  if "at::native::reduce_kernel" in r["Kernel_Name"] or "auto_range" in r["Kernel_Name"])
    inside = after = 0
    waits, lines = [], []
    for s, e, name in side:
        # the hot launch it ran beside (overlapping in time), if any
        cont = [h for h in hot if min(e, h[1]) > max(s, h[0])]
        prev = [h for h in hot if h[1] <= s]
        if cont:
            inside += 1
            where = f"beside a hot launch ({(s - cont[0][0]) / 1e3:+.1f} us from its start, " \
                    f"{(e - s) / 1e3:.1f} us of it overlapped)"
        else:
            after += 1
            gap = (s - prev[-1][1]) / 1e3 if prev else float("nan")
            waits.append(gap)
            where = f"between hot launches ({gap:.1f} us after the last one ended)"
        lines.append(f"  {name}: {(e - s) / 1e3:.1f} us, {where}")
    hd = [(e - s) / 1e6 for s, e in hot]
    gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(hot, hot[1:])]
    out = [f"hot launches: {len(hot)}, average {sum(hd) / max(len(hd), 1):.4f} ms, "
           f"gap between them average {sum(gaps) / max(len(gaps), 1):.1f} us, max {max(gaps, default=0):.1f} us",
           f"stand-in launches: {len(side)}: {inside} ran beside a hot launch, {after} between launches"]
    text = "\n".join(out + lines[-12:])
    print(text)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
