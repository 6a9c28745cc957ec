"""Summarise rocprofv3 --pmc passes (scripts/pmc_session.sh) for one kernel.

usage: python scripts/pmc_summary.py PMC_DIR KERNEL_SUBSTRING BYTES_PER_LAUNCH [OUT.json]

Averages every counter over the kernel's dispatches, then derives
  hbm_read_bytes_per_launch = FETCH_SIZE[KB] * 1024 * 2
(MI355X_MICROARCH.md, HBM section: on gfx950 FETCH_SIZE reports exactly half
the bytes of a wide coalesced streaming read, so it is doubled).  Calibrated
on a known byte count in the chroma kernel's own access pattern
(scripts/ubench/fetch_calib.hip calib_rows, profiles/r05/fetch_calib/): the
doubled figure is 1.0000 x the bytes read there (a lane-interleaved pattern,
two 16-B loads per 32-B lane chunk, reads 1.024 x: some of its requests are
64-B halves), so for this kernel the doubled figure is the traffic.
BYTES_PER_LAUNCH is the algorithmic input bytes of one launch (2 B/pixel),
written alongside so bench.py only uses the traffic figure for the same size.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    pmc_dir, kern, alg = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else None
    vals = collections.defaultdict(list)
    names = set()
    for path in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kern not in row["Kernel_Name"]:
                    continue
                names.add(row["Kernel_Name"])
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not vals:
        sys.exit(f"no dispatches of {kern!r} under {pmc_dir}")
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import source_digest  # the sources these passes ran (bench.py checks it)

    res = {"kernel": sorted(names)[0], "dispatches_per_counter": {k: len(v) for k, v in vals.items()},
           "counters_avg_per_launch": {k: round(v, 1) for k, v in sorted(avg.items())},
           "bytes_per_launch_algorithmic": alg, "source_digest": source_digest(),
           "measured": f"rocprofv3 --pmc, one counter group per run, {os.path.basename(os.path.normpath(pmc_dir))}"}
    if "FETCH_SIZE" in avg:
        hbm = avg["FETCH_SIZE"] * 1024 * 2
        res["hbm_read_bytes_per_launch"] = int(hbm)
        res["hbm_read_over_algorithmic"] = round(hbm / alg, 4)
        res["correction"] = ("FETCH_SIZE(KB)*1024*2 (gfx950 reports half of 16-B/lane streaming reads; 1.0000 x "
                             "the known bytes of a stream in the chroma kernel's own pattern, "
                             "profiles/r05/fetch_calib/)")
    px = alg / 2
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        res["valu_instr_per_pixel_per_lane"] = round(avg["SQ_INSTS_VALU"] * 64 / px, 2)
    if "SQ_INSTS_SALU" in avg and "SQ_WAVES" in avg:
        res["salu_instr_per_pixel_per_lane"] = round(avg["SQ_INSTS_SALU"] * 64 / px, 2)
    if "SQ_WAVE_CYCLES" in avg and "SQ_WAVES" in avg:
        res["waves"] = avg["SQ_WAVES"]
    if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
        res["lds_bank_conflict_frac"] = round(avg["SQ_LDS_BANK_CONFLICT"] / max(avg["SQ_LDS_IDX_ACTIVE"], 1), 4)
    text = json.dumps(res, indent=1)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
