"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs of
tools/atari_trunk_bench.py --only) into a JSON summary of the HBM bytes per dispatch of
frames_nhwc4_kernel (tsrl_frames_to_f32_nhwc), per launch shape, with the gfx950 FETCH_SIZE
correction of MI355X_MICROARCH.md §HBM (read count doubled), next to the algorithmic
28 224 B read + 112 896 B written per 4x84x84 frame stack.

    python tools/pmc_frames.py <fetch counter_collection.csv> <write ...csv> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict

KERNEL = "frames_nhwc4_kernel"
HW4 = 84 * 84 // 4  # threads per frame-stack row
RD, WR = 4 * 84 * 84, 4 * 4 * 84 * 84


def collect(path, counter):
    by = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            by[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    return by


def main(fetch_csv, write_csv, out):
    f, w = collect(fetch_csv, "FETCH_SIZE"), collect(write_csv, "WRITE_SIZE")
    res = {}
    for grid in sorted(set(f) & set(w)):
        rows = grid // HW4
        rd = 2.0 * sum(f[grid]) / len(f[grid]) * 1024
        wr = sum(w[grid]) / len(w[grid]) * 1024
        res[f"{rows}_rows"] = {
            "dispatches": [len(f[grid]), len(w[grid])], "grid": grid,
            "read_bytes_corrected": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
            "algorithmic_read": RD * rows, "algorithmic_write": WR * rows,
            "algorithmic_total": (RD + WR) * rows,
            "traffic_over_algorithmic": (rd + wr) / ((RD + WR) * rows)}
    res["note"] = ("FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM; counters from separate "
                   "rocprofv3 --pmc passes over tools/atari_trunk_bench.py --only")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
