"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs of
tools/gae_kernel_bench.py) into profiles/<name>.json: per-dispatch HBM bytes of the GAE row
kernel, with the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md §HBM (128-B read
requests tallied at 64 B: the read count is doubled), next to the algorithmic 26 B/transition.

    python tools/pmc_gae.py gpurun_out/pmc_f/run_counter_collection.csv \
        gpurun_out/pmc_w/run_counter_collection.csv profiles/r01_gae_pmc.json
"""
import csv
import json
import sys

KERNEL = "gae_rows_staged_kernel"
N = 4096 * 2048


def collect(path, counter):
    rows = [r for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    vals = [float(r["Counter_Value"]) for r in rows]
    r0 = rows[0]
    return {"dispatches": len(vals), "mean_kb": sum(vals) / len(vals), "min_kb": min(vals),
            "max_kb": max(vals), "vgpr": r0["VGPR_Count"], "agpr": r0["Accum_VGPR_Count"],
            "sgpr": r0["SGPR_Count"], "lds": r0["LDS_Block_Size"], "grid": r0["Grid_Size"],
            "wg": r0["Workgroup_Size"]}


def main(fetch_csv, write_csv, out):
    f = collect(fetch_csv, "FETCH_SIZE")
    w = collect(write_csv, "WRITE_SIZE")
    rd = 2.0 * f["mean_kb"] * 1024
    wr = w["mean_kb"] * 1024
    res = {"FETCH_SIZE": f, "WRITE_SIZE": w, "derived": {
        "kernel": f"{KERNEL}<true> (rew_norm f64 path, 4096 envs x 2048 steps)",
        "read_bytes_corrected": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
        "algorithmic_read": 18 * N, "algorithmic_write": 8 * N, "algorithmic_total": 26 * N,
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B "
                "requests at 64 B); counters from separate rocprofv3 --pmc passes over "
                f"{f['dispatches']} launches of tools/gae_kernel_bench.py"}}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["derived"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
