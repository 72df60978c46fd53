"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs of
tools/gae_kernel_bench.py) into profiles/<name>.json: per-dispatch HBM bytes of the GAE row
kernel, with the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md §HBM (128-B read
requests tallied at 64 B: the read count is doubled), next to the algorithmic 26 B/transition.

    python tools/pmc_gae.py gpurun_out/pmc_f/run_counter_collection.csv \
        gpurun_out/pmc_w/run_counter_collection.csv profiles/r01_gae_pmc.json
    python tools/pmc_gae.py --db gpurun_out/pmc_gf/run_results.db \
        gpurun_out/pmc_gw/run_results.db profiles/r05_gae_pmc.json

(the second form reads rocprofv3's rocpd databases, the default output since round 4).  The
record names the sha256 of csrc/gae.hip as it is when this runs (on the box: the source the
measured library was built from), which bench.py matches before it reports roofline.traffic.
"""
import csv
import hashlib
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join("tianshou-fork_amd", "csrc", "gae.hip")

KERNEL = os.environ.get("GAE_KERNEL", "gae_rows_staged_kernel")
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


def collect_db(path, counter):
    c = sqlite3.connect(path)
    rows = [(v, disp) for name, cn, v, disp in c.execute(
        "select kernel_name, counter_name, value, dispatch_id from counters_collection")
        if KERNEL in name and cn == counter]
    vals = [float(v) for v, _ in rows]
    return {"dispatches": len(vals), "mean_kb": sum(vals) / len(vals), "min_kb": min(vals),
            "max_kb": max(vals)}


def main(fetch_csv, write_csv, out, db=False):
    f = (collect_db if db else collect)(fetch_csv, "FETCH_SIZE")
    w = (collect_db if db else collect)(write_csv, "WRITE_SIZE")
    rd = 2.0 * f["mean_kb"] * 1024
    wr = w["mean_kb"] * 1024
    res = {"FETCH_SIZE": f, "WRITE_SIZE": w, "derived": {
        "kernel": f"{KERNEL}<true> (rew_norm f64 path, 4096 envs x 2048 steps)",
        "read_bytes_corrected": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
        "algorithmic_read": 18 * N, "algorithmic_write": 8 * N, "algorithmic_total": 26 * N,
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B "
                "requests at 64 B); counters from separate rocprofv3 --pmc passes over "
                f"{f['dispatches']} launches of tools/gae_kernel_bench.py",
        "source": SRC.replace(os.sep, "/")}}
    with open(os.path.join(ROOT, SRC), "rb") as fh:
        res["derived"]["source_sha256"] = hashlib.sha256(fh.read()).hexdigest()
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["derived"], indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--db":
        main(*sys.argv[2:5], db=True)
    else:
        main(*sys.argv[1:4])
