"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc.sh output).

Correction (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half
the bytes of wide (16 B/lane) coalesced streaming reads, so reads are doubled; WRITE_SIZE is exact
for 16 B/lane streaming stores. Both counters are in KiB per dispatch; Infinity-Cache hits are
counted as fabric requests. Gathers (4 B/lane) are uncalibrated -- the doubled figure is reported
as an upper bound. Usage: python tools/pmc_traffic.py gpurun_out/pmc_run out.json [workload tag]
The workload tag (bench.py --print-workload with the same arguments as the profiled bench) keys the
file for bench.py's roofline.traffic lookup.
"""
import csv
import collections
import glob
import json
import os
import sys

KERNELS = {"k_fused_train_grid": "k_fused_train_grid", "k_grid_bwd_lds": "k_grid_bwd_lds", "k_adam": "k_adam",
           "k_mlp_tile_train": "k_mlp_tile_train", "k_mlp_tile_infer": "k_mlp_tile_infer", "k_grid_fwd": "k_grid_fwd",
           "k_grid_bin": "k_grid_bin", "k_grid_acc": "k_grid_acc"}


def load(run_dir):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(run_dir, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for key, short in KERNELS.items():
                if key in r["Kernel_Name"]:
                    vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    run_dir, out = sys.argv[1], sys.argv[2]
    vals = load(run_dir)
    res = {}
    for k, d in vals.items():
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        fetch = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024.0
        write = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024.0
        res[k] = {"fetch_bytes_raw": fetch, "write_bytes": write, "hbm_bytes": 2.0 * fetch + write,
                  "dispatches": len(d["FETCH_SIZE"])}
        for c in ("TCC_HIT_sum", "TCC_MISS_sum"):
            if c in d:
                res[k][c] = sum(d[c]) / len(d[c])
    doc = {"correction": "reads x2 (gfx950 FETCH_SIZE = half of 16B-streaming bytes), writes as counted", "kernels": res}
    if len(sys.argv) > 3:
        doc["workload"] = sys.argv[3]
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
