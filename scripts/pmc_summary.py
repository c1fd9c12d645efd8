"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, KB per dispatch) per kernel and write
profiles/pmc_<tag>.json for bench.py's roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports 1/2 of the bytes of a wide
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
Counters are KB (1024 B).  Warm-up dispatches are included (same shape as timed ones).

    python scripts/pmc_summary.py gpurun_out/pmc knn:knn_scan range:range_ ... --round r01
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
# workload -> (profiles tag, kernel-name substrings of the bench's timed region, timed launches per step)
TAGS = {"knn": ("knn_scan", ("knn_pass",), 1),
        "range": ("range", ("range_fused", "range_scan", "scan_units", "range_emit"), 1),
        "join": ("join_probe", ("join_tile", "join_emit", "scan_seg_totals<unsigned long long>", "scan_totals<unsigned long long>",
                                 "scan_apply<unsigned long long>"), 1),
        "ppoly": ("ppoly_probe", ("ppoly_eval", "ppoly_emit", "ppoly_outside"), 1),
        "c5": ("knn_scan_c5", ("knn_pass",), 1),
        "ingest": ("ingest", ("ingest_count", "ingest_scan", "ingest_parse"), 1),
        "ppjoin": ("ppjoin", ("ppoly_eval", "ppoly_emit", "ppoly_outside"), 1),
        "ppknn": ("ppknn", ("rsel_", "ppknn_"), 1),
        "knn_incr": ("knn_incr", ("knn_pass", "knn_final"), 1),
        "ppoly_incr": ("ppoly_incr", ("ppoly_eval", "ppoly_emit", "ppoly_outside"), 1)}


def per_kernel(path):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            acc[name].append(float(row["Counter_Value"]))
    return acc


def main():
    d = Path(sys.argv[1])
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
    out_all = {}
    for w, (tag, match, per_step) in TAGS.items():
        fs, ws = d / f"{w}_FETCH_SIZE_counter_collection.csv", d / f"{w}_WRITE_SIZE_counter_collection.csv"
        if not fs.exists() or not ws.exists():
            continue
        F, W = per_kernel(fs), per_kernel(ws)
        kernels = {}
        for k in sorted(set(F) | set(W)):
            f = F.get(k, [0.0])
            wr = W.get(k, [0.0])
            kernels[k] = {"dispatches": len(f), "fetch_kb_raw_avg": sum(f) / len(f),
                          "hbm_read_bytes_avg": 2 * 1024 * sum(f) / len(f), "hbm_write_bytes_avg": 1024 * sum(wr) / len(wr)}
        hot = [k for k in kernels if any(m in k for m in match)]
        per_launch = sum(kernels[k]["hbm_read_bytes_avg"] + kernels[k]["hbm_write_bytes_avg"] for k in hot) / per_step
        rec = {"workload": w, "kernels_matched": hot, "hbm_bytes_per_launch": per_launch, "kernels": kernels,
               "note": "FETCH_SIZE x 2 (gfx950 streaming-read correction) + WRITE_SIZE, KB = 1024 B; "
                       "per timed launch: the matched kernels' average bytes per dispatch summed over one step "
                       "(each runs once per step) / timed launches per step; 5-step bench run"}
        (ROOT / "profiles" / f"pmc_{tag}.json").write_text(json.dumps(rec, indent=1) + "\n")
        out_all[w] = per_launch
        print(w, hot, f"{per_launch / 1e6:.1f} MB per launch")


if __name__ == "__main__":
    main()
