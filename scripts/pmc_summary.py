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
# per workload: (profiles tag, {kernel-name substring: dispatches per timed step}).  The join and
# point-polygon timed regions are the whole device step (binning included, r02); the bench's
# setup calls (count-only joins) run some of these kernels too, so per-step totals are the
# per-dispatch averages times these multiplicities, not dispatch totals over the run.
_BIN = {"bin_count<1,": 1, "bin_count<2,": 1, "bin_scatter<1,": 1, "bin_scatter<2,": 1, "bin1_offsets": 1,
        "bin2_plan": 1, "bin2_tiles<false>": 1, "bin2_tiles<true>": 1}
_PP = {**_BIN, "scan_seg_totals<unsigned int>": 1, "scan_totals<unsigned int>": 1, "scan_apply<unsigned int>": 1,
       "scan_seg_totals<unsigned long long>": 2, "scan_totals<unsigned long long>": 2,
       "scan_apply<unsigned long long>": 2, "ppoly_words": 1, "ppoly_eval": 1, "ppoly_emit": 1, "ppoly_outside": 1}
# streaming point-polygon step (r03): one pass over the window + candidate grouping + exact tests
_PS = {"ppoly_stream": 1, "ppoly_cand_refine": 1, "ppoly_cand_hist": 1, "ppoly_cand_plan": 1, "ppoly_cand_scatter": 1,
       "ppoly_cand_eval": 1}
# SQ_INSTS_VALU_FLOPS_FP64 counts per wave instruction: calibrated on synth_uniform (6 fp64
# add/mul per point in its ISA, 50M points -> 4,687,500 counted = 300M / 64), so lane FLOPs are
# the counted value times 64 (issued lanes: a divergent wave's idle lanes are included).
FP64_LANES = 64
# r04 join step: query lists, two binning passes into 16-B records, plan, one join pass
_JOIN = {"zero_step": 1, "jq_rect": 1, "jq_build<false>": 1, "jq_build<true>": 1, "jq_starts": 1, "jb_bands": 1,
         "jb_scan": 1, "jb_segs": 1, "jb_tiles": 1, "join_fused<false, true>": 1}
_PS = {**_PS, "zero_step": 1}
# (r06: the bench's set-up launches of the other kNN / range instantiations are told apart by their
# template arguments)
TAGS = {"knn": ("knn_scan", {"knn_pass<16, 0, false, false>": 1}),
        "range": ("range", {"range_set": 1}),
        "join": ("join_probe", _JOIN),
        "ppoly": ("ppoly_probe", _PS),
        "c5": ("knn_scan_c5", {"knn_pass<16, 0, true, true>": 1}),
        "ingest": ("ingest", {"ingest_fused": 1, "ingest_general": 1}),
        "ppjoin": ("ppjoin", _PS),
        "ppknn": ("ppknn", {"rsel_init": 1, "rsel_small": 1, "ppknn_scan_boxes": 1, "ppknn_dist": 1}),
        "knn_incr": ("knn_incr", {"knn_pass<16, 0, false, false>": 1, "knn_merge_panes": 1}),
        "ppoly_incr": ("ppoly_incr", _PS)}


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
    for w, (tag, mult) in TAGS.items():
        fs, ws = d / f"{w}_FETCH_SIZE_counter_collection.csv", d / f"{w}_WRITE_SIZE_counter_collection.csv"
        if not fs.exists() or not ws.exists():
            continue
        F, W = per_kernel(fs), per_kernel(ws)
        fp = d / f"{w}_SQ_INSTS_VALU_FLOPS_FP64_counter_collection.csv"
        FL = per_kernel(fp) if fp.exists() else {}
        kernels = {}
        for k in sorted(set(F) | set(W)):
            f = F.get(k, [0.0])
            wr = W.get(k, [0.0])
            kernels[k] = {"dispatches": len(f), "fetch_kb_raw_avg": sum(f) / len(f),
                          "hbm_read_bytes_avg": 2 * 1024 * sum(f) / len(f), "hbm_write_bytes_avg": 1024 * sum(wr) / len(wr)}
            if k in FL:
                kernels[k]["fp64_flops_avg"] = FP64_LANES * sum(FL[k]) / len(FL[k])

        def times(k):
            return sum(v for pat, v in mult.items() if pat in k)
        hot = {k: times(k) for k in kernels if times(k)}
        per_launch = sum((kernels[k]["hbm_read_bytes_avg"] + kernels[k]["hbm_write_bytes_avg"]) * m for k, m in hot.items())
        rec = {"workload": w, "kernels_matched": hot, "hbm_bytes_per_launch": per_launch, "kernels": kernels,
               "note": "FETCH_SIZE x 2 (gfx950 streaming-read correction) + WRITE_SIZE, KB = 1024 B; per timed step: "
                       "each matched kernel's average per dispatch times its dispatches per step (kernels_matched); "
                       "5-step bench run, one counter per rocprofv3 pass"}
        if FL:
            rec["fp64_flops_per_launch"] = sum(kernels[k].get("fp64_flops_avg", 0.0) * m for k, m in hot.items())
        (ROOT / "profiles" / f"pmc_{tag}.json").write_text(json.dumps(rec, indent=1) + "\n")
        out_all[w] = per_launch
        print(w, f"{per_launch / 1e6:.1f} MB per step", f"{rec.get('fp64_flops_per_launch', 0) / 1e9:.2f} GFLOP fp64")


if __name__ == "__main__":
    main()
