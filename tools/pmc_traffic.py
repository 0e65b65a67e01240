#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc.sh) per kernel: average counter value per dispatch and
the HBM traffic per launch, corrected for gfx950 as MI355X_MICROARCH.md §HBM prescribes
(FETCH_SIZE counts half the bytes of wide coalesced streaming reads -> x2; WRITE_SIZE exact; KB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for key in ("k_fused_np", "k_fused_fast", "k_fused", "k_scan0", "k_sample_hist", "k_hist_tau", "k_scan", "k_seg_prepare", "k_refine", "k_merge", "k_chunk_np", "k_chunk", "k_precomp",
                "k_progressive_final", "k_rescore", "k_level_scores", "k_cos_glds", "k_cos_g3", "k_cos_t", "k_cos_mfma", "k_cos_prepare"):
        if key in name:
            if key == "k_fused_fast":
                return "k_fused" + name.split("k_fused_fast<")[1].split(",")[0]
            if key == "k_chunk_np":
                return "k_chunk_np" + name.split("k_chunk_np<")[1].split(",")[0]
            if key == "k_fused_np":
                return "k_fused_np" + name.split("k_fused_np<")[1].split(",")[0]
            return key
    return None


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            if k:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        rec = {"counters_avg_per_dispatch": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            rec["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
            rec["raw_fetch_write_kb"] = [avg["FETCH_SIZE"], avg["WRITE_SIZE"]]
        out[k] = rec
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
