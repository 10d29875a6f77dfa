"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh output) per kernel.

python scripts/pmc_summary.py PMC_DIR [--match predict_ring] [--out profiles/x.json]

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced streaming read (16 B/lane, global_load / LDS-DMA alike), so it
is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Our fused kernel's
stores are 2 B/lane coalesced rows, which the guide lists as uncalibrated: the
write figure is reported raw next to the algorithmic write bytes.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(pmc_dir):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--algorithmic-read", type=float, default=None)
    ap.add_argument("--algorithmic-write", type=float, default=None)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    per = load(args.pmc_dir)
    out = {}
    for k, cs in per.items():
        if args.match and args.match not in k:
            continue
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["launches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_per_launch"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes_per_launch"] = d["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_per_launch"] + d["hbm_write_bytes_per_launch"]
        out[k] = d
    res = {"source": args.pmc_dir, "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 wide-read half count); "
                                                  "WRITE_SIZE KiB x1024", "kernels": out}
    if len(out) == 1:  # one kernel: its per-launch HBM figures at the top (bench.py reads them)
        (k, d), = out.items()
        res["kernel"] = k
        for f in ("hbm_read_bytes_per_launch", "hbm_write_bytes_per_launch", "hbm_bytes_per_launch"):
            if f in d:
                res[f] = d[f]
    if args.algorithmic_read is not None:
        res["algorithmic_read_bytes"] = args.algorithmic_read
    if args.algorithmic_write is not None:
        res["algorithmic_write_bytes"] = args.algorithmic_write
    s = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
