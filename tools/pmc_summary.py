#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter-collection CSVs (one pass per counter set).

Usage: pmc_summary.py OUT.json DIR_OR_CSV...
For every kernel of interest: mean of each counter per dispatch, the mean grid size
(= signatures per dispatch: one lane per signature), and HBM traffic per dispatch and per
signature, corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes for gfx950:
FETCH_SIZE (KB) reports half the bytes of wide coalesced reads -> x2; WRITE_SIZE (KB) is exact
for 16-B stores.  bench.py reads the result (profiles/pmc_summary.json) for roofline.traffic."""
import collections
import csv
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tendermint-fork_amd"))
from tmed.srcdigest import kernel_src_digest  # noqa: E402

KERNELS = ("verify_main_hs_kernel", "verify_prep_r_kernel", "verify_main_kernel", "verify_prep_kernel", "verify_finish_kernel",
           "verify_keyset_main_kernel", "verify_keyset_prep_kernel", "verify_keyset_lat_kernel", "verify_lat_finish_kernel",
           "verify_glat_prep_kernel", "verify_glat_main_kernel", "sign_kernel", "merkle", "sha256", "valu_probe")


def files(args):
    for a in args:
        if os.path.isdir(a):
            yield from glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True)
        else:
            yield a


def short(name):
    for k in KERNELS:
        if k in name:
            if k == "verify_main_kernel" and "<" in name:
                return k + name[name.index("<"):name.index(">") + 1]
            return k
    return None


def main():
    out_path, srcs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = collections.defaultdict(list)
    for f in files(srcs):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[k].append(int(r["Grid_Size"]))
    # dispatch durations from the kernel traces of the same runs (effective clock)
    dur = collections.defaultdict(list)
    for a in srcs:
        for f in (glob.glob(os.path.join(a, "**", "*kernel_trace.csv"), recursive=True) if os.path.isdir(a) else []):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if k:
                    dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for k, cs in acc.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        d["grid_mean"] = sum(grid[k]) / len(grid[k])
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            fb = d["FETCH_SIZE"] * 1024 * 2   # gfx950: FETCH_SIZE counts half of wide reads
            wb = d["WRITE_SIZE"] * 1024
            d["hbm_bytes_per_dispatch"] = fb + wb
            d["hbm_read_bytes_per_sig"] = fb / d["grid_mean"]
            d["hbm_write_bytes_per_sig"] = wb / d["grid_mean"]
            d["hbm_bytes_per_sig"] = (fb + wb) / d["grid_mean"]
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
            d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        if dur[k]:
            d["dispatch_ms_mean"] = sum(dur[k]) / len(dur[k]) / 1e6
            if "GRBM_GUI_ACTIVE" in d:  # GUI-active cycles summed over the 8 XCDs
                d["effective_clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8 / (d["dispatch_ms_mean"] * 1e6)
        if "SQ_WAVE_CYCLES" in d and "SQ_ACTIVE_INST_ANY" in d:  # the wave-state partition
            wc = d["SQ_WAVE_CYCLES"]
            d["active_inst_any_frac"] = d["SQ_ACTIVE_INST_ANY"] / wc
            d["wait_inst_any_frac"] = d.get("SQ_WAIT_INST_ANY", 0) / wc
            d["wait_any_frac"] = d.get("SQ_WAIT_ANY", 0) / wc
            d["valu_active_frac"] = d.get("SQ_ACTIVE_INST_VALU", 0) / wc
        res[k] = d
    # the kernel sources these counters belong to: bench.py leaves the summary out once they change
    res["_meta"] = {"kernel_src_sha16": kernel_src_digest(), "collected": time.strftime("%Y-%m-%d %H:%M:%S UTC", time.gmtime())}
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, d in res.items():
        if k == "_meta":
            continue
        print(k, {x: round(d[x], 3) for x in ("hbm_bytes_per_sig", "valu_insts_per_wave", "dispatch_ms_mean",
                                              "effective_clock_ghz", "active_inst_any_frac", "wait_inst_any_frac",
                                              "wait_any_frac") if x in d})


if __name__ == "__main__":
    main()
