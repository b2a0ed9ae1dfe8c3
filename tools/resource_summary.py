#!/usr/bin/env python3
"""Table of per-kernel register / scratch / occupancy figures from `make isa`'s
-Rpass-analysis=kernel-resource-usage output (tendermint-fork_amd/lib/resource_usage.txt)."""
import re
import subprocess
import sys


def parse(path):
    rows, cur = [], None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: [^ ]+ +(\S[^:]*): (\S+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return [o.split("(")[0] for o in out[:len(names)]]
    except OSError:
        return names


def main():
    rows = parse(sys.argv[1] if len(sys.argv) > 1 else "tendermint-fork_amd/lib/resource_usage.txt")
    names = demangle([r["kernel"] for r in rows])
    print("%-44s %5s %5s %6s %6s %8s %5s %6s" % ("kernel", "VGPR", "AGPR", "vspill", "sspill", "scratch", "occ", "LDS"))
    for n, r in zip(names, rows):
        print("%-44s %5s %5s %6s %6s %8s %5s %6s" % (n[-44:], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"),
                                                     r.get("SGPRs Spill"), r.get("ScratchSize [bytes/lane]"),
                                                     r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))


if __name__ == "__main__":
    main()
