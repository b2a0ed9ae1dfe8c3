"""Digest of the device-code sources (csrc/kernels.hip and every csrc/*.h header): the tag that ties
an archived rocprofv3 PMC summary (profiles/pmc_summary.json, tools/pmc_summary.py) to the kernels
it was collected on, so bench.py can leave out figures from an older build."""
from __future__ import annotations

import glob
import hashlib
import os

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def kernel_src_digest(csrc: str = CSRC) -> str:
    h = hashlib.sha256()
    for p in [os.path.join(csrc, "kernels.hip")] + sorted(glob.glob(os.path.join(csrc, "*.h"))):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
