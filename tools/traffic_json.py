#!/usr/bin/env python3
"""Turn a rocprofv3 FETCH_SIZE pass (tools/pmc.sh) into profiles/<tag>_pmc_traffic.json,
which bench.py reads for `roofline.traffic`.

FETCH_SIZE is reported in KiB, and on gfx950 it counts exactly half of the
bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, "HBM [CDNA4]"):
bytes = FETCH_SIZE * 1024 * 2.

usage: tools/traffic_json.py <fetch counter_collection.csv> <out.json> [workload_bytes] [kernel]
(kernel: "scan_kernel", the default, or "read_kernel" -- the bench's bare read of
the same stream, whose ratio calibrates the scan's)

The JSON records the library's source digest (chunkfs_amd.build.source_digest)
so bench.py only quotes traffic measured on the build that is running.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chunkfs_amd import build  # noqa: E402


def main():
    src, dst = sys.argv[1], sys.argv[2]
    workload = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 30
    kern = sys.argv[4] if len(sys.argv) > 4 else "scan_kernel"
    vals, name = [], None
    for r in csv.DictReader(open(src)):
        # FastCDC's scan (cdc::p3::scan_kernel), not the walk engine's prefix scan
        k = r["Kernel_Name"]
        if r["Counter_Name"] == "FETCH_SIZE" and kern in k and (kern != "scan_kernel" or "p3::" in k):
            vals.append(float(r["Counter_Value"]))
            name = k
    if not vals:
        sys.exit(f"no {kern} FETCH_SIZE rows in " + src)
    per_launch = sum(vals) / len(vals) * 1024 * 2
    out = {
        "kernel": kern,
        "kernel_symbol": name,
        "source_digest": build.source_digest(),
        "workload_bytes": workload,
        "dispatches": len(vals),
        "fetch_size_kib_mean": sum(vals) / len(vals),
        "hbm_read_bytes_per_launch": per_launch,
        "ratio_to_algorithmic": per_launch / workload,
        "correction": "FETCH_SIZE[KiB] x 1024 x 2 (gfx950 half-count of wide streaming reads)",
        "source": src,
    }
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
