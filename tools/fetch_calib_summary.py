#!/usr/bin/env python3
"""Join tools/fetch_calib's byte counts with its rocprofv3 FETCH_SIZE / WRITE_SIZE passes:
   tools/fetch_calib_summary.py <dir with fcal_fetch/ fcal_write/ fcal_fetch.out> > calibration.json
FETCH_SIZE / WRITE_SIZE are in KiB; the ratio counter bytes / known bytes per access pattern is
the calibration (MI355X_MICROARCH.md: 0.5 for a 16 B/lane coalesced read on gfx950)."""
import collections
import csv
import json
import sys
from pathlib import Path


def load(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "rocclr" in r["Kernel_Name"]:
            continue  # the probe's hipMemset fills
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        agg[k] = agg.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    return list(agg.items())


d = Path(sys.argv[1])
fetch = load(d / "fcal_fetch" / "run_counter_collection.csv")
write = load(d / "fcal_write" / "run_counter_collection.csv")
known = [json.loads(x) for x in open(d / "fcal_fetch.out")]
out = {"source": str(d), "units": "bytes (FETCH_SIZE / WRITE_SIZE KiB x 1024)", "patterns": {}}
for ((_, kname), fb), (_, wb), kn in zip(fetch, write, known):
    b = kn.get("read_bytes") or kn.get("write_bytes")
    out["patterns"][kn["kernel"]] = {"kernel": kname, "known_bytes": b, "fetch_bytes": fb, "write_bytes": wb,
                                     "fetch_over_known": round(fb / b, 4), "write_over_known": round(wb / b, 4)}
json.dump(out, sys.stdout, indent=1)
print()
