#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into one JSON: per-kernel average duration from the
rocprofv3 --kernel-trace --stats pass, and per-dispatch HBM traffic from the separate
FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md "HBM"), so reads are doubled
("fetch_bytes_corrected"); WRITE_SIZE is taken as is.

usage: tools/prof_summary.py <gpurun_out/prof_tag> <out.json> [<alg|mode|chunk> key]
With a key, the per-dispatch HBM bytes are also recorded in profiles/pmc_traffic.json, which
bench.py reads to fill roofline.traffic for the same configuration.
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


# ML-KEM role kernels (mlkem.hip k_multi / k_role; k_pair / k_tri in older builds): the rocprof name
# carries the role types; the library's own launch names (QRK_LAUNCH, bench.py's kernel tables)
# join the roles with '+'
ROLES = {"RFrontEnc": "k_front_encaps", "RPrf": "k_prf", "RDecrypt": "k_decrypt_core", "RJDec": "k_j_decaps",
         "RGDec": "k_g_decaps", "RCore": "k_encrypt_core"}


def role_name(t: str) -> str:
    t = t.strip().replace("qrk::mlkem::", "")
    m = re.match(r"RXof<\d+, (true|false)>", t)
    if m:
        return "k_xof_fix" if m.group(1) == "true" else "k_xof"
    for k, v in ROLES.items():
        if t.startswith(k):
            return v
    return t


def short(name: str) -> str:
    m = re.search(r"(k_multi|k_pair|k_tri|k_role)<(.*)>\(", name)
    if m:
        args, depth, cur = [], 0, ""
        for ch in m.group(2):
            if ch == "," and depth == 0:
                args.append(cur)
                cur = ""
                continue
            depth += ch == "<"
            depth -= ch == ">"
            cur += ch
        args.append(cur)
        return "+".join(role_name(a) for a in args)
    m = re.search(r"(k_\w+)(<[^(]*>)?\(", name)
    if not m:
        return name.split("(")[0][:60]
    return m.group(1) + (m.group(2) or "")


def main():
    d, out = Path(sys.argv[1]), Path(sys.argv[2])
    res = {"source": str(d), "kernels": {}}
    with open(d / "trace" / "run_kernel_stats.csv") as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            res["kernels"][k] = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) / 1e6,
                                 "total_ms": float(row["TotalDurationNs"]) / 1e6,
                                 "percent": float(row["Percentage"])}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        acc = defaultdict(list)
        p = d / sub / "run_counter_collection.csv"
        if not p.exists():
            continue
        with open(p) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter:
                    acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)
        for k, v in acc.items():
            e = res["kernels"].setdefault(k, {})
            key = "fetch_bytes" if counter == "FETCH_SIZE" else "write_bytes"
            e[key + "_per_dispatch"] = sum(v) / len(v)
            e[key + "_dispatches"] = len(v)
    for k, e in res["kernels"].items():
        if "fetch_bytes_per_dispatch" in e:
            e["fetch_bytes_corrected_per_dispatch"] = 2 * e["fetch_bytes_per_dispatch"]
            e["hbm_bytes_per_dispatch"] = e["fetch_bytes_corrected_per_dispatch"] + e.get("write_bytes_per_dispatch", 0.0)
    out.write_text(json.dumps(res, indent=1))
    if len(sys.argv) > 3:
        idx = Path(__file__).resolve().parents[1] / "profiles" / "pmc_traffic.json"
        table = json.loads(idx.read_text()) if idx.exists() else {}
        table[sys.argv[3]] = {"source": str(out.relative_to(idx.parent.parent)) if out.is_absolute() else str(out),
                              "hbm_bytes_per_dispatch": {k: e["hbm_bytes_per_dispatch"] for k, e in res["kernels"].items()
                                                         if "hbm_bytes_per_dispatch" in e}}
        idx.write_text(json.dumps(table, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
