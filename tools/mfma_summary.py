#!/usr/bin/env python3
"""Summarise a tools/pmc_mfma.sh pass: per kernel, int8 MFMA instructions, MFMA MOPs
(SQ_INSTS_VALU_MFMA_MOPS_I8 counts 512 int8 ops each, the unit of rocprofiler-sdk's derived
MFMA FLOP counters), MFMA-pipe busy cycles and the derived utilisation
MFMA_UTIL = SQ_VALU_MFMA_BUSY_CYCLES / (max-over-XCDs GRBM_GUI_ACTIVE x SIMD count)
(rocprofiler-sdk counter_defs.yaml: reduce(GRBM_GUI_ACTIVE, max)).  The CSV value of
GRBM_GUI_ACTIVE is the sum over the 8 XCD instances, so it is divided by 8 here (the
per-XCD value then matches the traced kernel time at ~2.3 GHz).  Kernel durations come from a --kernel-trace summary of the same
configuration (tools/prof_summary.py output) to turn MOPs into an achieved int8 op rate.

usage: tools/mfma_summary.py <gpurun_out/mfma_tag> <trace summary json> <out.json> <alg|mode|chunk>
Records the summary under the key in profiles/mfma_util.json, which bench.py reads.
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

SIMDS = 256 * 4
XCDS = 8
MFMA_I8_PEAK = 5.0e15


def short(name: str) -> str:
    m = re.search(r"(k_\w+)(<[^(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:60]


def main():
    d, trace, out, key = Path(sys.argv[1]), Path(sys.argv[2]), Path(sys.argv[3]), sys.argv[4]
    vals = defaultdict(lambda: defaultdict(list))
    with open(d / "m" / "run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    tr = json.loads(trace.read_text())["kernels"]
    res = {"source": str(d), "trace": str(trace), "kernels": {}}
    for k, c in vals.items():
        if not c.get("SQ_INSTS_VALU_MFMA_I8") or max(c["SQ_INSTS_VALU_MFMA_I8"]) == 0:
            continue
        n = len(c["SQ_INSTS_VALU_MFMA_I8"])
        avg = {name: sum(v) / len(v) for name, v in c.items()}
        e = {"dispatches": n, "mfma_i8_instrs_per_dispatch": avg["SQ_INSTS_VALU_MFMA_I8"],
             "mfma_mops_i8_per_dispatch": avg.get("SQ_INSTS_VALU_MFMA_MOPS_I8"),
             "mfma_busy_cycles_per_dispatch": avg.get("SQ_VALU_MFMA_BUSY_CYCLES"),
             "gui_active_cycles_per_dispatch": avg.get("GRBM_GUI_ACTIVE"),
             "valu_instrs_per_dispatch": avg.get("SQ_INSTS_VALU")}
        t = tr.get(k, {}).get("avg_ms")
        if e["mfma_busy_cycles_per_dispatch"] and e["gui_active_cycles_per_dispatch"]:
            e["mfma_util"] = e["mfma_busy_cycles_per_dispatch"] / (e["gui_active_cycles_per_dispatch"] / XCDS * SIMDS)
        t = tr.get(k, {}).get("avg_ms")
        if t and e["gui_active_cycles_per_dispatch"]:
            e["clock_GHz_from_gui_active"] = e["gui_active_cycles_per_dispatch"] / XCDS / (t * 1e-3) / 1e9
        if t and e["mfma_mops_i8_per_dispatch"]:
            ops = e["mfma_mops_i8_per_dispatch"] * 512
            e["avg_ms"] = t
            e["int8_ops_per_dispatch"] = ops
            e["achieved_Tops"] = ops / (t * 1e-3) / 1e12
            e["frac_of_int8_peak"] = ops / (t * 1e-3) / MFMA_I8_PEAK
        res["kernels"][k] = e
    out.write_text(json.dumps(res, indent=1))
    idx = Path(__file__).resolve().parents[1] / "profiles" / "mfma_util.json"
    table = json.loads(idx.read_text()) if idx.exists() else {}
    table[key] = {"source": str(out), "kernels": res["kernels"]}
    idx.write_text(json.dumps(table, indent=1, sort_keys=True))
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main()
