#!/usr/bin/env python3
"""Per-kernel SQ counter summary from tools/pmc_sq.sh output: tools/sq_summary.py gpurun_out/sq_<tag>"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from prof_summary import short  # noqa: E402  (multi-role launch names)

d = Path(sys.argv[1])
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for sub in ("a", "b"):
    p = d / sub / "run_counter_collection.csv"
    if not p.exists():
        continue
    for row in csv.DictReader(open(p)):
        if not re.search(r"k_\w+", row["Kernel_Name"]):
            continue
        k = short(row["Kernel_Name"])
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[k][row["Counter_Name"]] += 1
for k, c in acc.items():
    n = {x: c[x] / max(cnt[k][x], 1) for x in c}  # per dispatch
    waves = n.get("SQ_WAVES", 0)
    cyc = n.get("SQ_WAVE_CYCLES", 0)
    line = [k[:40].ljust(40)]
    if waves:
        line.append(f"valu/wave {n.get('SQ_INSTS_VALU', 0) / waves:8.0f}")
        line.append(f"lds/wave {n.get('SQ_INSTS_LDS', 0) / waves:6.0f}")
        line.append(f"salu/wave {n.get('SQ_INSTS_SALU', 0) / waves:6.0f}")
    if cyc:
        line.append(f"wait_any {n.get('SQ_WAIT_ANY', 0) / cyc:5.2f}")
        line.append(f"wait_inst {n.get('SQ_WAIT_INST_ANY', 0) / cyc:5.2f}")
        line.append(f"valu_active {n.get('SQ_ACTIVE_INST_VALU', 0) / cyc:5.2f}")
    if n.get("SQ_BUSY_CYCLES"):
        line.append(f"lds_bank_conf/active_lds {n.get('SQ_LDS_BANK_CONFLICT', 0) / max(n.get('SQ_ACTIVE_INST_LDS', 1), 1):5.2f}")
    print(" ".join(line))
