#!/usr/bin/env python3
"""Issued VALU op rate per kernel from a tools/pmc_sq.sh pass, against the gfx950 peak.

    tools/valu_rate.py gpurun_out/sq_<tag>[,sq_<tag2>] <bench line .json>[,<bench2>] <out.json> [<alg|mode|chunk> key]

Several SQ passes (e.g. the default schedule, whose multi-role launches run several kernels in
one dispatch, and the serial --streams 1 schedule, one kernel per dispatch) are merged, each with
the durations of its own bench line: "kernels" (the serial profiled step) or, for the multi-role
launches, "kernels_timed_region".

With a key, the per-kernel issued rates are also recorded in profiles/valu_rate.json, which
bench.py reads to add roofline.issued for the same configuration.

SQ_INSTS_VALU (wave instructions per dispatch, pass "a") x 64 lanes = issued 32-bit lane-ops;
divided by the kernel's isolated average duration from the bench line's "kernels" object (the
serial profiled step: rocprofv3 serialises dispatches while it collects counters, so the
isolated duration is the matching one).  Reported against the nominal 78.6 T lane-ops/s
(256 CU x 4 SIMD x 32 lanes x 2.4 GHz, bench.py VALU_PEAK) and the measured full-rate issue
ceiling (v_xor / v_add / v_bitop3 microbenchmark, profiles/r1/valu_peak_r1b.json).  Half-rate
instructions (v_alignbit, v_perm, VOP3 and/or/lshl_or, 24-bit multiplies) count once here but
occupy two issue slots, so issued/peak understates how busy the VALU is; the bench line's
algorithmic rate ("achieved_Tops") divided by the issued rate gives the fraction of issued
instructions that the algorithmic count covers.
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from prof_summary import short  # noqa: E402  (multi-role launch names)

PEAK = 78.6432  # T lane-ops/s
FULL_RATE = 61.26  # v_xor_b32 measured, T lane-ops/s


def bench_name(pmc_name: str) -> str:
    return pmc_name.split("<")[0]  # short() already maps the multi-role launches to launch names


def main() -> None:
    dirs = [Path(x) for x in sys.argv[1].split(",")]
    benches = [Path(x) for x in sys.argv[2].split(",")]
    out = Path(sys.argv[3])
    res = {}
    for d, bench_path in zip(dirs, benches):
        res.update(one_pass(d, bench_path))
    summary = {"source": ",".join(map(str, dirs)), "bench": ",".join(map(str, benches)), "peak_Tops": PEAK,
               "full_rate_ceiling_Tops": FULL_RATE, "kernels": res}
    finish(summary, res, out)


def one_pass(d: Path, bench_path: Path) -> dict:
    bench = json.loads(bench_path.read_text().strip().splitlines()[-1])
    kernels = dict(bench.get("kernels_timed_region") or {})
    kernels.update(bench.get("kernels") or {})
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
    res = {}
    for k, c in acc.items():
        n = {x: c[x] / max(cnt[k][x], 1) for x in c}
        b = kernels.get(bench_name(k))
        if not b or "SQ_INSTS_VALU" not in n:
            continue
        t = b["avg_ms"] * 1e-3
        issued = n["SQ_INSTS_VALU"] * 64 / t / 1e12
        r = {"valu_wave_instrs_per_dispatch": n["SQ_INSTS_VALU"], "lds_instrs_per_dispatch": n.get("SQ_INSTS_LDS"),
             "avg_ms_isolated": b["avg_ms"], "issued_Tops": issued, "issued_frac_of_peak": issued / PEAK,
             "issued_frac_of_full_rate_ceiling": issued / FULL_RATE}
        if n.get("SQ_WAVE_CYCLES"):
            r["wave_cycles_valu_active"] = n.get("SQ_ACTIVE_INST_VALU", 0) / n["SQ_WAVE_CYCLES"]
            r["wave_cycles_waiting"] = n.get("SQ_WAIT_ANY", 0) / n["SQ_WAVE_CYCLES"]
        if b.get("achieved_Tops"):
            r["algorithmic_Tops"] = b["achieved_Tops"]
            r["algorithmic_over_issued"] = b["achieved_Tops"] / issued
        res[k] = r
    return res


def finish(summary: dict, res: dict, out: Path) -> None:
    out.write_text(json.dumps(summary, indent=1) + "\n")
    if len(sys.argv) > 4:
        idx = Path(__file__).resolve().parent.parent / "profiles" / "valu_rate.json"
        all_ = json.loads(idx.read_text()) if idx.exists() else {}
        all_[sys.argv[4]] = {"issued_Tops": {k: r["issued_Tops"] for k, r in res.items()},
                             "source": str(out)}
        idx.write_text(json.dumps(all_, indent=1, sort_keys=True) + "\n")
    for k, r in sorted(res.items(), key=lambda kv: -kv[1]["avg_ms_isolated"]):
        print(f"{k[:34]:34s} {r['avg_ms_isolated']:7.3f} ms  issued {r['issued_Tops']:5.1f} Tops "
              f"= {r['issued_frac_of_peak']:.2f} of peak, {r['issued_frac_of_full_rate_ceiling']:.2f} of full-rate"
              + (f"  alg/issued {r['algorithmic_over_issued']:.2f}" if "algorithmic_over_issued" in r else ""))


if __name__ == "__main__":
    main()
