#!/usr/bin/env python3
"""Per-kernel MFMA utilisation of the encoder (session step encpmc):
rocprofv3 --kernel-trace --stats gives each kernel's average duration,
a --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass its MFMA-busy cycles
(summed over the 1024 SIMDs; MI355X_MICROARCH.md).  Per kernel:
  util_live = busy / (avg duration x 2.4 GHz x 1024 SIMDs)
  util_active = busy / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
Usage: enc_mfma_summary.py TRACE_DIR PMC_DIR OUT_TXT"""
import collections
import csv
import sys

CLOCK_HZ, SIMDS, XCDS = 2.4e9, 1024, 8


def short(name):
    return name.split("(")[0].replace("void ", "")[:60]


def main():
    tdir, pdir, out = sys.argv[1:4]
    dur = {}
    for r in csv.DictReader(open(f"{tdir}/run_kernel_stats.csv")):
        dur[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]), float(r["Percentage"]))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{pdir}/run_counter_collection.csv")):
        per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = [f"{'kernel':60s} {'calls':>5s} {'avg us':>8s} {'%time':>6s} {'mfma busy/launch':>16s} "
             f"{'util_live':>9s} {'util_active':>11s}"]
    for k, (ns, calls, pct) in sorted(dur.items(), key=lambda kv: -kv[1][2]):
        c = per.get(k, {})
        busy = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])) / max(1, len(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])))
        grbm = sum(c.get("GRBM_GUI_ACTIVE", [0])) / max(1, len(c.get("GRBM_GUI_ACTIVE", [0])))
        ul = busy / (ns * 1e-9 * CLOCK_HZ * SIMDS) if ns else 0.0
        ua = busy / (grbm / XCDS * SIMDS) if grbm else 0.0
        lines.append(f"{k:60s} {calls:5d} {ns / 1e3:8.2f} {pct:6.2f} {busy:16.0f} {ul:9.3f} {ua:11.3f}")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
