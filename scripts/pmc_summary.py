#!/usr/bin/env python3
"""Per-dispatch HBM traffic of one kernel from rocprofv3 --pmc CSVs
(scripts/pmc_pass.sh), corrected as MI355X_MICROARCH.md § HBM prescribes:
FETCH_SIZE (KB) reports half the bytes of 16-B-per-lane streaming reads on
gfx950 -> doubled; WRITE_SIZE (KB) is exact.  Writes a JSON summary that
bench.py reads for roofline.traffic.
Usage: pmc_summary.py FETCH_CSV WRITE_CSV KERNEL_SUBSTRING OUT_JSON [note]"""
import csv
import json
import sys


def per_dispatch(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no dispatch of {kernel!r} in {path}")
    return sum(vals) / len(vals), len(vals), min(vals), max(vals)


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    note = sys.argv[5] if len(sys.argv) > 5 else ""
    f_kb, nf, fmin, fmax = per_dispatch(fetch_csv, kernel)
    w_kb, nw, wmin, wmax = per_dispatch(write_csv, kernel)
    fetch_b = 2.0 * f_kb * 1024.0
    write_b = w_kb * 1024.0
    res = {
        "kernel": kernel,
        "dispatches": {"fetch": nf, "write": nw},
        "FETCH_SIZE_KB": {"mean": f_kb, "min": fmin, "max": fmax},
        "WRITE_SIZE_KB": {"mean": w_kb, "min": wmin, "max": wmax},
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "traffic_bytes": fetch_b + write_b,
        "correction": "FETCH_SIZE x 2 (gfx950 16-B streaming reads), WRITE_SIZE as is; KB = 1024 B",
        "note": note,
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
