#!/usr/bin/env python3
"""MFMA utilisation of the encoder kernels from scripts/pmc_mfma.sh output.
SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per v_mfma_f32_32x32x16_f16 (summed
over SIMDs); GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md).
util_profiled = busy / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) over the profiled
dispatch; util_live = busy / (live avg duration x 2.4 GHz x 1024), the live
duration being bench.py's hipEvent average from the bench JSON.
Usage: mfma_summary.py GPURUN_OUT_PREFIX BENCH_JSON OUT_JSON"""
import collections
import csv
import json
import sys

KERNELS = {1: ("k_gemm", "enc_mlp0"), 2: ("k_attn_enc4", "enc_attn"), 3: ("k_gemm", "cross_kv")}
CLOCK_HZ, SIMDS = 2.4e9, 1024


def main():
    prefix, bench_json, out = sys.argv[1:4]
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    res = {}
    for w, (kname, bkey) in KERNELS.items():
        d = collections.defaultdict(dict)
        for r in csv.DictReader(open(f"{prefix}_{w}/run_counter_collection.csv")):
            if kname in r["Kernel_Name"]:
                d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(d)[-20:]  # the probe's back-to-back launches come last
        busy = sum(d[i]["SQ_VALU_MFMA_BUSY_CYCLES"] for i in ids) / len(ids)
        grbm = sum(d[i]["GRBM_GUI_ACTIVE"] for i in ids) / len(ids)
        kb = bench["kernels"][bkey]
        alg_flops = kb["TFLOP/s"] * 1e12 * kb["avg_us"] * 1e-6
        res[bkey] = {
            "kernel": kb["kernel"],
            "dispatches": len(ids),
            "SQ_VALU_MFMA_BUSY_CYCLES": busy,
            "mfma_instructions": busy / 32.0,
            "algorithmic_mfma_instructions": alg_flops / 32768.0,
            "GRBM_GUI_ACTIVE_per_xcd": grbm / 8.0,
            "util_profiled": busy / (grbm / 8.0 * SIMDS),
            "live_avg_us": kb["avg_us"],
            "util_live": busy / (kb["avg_us"] * 1e-6 * CLOCK_HZ * SIMDS),
        }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
