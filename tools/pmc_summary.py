"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) per mq_* kernel.

Reads <dir>/p*/run_counter_collection.csv, averages every counter per dispatch for each of the
library's kernels and prints derived figures:
  VALU/wave        SQ_INSTS_VALU / SQ_WAVES
  VALU busy        SQ_ACTIVE_INST_VALU / (SQ_BUSY_CYCLES * 4 SIMDs) is not exposed per SIMD, so
                   the ratio of SQ_ACTIVE_INST_VALU to SQ_WAVE_CYCLES (wave-level) is reported
  HBM bytes        FETCH_SIZE * 2 (gfx950: FETCH_SIZE counts half of wide streaming reads) +
                   WRITE_SIZE, both in KiB units from rocprofv3
With --json PATH also writes {"kernel": {"hbm_bytes_per_launch": ..., ...}} for bench.py.
Usage: python tools/pmc_summary.py gpurun_out/pmc_b [--json profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    files = sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv")))
    files += sorted(glob.glob(os.path.join(d, "run_counter_collection.csv")))
    for f in files:
        with open(f) as fh:
            per = defaultdict(float)  # (dispatch, kernel, counter) -> sum
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0]
                k = k[5:] if k.startswith("void ") else k  # templated kernels: "void mq_...<..>(...)"
                if not k.startswith("mq_"):
                    continue
                per[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, k, c), v in per.items():
                acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    d = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    # --tiles T: per-tile counts for the tile kernels (the AES kernels are persistent: one wave
    # walks many tiles, so per-wave counts are not per-tile there)
    tiles = int(sys.argv[sys.argv.index("--tiles") + 1]) if "--tiles" in sys.argv else None
    res = load(d)
    summary = {}
    for k in sorted(res):
        c = res[k]
        print(f"== {k}")
        for name in sorted(c):
            print(f"   {name:28s} {c[name]:16.1f}")
        w = c.get("SQ_WAVES")
        s = {}
        if w and "SQ_INSTS_VALU" in c:
            s["valu_per_wave"] = c["SQ_INSTS_VALU"] / w
            print(f"   -> VALU instr / wave       {s['valu_per_wave']:.0f}")
        if w and "SQ_INSTS_LDS" in c:
            print(f"   -> LDS instr / wave        {c['SQ_INSTS_LDS'] / w:.0f}")
        if tiles and "hp_kernel" not in k and "partition" not in k:
            for x in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if x in c:
                    s[x.lower() + "_per_tile"] = c[x] / tiles
                    print(f"   -> {x} / tile {c[x] / tiles:10.0f}")
        if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
            s["valu_active_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
            print(f"   -> VALU active / wave cyc  {s['valu_active_frac_of_wave_cycles']:.3f}")
        if "SQ_WAVE_CYCLES" in c:
            for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if x in c:
                    print(f"   -> {x:24s} {c[x] / c['SQ_WAVE_CYCLES']:.3f} of wave cycles")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c:
            print(f"   -> LDS bank conflict / LDS active {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_ACTIVE_INST_LDS']):.3f}")
        if "FETCH_SIZE" in c:
            s["fetch_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            s["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "fetch_bytes" in s and "write_bytes" in s:
            s["hbm_bytes_per_launch"] = s["fetch_bytes"] + s["write_bytes"]
            print(f"   -> HBM bytes / launch      {s['hbm_bytes_per_launch'] / 1e9:.4f} GB "
                  f"(read x2 {s['fetch_bytes'] / 1e9:.4f} + write {s['write_bytes'] / 1e9:.4f})")
        summary[k] = s
    if out_json:
        with open(out_json, "w") as fh:
            json.dump({"source": d, "note": "per-launch means over the profiled dispatches; "
                       "fetch = FETCH_SIZE x 2 (gfx950 correction), write = WRITE_SIZE",
                       "kernels": summary}, fh, indent=1)


if __name__ == "__main__":
    main()
