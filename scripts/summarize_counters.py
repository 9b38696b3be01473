"""Summarise the rocprofv3 --pmc passes of scripts/gpu.sh (task `counters`) into one JSON
(profiles/<tag>_counters.json): per kernel the mean counter value per dispatch and
derived ratios.

Units (MI355X_MICROARCH.md, "Per-instruction cycle constants" / "DVFS"):
SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles (summed over waves);
SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles (summed over SIMDs); GRBM_GUI_ACTIVE is
summed over the 8 XCDs, so the effective clock = GRBM_GUI_ACTIVE / 8 / duration.

    python scripts/summarize_counters.py --tag round2 [--src gpurun_out]
"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
N_SIMD = 256 * 4


def load(d):
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(Path(d).glob("*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                if row["Counter_Name"] == next(iter(per[k])):
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return per, dur


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tag", required=True)
    p.add_argument("--src", default=str(REPO / "gpurun_out"))
    p.add_argument("--mfma-per-launch", type=json.loads, default={},
                   help='{"kernel substring": algorithmic MFMA count per launch}')
    a = p.parse_args()
    kernels = defaultdict(dict)
    for d in sorted(Path(a.src).glob("pmc_*")):
        if not d.is_dir():
            continue
        per, dur = load(d)
        for k, cs in per.items():
            e = kernels[k]
            for c, v in cs.items():
                e.setdefault("counters", {})[c] = sum(v) / len(v)
            e.setdefault("duration_s_by_pass", {})[d.name] = sum(dur[k]) / max(1, len(dur[k]))
            e["dispatches"] = len(next(iter(cs.values())))
    out = {"unit": "mean per dispatch; SQ_WAVE/WAIT/ACTIVE in quad-cycles summed over waves, "
                   "SQ_VALU_MFMA_BUSY_CYCLES in SIMD cycles summed over SIMDs, GRBM_GUI_ACTIVE "
                   "summed over 8 XCDs",
           "kernels": {}}
    for k, e in kernels.items():
        c = e.get("counters", {})
        d = {"counters": c, "duration_s_by_pass": e["duration_s_by_pass"]}
        grbm = c.get("GRBM_GUI_ACTIVE")
        t2 = next((v for n, v in e["duration_s_by_pass"].items() if n.endswith("2")), None)
        if grbm and t2:
            clk = grbm / 8 / t2
            d["effective_clock_GHz"] = clk / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                d["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (grbm / 8 * N_SIMD)
        if "SQ_INSTS_MFMA" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            d["mfma_busy_cycles_per_mfma"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_INSTS_MFMA"]
        if "SQ_INSTS_MFMA" in c and "SQ_INSTS_VALU" in c:
            d["valu_per_mfma"] = c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_MFMA", "SQ_WAIT_INST_LDS"):
                if n in c:
                    d[f"{n}_frac_of_wave_cycles"] = c[n] / wc
        out["kernels"][k] = d
    dst = REPO / "profiles" / f"{a.tag}_counters.json"
    dst.write_text(json.dumps(out, indent=1, sort_keys=True))
    print(json.dumps({k: {n: v for n, v in d.items() if n != "counters"}
                      for k, d in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
