"""Turn a gpu_profile.sh run (gpurun_out/prof_*) into the committed profiles/.

  python scripts/summarize_profiles.py --tag round1 [--batch 32] [--src gpurun_out]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_traffic.json       per-kernel HBM bytes per launch from the FETCH_SIZE /
                                    WRITE_SIZE passes, with the gfx950 correction
  profiles/field_traffic.json       what bench.py reports as roofline.traffic

Counter units and corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE reads exactly half the bytes of a wide coalesced
streaming read on gfx950, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
stores.  One rule for every kernel: traffic = 2 x FETCH_SIZE + WRITE_SIZE (the
counter tallies 64 B per 128-B memory-side request).  The raw FETCH_SIZE is kept
beside it; for the encode kernel's 8/16-B gathers the width is uncalibrated, so
its doubled figure is an upper bound and the raw one a lower bound.
"""
import argparse
import csv
import json
import shutil
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
# fp32 ngp / f16x3 ngp / f16x3 siren field kernels, the decoder's regular convs
FIELDS = ("ngp_field_kernel", "field_r_kernel<sdfr::NgpNet>", "field_p_kernel<sdfr::SirenNet>",
          "field_x_kernel<0, sdfr::NgpNet>", "field_x_kernel<0, sdfr::SirenNet>",
          "conv_h_kernel")                  # (and the decoder's largest kernel)
ENCODE = "ngp_encode_kernel"


def counters(path):
    per = defaultdict(list)
    for f in sorted(Path(path).glob("*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def pick(d, name):
    """Duration of kernel `name`: exact name, else the same name up to its argument
    list (the counter and trace CSVs may differ in the 'void ' prefix)."""
    if name in d:
        return d[name]
    def base(k):
        k = k[5:] if k.startswith("void ") else k
        return k[:k.rfind("(")] if k.endswith(")") else k
    hits = [k for k in d if base(k) == base(name)]
    return d[hits[0]] if hits else None


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tag", required=True)
    p.add_argument("--batch", type=int, default=32, help="faces per launch in the profiled bench")
    p.add_argument("--src", default=str(REPO / "gpurun_out"))
    a = p.parse_args()
    src, dst = Path(a.src), REPO / "profiles"
    dst.mkdir(exist_ok=True)

    stats = next((src / "prof_trace").glob("*kernel_stats.csv"), None)
    if stats is None:
        raise SystemExit(f"no kernel_stats.csv under {src / 'prof_trace'}")
    shutil.copy(stats, dst / f"{a.tag}_kernel_stats.csv")
    durations = {}
    with open(stats) as fh:
        for row in csv.DictReader(fh):
            durations[row["Name"]] = float(row["AverageNs"])

    fetch, nf = counters(src / "prof_fetch")
    write, nw = counters(src / "prof_write")
    out = {"batch_faces_per_launch": a.batch, "unit": "bytes per launch",
           "fetch_correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-stream undercount)",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        if "sdfr::" not in name:
            continue
        f = fetch.get(name)
        w = write.get(name)
        out["kernels"][name] = {
            "fetch_bytes_raw": None if f is None else f * 1024,
            "fetch_bytes_corrected": None if f is None else f * 1024 * 2,
            "write_bytes": None if w is None else w * 1024,
            "dispatches": {"fetch": nf.get(name), "write": nw.get(name)},
            "avg_duration_ns": pick(durations, name),
        }
    (dst / f"{a.tag}_traffic.json").write_text(json.dumps(out, indent=1))

    tj = dst / "field_traffic.json"
    prev = json.loads(tj.read_text()) if tj.exists() else {}
    per = prev.get("kernels", {}) if isinstance(prev.get("kernels"), dict) else {}
    for fname in FIELDS:
        fk = next((v for k, v in out["kernels"].items() if f"::{fname}" in k), None)
        if fk and fk["fetch_bytes_corrected"] is not None and fk["write_bytes"] is not None:
            total = fk["fetch_bytes_corrected"] + fk["write_bytes"]
            per[fname] = {"source": f"profiles/{a.tag}_traffic.json",
                          "bytes_per_launch_per_face": total / a.batch,
                          "fetch_bytes_per_face": fk["fetch_bytes_corrected"] / a.batch,
                          "write_bytes_per_face": fk["write_bytes"] / a.batch}
    ek = next((v for k, v in out["kernels"].items() if f"::{ENCODE}" in k), None)
    if ek and ek["fetch_bytes_raw"] is not None and ek["write_bytes"] is not None:
        # same rule as every kernel; for these gathers the width is uncalibrated, so
        # the raw figure (a lower bound) is kept beside it
        per[ENCODE] = {"source": f"profiles/{a.tag}_traffic.json",
                       "bytes_per_launch_per_face":
                           (ek["fetch_bytes_corrected"] + ek["write_bytes"]) / a.batch,
                       "bytes_per_launch_per_face_fetch_raw":
                           (ek["fetch_bytes_raw"] + ek["write_bytes"]) / a.batch,
                       "fetch_bytes_per_face": ek["fetch_bytes_corrected"] / a.batch,
                       "write_bytes_per_face": ek["write_bytes"] / a.batch}
    tj.write_text(json.dumps({"unit": "HBM bytes per face per launch (2 x FETCH_SIZE + WRITE_SIZE, "
                                      "every kernel)",
                              "kernels": per}, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
