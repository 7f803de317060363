"""Dev tool: per-launch HBM traffic of one kernel from rocprofv3 --pmc passes (one directory per
pass, as tools/gpu_bins.sh writes them) -> profiles/pmc_<name>.json, read by bench.py for
roofline.traffic.

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE counts half of the bytes of a wide coalesced stream, and other access
widths are uncalibrated. `hbm_bytes_per_launch` uses the gfx950 correction (2 x FETCH_SIZE) -- the
upper of the two readings; the raw reading is kept beside it.

    python tools/pmc_traffic.py gpurun_out/pmc22 'task_kernel<cbh::PlusTimesD<double>, 4096' profiles/pmc_num_large.json
"""
import collections
import csv
import glob
import json
import sys


def main(src, pattern, dst, note=""):
    vals = collections.defaultdict(list)
    name = None
    for f in sorted(glob.glob(src + "/pmc*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if pattern not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not name:
        sys.exit(f"no dispatch of {pattern!r} under {src}")
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    launches = len(vals.get("FETCH_SIZE", []))
    fetch = avg["FETCH_SIZE"] * 1024
    write = avg["WRITE_SIZE"] * 1024
    out = {
        "kernel": name.split("(")[0].replace("void ", ""),
        "launches_profiled": launches,
        "fetch_bytes_per_launch_raw": round(fetch),
        "write_bytes_per_launch": round(write),
        "hbm_bytes_per_launch_raw": round(fetch + write),
        "hbm_bytes_per_launch": round(2 * fetch + write),
        "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM); raw = FETCH_SIZE+WRITE_SIZE in KiB x 1024",
        "l2_hit_rate": round(avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]), 4)
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg else None,
        "lds_bank_conflict_frac": round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 4)
        if "SQ_LDS_IDX_ACTIVE" in avg else None,
        "wait_frac": round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 4) if "SQ_WAVE_CYCLES" in avg else None,
        "counters_avg_per_launch": {k: v for k, v in sorted(avg.items())},
        "source": src,
        "note": note,
    }
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out[k] for k in out if k != "counters_avg_per_launch"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
